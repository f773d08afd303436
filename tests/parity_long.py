"""C2 (MF-BPR, ML-20M shape, d = 64, B = 8192, n = 5, Adam) run longer than the test suite does:
S native steps (default 60) against the oracle in fp32, fp64 and fp32 summing in another order
(oracle/mf.py; tests/test_configs_gpu.py's setup).  Every step: the loss within 1e-5 relative and
the MT state bit-exact (exit status 1 otherwise); at the checked steps every element of the four
tables through tests/parity_report.check (the band, the counts outside 1e-5, the reference's own
count in another fp32 order), appended to gpurun_out/parity_elementwise.jsonl.

    python tests/parity_long.py [--steps 60] [--loss bpr] [--dim 64]

(Test infrastructure: it lives under tests/ because it runs the oracle; pytest does not collect it.)
"""
import argparse
import json
import os
import sys
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import mf as omf  # noqa: E402
from oracle import rng as orng  # noqa: E402
from tests import parity_report  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--loss", default="bpr")
    ap.add_argument("--dim", type=int, default=64)
    args = ap.parse_args()
    from recommendation_gans_amd.mf_engine import MFEngine
    from recommendation_gans_amd.synthetic import ML20M, movielens_like
    warnings.simplefilter("ignore")
    data = movielens_like(ML20M, seed=0)
    dev = torch.device("cuda:0")
    U, I, B, n, d, steps = data.num_users, data.num_items, 8192, 5, args.dim, args.steps
    torch.manual_seed(0)
    tabs = omf.init_tables(U, I, d)
    st = orng.py_seed_state(0)
    kw = dict(loss=args.loss, optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
    o = omf.MFOracle(*[t.clone() for t in tabs], data.pool_u, data.pool_i, st.copy(), **kw)
    o64 = omf.MFOracle(*[t.clone().double() for t in tabs], data.pool_u, data.pool_i, st.copy(), noise=True, **kw)
    oalt = omf.MFOracle(*[t.clone() for t in tabs], data.pool_u, data.pool_i, st.copy(), order_seed=1, **kw)
    e = MFEngine(tabs[0], tabs[1], tabs[2].reshape(-1), tabs[3].reshape(-1), data.pool_u, data.pool_i, st.copy(),
                 device=dev, **kw)
    tu = torch.from_numpy(data.train_u[:(steps + 1) * B].astype(np.int64)).to(dev)
    ti = torch.from_numpy(data.train_i[:(steps + 1) * B].astype(np.int64)).to(dev)
    ins = [e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], B, e.make_plan(ti[s * B:(s + 1) * B]))
           for s in range(steps + 1)]
    checked = {0, 9, 19, 29, 39, 49, steps - 1}
    worst_loss, bad = 0.0, 0
    for s in range(steps):
        got = float(e.train_step_in(ins[s], ins[s + 1])[0])
        pu, pi = data.train_u[s * B:(s + 1) * B], data.train_i[s * B:(s + 1) * B]
        lref = o.step(pu, pi)
        o64.step(pu, pi)
        oalt.step(pu, pi)
        torch.cuda.synchronize()
        rel = abs(got - lref) / abs(lref)
        worst_loss = max(worst_loss, rel)
        mt_ok = bool((e.mt_state() == o.state).all())
        if rel > 1e-5 or not mt_ok:
            bad += 1
        line = {"step": s, "loss_gpu": got, "loss_ref32": lref, "loss_rel": rel, "mt_exact": mt_ok}
        if s in checked:
            line["tables"] = []
            for k in range(4):
                ok, msg = parity_report.check(f"C2 d{d} {args.loss} long step {s} table {k}", e.params()[k],
                                              o.params[k], o64.params[k], noise=o64.noise[k],
                                              order32=oalt.params[k])
                line["tables"].append({"table": k, "ok": ok, "msg": msg})
        print(json.dumps(line), flush=True)
    print(json.dumps({"steps": steps, "worst_loss_rel": worst_loss, "steps_failing_loss_or_mt": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
