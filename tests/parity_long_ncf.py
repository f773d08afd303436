"""C3 (ncf_spotlight.py at ML-20M shape: mlp_embedding_dim 64, tower [128, 64, 32, 16, 8],
B = 8192, n = 5, pointwise, Adam lr 1e-3, wd 1e-5) run longer than the test suite does
(tests/test_configs_gpu.py::test_ncf_full_size_steps runs 10): S native steps (default 20) with
item plans and recorded dropout masks against oracle/ncf.py in fp32, fp64 and two more fp32
restatements summing in other orders, and one deciding every LeakyReLU within fp32 rounding of
its kink the other way (oracle/ncf.py kink_flip).  Every step: the loss within 1e-5 relative and the MT
state bit-exact (exit status 1 otherwise); at the checked steps every parameter through
tests/parity_report.check, one JSON line per step.

    python tests/parity_long_ncf.py [--steps 20] [--neumf]

--neumf: neuMF_spotlight.py's defaults instead (mlp_embedding_dim 16, mf_embedding_dim 50; the
GMF tables included), as tests/test_configs_gpu.py::test_neumf_full_size_steps for 10 steps.

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

from oracle import ncf as oncf  # noqa: E402
from oracle import rng as orng  # noqa: E402
from tests import parity_report  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--neumf", action="store_true")
    ap.add_argument("--dump", type=int, default=0,
                    help="at the last step print the N elements farthest outside the fp32 orders' spread")
    ap.add_argument("--track", default="", metavar="PARAM:ROW,...",
                    help="print every step's max |GPU - fp32 reference| over these parameter rows")
    args = ap.parse_args()
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from recommendation_gans_amd.ncf_spotlight import mlp_layers
    from recommendation_gans_amd.spotlight.dnn_models.mlp import MLP
    from recommendation_gans_amd.spotlight.dnn_models.neuMF import NeuMF
    from recommendation_gans_amd.synthetic import ML20M, movielens_like
    warnings.simplefilter("ignore")
    data = movielens_like(ML20M, seed=0)
    dev = torch.device("cuda:0")
    E = 16 if args.neumf else 64
    U, I, B, n, steps = data.num_users, data.num_items, 8192, 5, args.steps
    torch.manual_seed(0)                                   # ncf_spotlight.py / neuMF_spotlight.py init
    net = (NeuMF(mlp_layers(E), U, I, mf_embedding_dim=50, mlp_embedding_dim=E) if args.neumf
           else MLP(layers=mlp_layers(E), num_users=U, num_items=I, embedding_dim=E))
    names = [k for k, _ in net.named_parameters()]
    params = [p.detach().clone() for p in net.parameters()]
    mt = orng.py_seed_state(0)
    kw = dict(loss="pointwise", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
    if args.neumf:
        e = NCFEngine(params[0], params[1], params[4:], data.pool_u, data.pool_i, mt.copy(), optimizer="adam",
                      device=dev, mf_user_w=params[2], mf_item_w=params[3], **kw)
    else:
        e = NCFEngine(params[0], params[1], params[2:], data.pool_u, data.pool_i, mt.copy(), optimizer="adam",
                      device=dev, **kw)
    Oracle = oncf.NeuMFOracle if args.neumf else oncf.NCFOracle
    o32 = Oracle([t.clone() for t in params], names, data.pool_u, data.pool_i, mt.copy(), **kw)
    o64 = Oracle([t.double() for t in params], names, data.pool_u, data.pool_i, mt.copy(), **kw)
    o32b = ([Oracle([t.clone() for t in params], names, data.pool_u, data.pool_i, mt.copy(), order_seed=k, **kw)
             for k in (1, 2)] +
            [Oracle([t.clone() for t in params], names, data.pool_u, data.pool_i, mt.copy(), kink_flip=4.0, **kw)])
    widths = oncf.layer_sizes(E)[1:]                        # one dropout per hidden Linear
    rs = np.random.RandomState(6 if args.neumf else 5)
    tag = "NeuMF" if args.neumf else "C3 ncf"
    checked = {0, 9, steps - 1}
    worst, bad, tbad = 0.0, 0, 0
    for s in range(steps):
        pu = data.train_u[s * B:(s + 1) * B].astype(np.int64)
        pi = data.train_i[s * B:(s + 1) * B].astype(np.int64)
        mp = [torch.from_numpy((rs.rand(B, w) >= 0.5).astype(np.uint8)) for w in widths]
        mn = [torch.from_numpy((rs.rand(n * B, w) >= 0.5).astype(np.uint8)) for w in widths]
        masks = (torch.cat(mp, 1).to(dev).contiguous(), torch.cat(mn, 1).to(dev).contiguous())
        prev = [t.detach().cpu().clone() for t in e.params()]
        pi_d = torch.from_numpy(pi).to(dev)
        got = float(e.train_step(torch.from_numpy(pu).to(dev), pi_d, plan=e.make_plan(pi_d), masks=masks)[0])
        l32 = o32.step(pu, pi, mp, mn)
        o64.step(pu, pi, mp, mn)
        for ob in o32b:
            ob.step(pu, pi, mp, mn)
        torch.cuda.synchronize()
        rel = abs(got - l32) / abs(l32)
        worst = max(worst, rel)
        mt_ok = bool((e.mt_state() == o32.state).all())
        bad += int(rel > 1e-5 or not mt_ok)
        line = {"step": s, "loss_gpu": got, "loss_ref32": l32, "loss_rel": rel, "mt_exact": mt_ok,
                "kink_flips": o32b[-1].flips[-1]}
        for tr in filter(None, args.track.split(",")):
            pname, prow = tr.rsplit(":", 1)
            k = names.index(pname)
            gp = e.params()[k].detach().cpu().reshape(o32.P.t[k].shape)
            line[f"track {tr}"] = float((gp[int(prow)].double() - o32.P.t[k][int(prow)].double()).abs().max())
        if s in checked:
            line["tables"] = []
            for k, (nm, p, r32, r64) in enumerate(zip(names, e.params(), o32.P.t, o64.P.t)):
                ok, msg = parity_report.check(f"{tag} long step {s} {nm}", p.reshape(r32.shape), r32, r64,
                                              before=prev[k].reshape(r32.shape), alt32=[ob.P.t[k] for ob in o32b])
                line["tables"].append({"param": nm, "ok": ok, "msg": msg})
                tbad += int(not ok)
        print(json.dumps(line), flush=True)
        if args.dump and s == steps - 1:
            seen = np.concatenate([data.train_u[:steps * B]]).astype(np.int64)
            cnt = np.bincount(seen, minlength=U)
            last = np.bincount(pu, minlength=U)
            for k, (nm, p, r32, r64) in enumerate(zip(names, e.params(), o32.P.t, o64.P.t)):
                g = p.detach().cpu().double().reshape(-1)
                r64d, r32d = r64.double().reshape(-1), r32.double().reshape(-1)
                spread = (r32d - r64d).abs()
                for ob in o32b:
                    spread = torch.maximum(spread, (ob.P.t[k].double().reshape(-1) - r64d).abs())
                score = (g - r64d).abs() / (spread + 1e-7 * r64d.abs() + 1e-30)
                top = torch.topk(score, min(args.dump, score.numel())).indices.tolist()
                shape = tuple(r32.shape)
                for ix in top[:args.dump]:
                    row, col = (ix // shape[1], ix % shape[1]) if len(shape) == 2 else (ix, 0)
                    rec = {"param": nm, "row": row, "col": col, "score": float(score[ix]), "gpu": float(g[ix]),
                           "ref32": float(r32d[ix]), "ref64": float(r64d[ix]),
                           "alt32": [float(ob.P.t[k].double().reshape(-1)[ix]) for ob in o32b]}
                    if "user" in nm and len(shape) == 2:
                        rec["user_positives_so_far"] = int(cnt[row])
                        rec["user_positives_last_step"] = int(last[row])
                    print(json.dumps({"dump": rec}), flush=True)
    print(json.dumps({"steps": steps, "worst_loss_rel": worst, "steps_failing_loss_or_mt": bad,
                      "table_checks_failing": tbad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
