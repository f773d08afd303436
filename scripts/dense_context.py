"""The MF dense pass in the bench's own process and buffers: is the step's dense pass slower
than the same kernel launched back to back on the same tables?

    python scripts/dense_context.py [--iters 30]

ML-20M-shaped (d = 64, B = 8192, BPR, Adam) like bench.py: 10 steps, then
  in_step   the dense pass inside 30 training steps (HIP events around its launch)
  alone     rg_mf_apply over every row, 30 launches back to back on the same tables (every
            contribution count is zero after a step: a pure stream of p, m, v, biases, counts)
  alone_gap the same with a 2 ms spin between launches (nothing of the previous pass in flight)
  alone_flip  back to back, each launch reading the table set the previous one wrote
  split_apply  rg_mf_pairs then rg_mf_apply by hand (the step's pulls, no prepare / MT in the launch)
  alone_mt  alone, with one step's MT walk (rg_mt_generate, one workgroup) launched beside each pass
Diagnostic only: the 'alone' launches do not flip the table sets (not a training state).
"""
import argparse
import json
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from recommendation_gans_amd import _lib  # noqa: E402
from recommendation_gans_amd.mf_engine import MFEngine  # noqa: E402
from recommendation_gans_amd.synthetic import ML20M, movielens_like  # noqa: E402


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--dim", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    d, B, n = args.dim, 8192, 5
    data = movielens_like(ML20M, seed=0)
    U, I = data.num_users, data.num_items
    torch.manual_seed(0)
    Uw, Iw = torch.empty(U, d).normal_(0, 1.0 / d), torch.empty(I, d).normal_(0, 1.0 / d)
    random.seed(0)
    e = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), data.pool_u, data.pool_i,
                 np.asarray(random.getstate()[1], dtype=np.uint32), loss="bpr", optimizer="adam", lr=1e-3,
                 weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
    tu = torch.from_numpy(data.train_u.astype(np.int64)).to(dev)
    ti = torch.from_numpy(data.train_i.astype(np.int64)).to(dev)
    steps = 10 + args.iters
    ins = [e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], B, e.make_plan(ti[s * B:(s + 1) * B]))
           for s in range(steps + 2)]
    for s in range(10):
        e.train_step_in(ins[s], ins[s + 1], next2=ins[s + 2])
    torch.cuda.synchronize()
    res = {}
    evs = [(ev(), ev()) for _ in range(args.iters)]
    for x, y in evs:        # torch creates the HIP event lazily on its first record
        x.record()
        y.record()
    for s in range(10, steps):
        e.train_step_in(ins[s], ins[s + 1], apply_events=evs[s - 10], next2=ins[s + 2])
    torch.cuda.synchronize()
    res["in_step_us"] = float(np.median([_lib.elapsed_ms(x, y) for x, y in evs]) * 1e3)
    e._work_step = e._work
    e._global_pos = B
    side = torch.cuda.Stream()
    st = torch.from_numpy(np.asarray(random.getstate()[1], dtype=np.uint32).view(np.int32).copy()).to(dev)
    words = torch.empty(2 * n * B + _lib.RG_MT_PAD, dtype=torch.int32, device=dev)
    for mode in ("alone", "alone_gap", "alone_flip", "alone_mt"):
        ts = []
        for _ in range(args.iters):
            if mode == "alone_gap":
                torch.cuda._sleep(4_000_000)
            if mode == "alone_mt":      # one step's MT walk (one workgroup) beside the pass, as in a step
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    _lib.check(e.lib.rg_mt_generate(_lib.stream_handle(), _lib.ptr(st), _lib.ptr(words), 2 * n * B,
                                                    None), "rg_mt_generate")
            a, b = ev(), ev()
            a.record()
            e.apply_rows(0, U + I, loss=False)
            b.record()
            if mode == "alone_flip":     # the next launch reads the set this one wrote
                e.finish_step()
            ts.append((a, b))
        torch.cuda.synchronize()
        res[mode + "_us"] = float(np.median([a.elapsed_time(b) for a, b in ts[3:]]) * 1e3)
    # the split step by hand: rg_mf_pairs (lists of this step), then rg_mf_apply over every row
    # (mf_apply_kernel: the pulls, no next-step prepare, no MT walk in the launch)
    ts = []
    for s in range(args.iters):
        g = 10 + s
        e.pairs_and_lists(tu[g * B:(g + 1) * B], ti[g * B:(g + 1) * B], B, e.make_plan(ti[g * B:(g + 1) * B]))
        a, b = ev(), ev()
        a.record()
        e.apply_rows(0, U + I, loss=True)
        b.record()
        e.finish_step()
        ts.append((a, b))
    torch.cuda.synchronize()
    res["split_apply_us"] = float(np.median([a.elapsed_time(b) for a, b in ts[3:]]) * 1e3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
