"""Per-kernel timing of the MF step on one GPU.

    python scripts/mf_kernel_bench.py [--zipf 1.0 0.5 0.0] [--dim 64] [--batch 8192]

Times rg_mt_generate alone, then the whole step (native stepper, words generated
ahead) and rg_mf_apply (HIP events around its launch) for each item-popularity skew
on ML-20M-shaped synthetic data.  Kernel-level durations: use rocprofv3.
"""
import argparse
import json
import os
import random
import sys
import time

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
    ap.add_argument("--zipf", type=float, nargs="+", default=[1.0, 0.0])
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--plan", type=int, default=1)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    d, B, n = args.dim, args.batch, 5
    res = {}
    st = torch.from_numpy(np.asarray(random.getstate()[1], dtype=np.uint32).view(np.int32).copy()).to(dev)
    out = torch.empty(2 * n * B + _lib.RG_MT_PAD, dtype=torch.int32, device=dev)
    ts = []
    for _ in range(args.iters):
        a, b = ev(), ev()
        a.record()
        _lib.check(lib.rg_mt_generate(_lib.stream_handle(), _lib.ptr(st), _lib.ptr(out), 2 * n * B, None), "gen")
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    res["mt_generate_us"] = float(np.median([a.elapsed_time(b) for a, b in ts[3:]]) * 1e3)
    for z in args.zipf:
        data = movielens_like(ML20M, seed=0, zipf_s=z)
        U, I = data.num_users, data.num_items
        torch.manual_seed(0)
        Uw, Iw = torch.empty(U, d).normal_(0, 1.0 / d), torch.empty(I, d).normal_(0, 1.0 / d)
        random.seed(0)
        e = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), data.pool_u, data.pool_i,
                     np.asarray(random.getstate()[1], dtype=np.uint32), loss="bpr", optimizer="adam", lr=1e-3,
                     weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
        tu = torch.from_numpy(data.train_u).to(dev)
        ti = torch.from_numpy(data.train_i).to(dev)
        ins = []
        for s in range(args.iters + 1):
            u, i = tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B]
            ins.append(e.step_input(u, i, B, e.make_plan(i) if args.plan else None))
        evs = [(ev(), ev()) for _ in range(args.iters)]
        for x, y in evs:
            x.record()
            y.record()
        for s in range(5):
            e.train_step_in(ins[s], ins[s + 1])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(5, args.iters):
            e.train_step_in(ins[s], ins[s + 1], apply_events=evs[s])
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / (args.iters - 5)
        cnt = np.bincount(data.train_i[:B], minlength=I)
        res[f"zipf{z}"] = {"step_us": el * 1e6,
                           "apply_us": float(np.median([_lib.elapsed_ms(x, y) for x, y in evs[5:]]) * 1e3),
                           "max_item_hits_in_batch": int(cnt.max()), "items_over_cap": int((cnt > 8).sum())}
        del e
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
