"""Where the MF pair pass spends its time: per-wave phase stamps from the diagnostic
library (python -m recommendation_gans_amd.build --diag -> librg_hip_diag.so, built
with RG_DIAG_STAMPS; the product library has no stamp code).

    python scripts/mf_pairs_stamps.py [--steps 20]

Runs the bench configuration (ML-20M-shaped, d=64, B=8192, bpr, Adam) through the
native stepper and reads, for the last steps' pair kernels, each wave's
s_memrealtime (100 MHz) at: entry, ids landed, rows gathered + dots, dz in LDS,
list entries issued, exit.  Every stamp drains vmcnt first, so the build runs
slower than the product: read the phase SHARES, not the total.
"""
import argparse
import ctypes
import json
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from recommendation_gans_amd import _lib, build  # noqa: E402

PHASES = ["ids", "gather+dot", "loss+dz+lds", "lists", "partials+exit"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--gap", action="store_true", help="synchronize + idle 20 ms between steps")
    ap.add_argument("--flags", type=int, default=0, help="diag flags (bit 0: skip list-slot atomics)")
    args = ap.parse_args()
    lib = _lib.load(build.DIAG_LIB)
    lib.rg_diag_set_stamps.argtypes = [ctypes.c_void_p]
    lib.rg_diag_set_flags.argtypes = [ctypes.c_int]
    from recommendation_gans_amd.mf_engine import MFEngine
    from recommendation_gans_amd.synthetic import ML20M, movielens_like
    dev = torch.device("cuda:0")
    d, B, n = 64, 8192, 5
    data = movielens_like(ML20M, seed=0, zipf_s=1.0)
    U, I = data.num_users, data.num_items
    torch.manual_seed(0)
    Uw, Iw = torch.empty(U, d).normal_(0, 1.0 / d), torch.empty(I, d).normal_(0, 1.0 / d)
    random.seed(0)
    e = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), data.pool_u, data.pool_i,
                 np.asarray(random.getstate()[1], dtype=np.uint32), loss="bpr", optimizer="adam", lr=1e-3,
                 weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
    tu = torch.from_numpy(data.train_u).to(dev)
    ti = torch.from_numpy(data.train_i).to(dev)
    ins = [e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], B, e.make_plan(ti[s * B:(s + 1) * B]))
           for s in range(args.steps + 1)]
    nwaves = (B // 16) * 4
    buf = torch.zeros(nwaves * 8, dtype=torch.int64, device=dev)
    _lib.check(lib.rg_diag_set_stamps(buf.data_ptr()), "rg_diag_set_stamps")
    _lib.check(lib.rg_diag_set_flags(args.flags), "rg_diag_set_flags")
    per_step = []
    import time
    for s in range(args.steps):
        if args.gap:
            torch.cuda.synchronize()
            time.sleep(0.02)
        e.train_step_in(ins[s], ins[s + 1])
        torch.cuda.synchronize()
        if s >= args.steps // 2:
            per_step.append(buf.view(nwaves, 8)[:, :6].cpu().numpy().astype(np.int64))
    # the same pair pass isolated: validation pairs (no backward) after a sync and an idle
    # gap, alone or right behind a big fill / copy / training step
    vu, vi = tu[:B].contiguous(), ti[:B].contiguous()
    big_a = torch.empty(31 * 2 ** 20, dtype=torch.float32, device=dev)      # 124 MiB
    big_b = torch.empty_like(big_a)
    pre = {"idle": None, "fill124MB": lambda: big_a.fill_(1.0), "copy124MB": lambda: big_b.copy_(big_a),
           "train_step": lambda: e.train_step_in(ins[0], ins[1])}
    plan_v = e.make_plan(vi)

    def bwd(plan):
        e.pairs_and_lists(vu, vi, plan=plan)
        torch.cuda.synchronize()
        e.row_count.zero_()
        e.hot_grad.zero_()
        e.hot_bias.zero_()
    measured = {"val": lambda: e.val_loss(vu, vi), "bwd_noplan": lambda: bwd(None), "bwd_plan": lambda: bwd(plan_v)}
    iso = {}
    for name, fn in [(f"{m}_after_{p}", (fp, fm)) for m, fm in measured.items() for p, fp in pre.items()
                     if m == "val" or p == "idle"]:
        fn, meas = fn
        rows = []
        for _ in range(5):
            torch.cuda.synchronize()
            time.sleep(0.02)
            if fn is not None:
                fn()
            meas()
            torch.cuda.synchronize()
            st = buf.view(nwaves, 8)[:, :2].cpu().numpy().astype(np.int64)
            t = (st - st[:, 0].min()) * 0.01
            rows.append([float(np.median(t[:, 1] - t[:, 0])), float(np.percentile(t[:, 1] - t[:, 0], 90)),
                         float(t[:, 1].max())])
        iso[name] = np.median(np.array(rows), 0).round(2).tolist()
    _lib.check(lib.rg_diag_set_stamps(0), "rg_diag_set_stamps")
    res = {"span_us": [], "start_spread_us": [], "phase_median_us": {p: [] for p in PHASES},
           "phase_p90_us": {p: [] for p in PHASES}}
    for st in per_step:
        t = (st - st[:, 0].min()) * 0.01          # 100 MHz -> us
        res["span_us"].append(float(t[:, 5].max()))
        res["start_spread_us"].append(float(np.percentile(t[:, 0], 90)))
        for k, p in enumerate(PHASES):
            dk = t[:, k + 1] - t[:, k]
            res["phase_median_us"][p].append(float(np.median(dk)))
            res["phase_p90_us"][p].append(float(np.percentile(dk, 90)))
    t = (per_step[-1] - per_step[-1][:, 0].min()) * 0.01
    order = np.argsort(t[:, 0])
    q = len(order) // 4
    res["ids_landed_abs_us_by_start_quartile"] = [round(float(np.median(t[order[k * q:(k + 1) * q], 1])), 2)
                                                  for k in range(4)]
    res["ids_phase_us_by_start_quartile"] = [round(float(np.median(t[order[k * q:(k + 1) * q], 1] -
                                                                   t[order[k * q:(k + 1) * q], 0])), 2)
                                             for k in range(4)]
    res["ids_landed_abs_pct_us"] = np.percentile(t[:, 1], [5, 25, 50, 75, 95]).round(2).tolist()
    out = {"span_us": float(np.median(res["span_us"])), "span_per_step_us": [round(x, 1) for x in res["span_us"]],
           "ids_median_per_step_us": [round(float(np.median((st[:, 1] - st[:, 0]) * 0.01)), 1) for st in per_step],
           "ids_landed_abs_us_by_start_quartile": res["ids_landed_abs_us_by_start_quartile"],
           "ids_phase_us_by_start_quartile": res["ids_phase_us_by_start_quartile"],
           "ids_landed_abs_pct_us": res["ids_landed_abs_pct_us"], "wave_start_p90_us": float(np.median(res["start_spread_us"])),
           "phase_median_us": {p: round(float(np.median(v)), 2) for p, v in res["phase_median_us"].items()},
           "phase_p90_us": {p: round(float(np.median(v)), 2) for p, v in res["phase_p90_us"].items()},
           "val_pairs_ids_median_p90_lastlanded_us_after": iso}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
