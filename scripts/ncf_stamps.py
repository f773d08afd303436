"""Where the NCF / NeuMF pair kernel spends a tile: per-phase s_memrealtime stamps of the
first two tiles of every workgroup, from the diagnostic library (python -m
recommendation_gans_amd.build --diag -> librg_hip_diag.so).

    python scripts/ncf_stamps.py [--dim 64] [--mf-dim 0] [--steps 10]

Runs the bench configuration (ML-20M-shaped, B=8192, 5 negatives, pointwise, Adam,
device dropout) through NCFEngine and prints median phase durations (us)."""
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

# the backward runs one 16-example block at a time (three per 48-row tile): the stamps inside its
# block loop are block 0's (round 6; before, each block overwrote them, so the phase then named
# "X0 re-read issue + dA2" spanned blocks 0 and 1 whole and block 2 up to dA2)
WAVE_PHASES = ["ids+slots", "gather issue", "gather + fwd layer 1", "fwd rest + output", "loss + next-tile warm",
               "(backward entry)", "blk0: X0 re-read issue, out layer, dW4, dA3, dW3, dA2", "blk0: dW2",
               "blk0: dA1 + stage", "blk0: dW1", "blk0: dX0 + contrib stores", "blocks 1-2: whole backward",
               "overflow + planned"]
PHASES = ["ids+slots", "gather", "forward layer 0", "forward rest + output", "loss", "backward first layer", "backward rest + rows"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--mf-dim", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--wave", action="store_true", help="the E = 64 wave-per-tile kernel (16 stamps per wave tile)")
    args = ap.parse_args()
    lib = _lib.load(build.DIAG_LIB)
    lib.rg_diag_set_ncf_stamps.argtypes = [ctypes.c_void_p]
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from recommendation_gans_amd.synthetic import ML20M, movielens_like
    from recommendation_gans_amd.ncf_spotlight import mlp_layers
    from recommendation_gans_amd.spotlight.dnn_models.mlp import MLP
    from recommendation_gans_amd.spotlight.dnn_models.neuMF import NeuMF
    dev = torch.device("cuda:0")
    E, M, B, n = args.dim, args.mf_dim, 8192, 5
    data = movielens_like(ML20M, seed=0, zipf_s=1.0)
    U, I = data.num_users, data.num_items
    torch.manual_seed(0)
    net = NeuMF(mlp_layers(E), U, I, mf_embedding_dim=M, mlp_embedding_dim=E) if M else \
        MLP(layers=mlp_layers(E), num_users=U, num_items=I, embedding_dim=E)
    ps = [p.detach() for p in net.parameters()]
    random.seed(0)
    mt = np.asarray(random.getstate()[1], dtype=np.uint32)
    extra = dict(mf_user_w=ps[2], mf_item_w=ps[3]) if M else {}
    e = NCFEngine(ps[0], ps[1], ps[4:] if M else ps[2:], data.pool_u, data.pool_i, mt, loss="pointwise", lr=1e-3,
                  weight_decay=1e-5, n_neg=n, batch_size=B, device=dev, seed=0, **extra)
    tu, ti = torch.from_numpy(data.train_u).to(dev), torch.from_numpy(data.train_i).to(dev)
    plans = [e.make_plan(ti[s * B:(s + 1) * B]) for s in range(args.steps)]
    if args.wave:
        return wave_main(lib, e, tu, ti, plans, args, B)
    buf = torch.zeros(e.blocks * 2 * 8, dtype=torch.int64, device=dev)
    res = {p: [] for p in PHASES}
    tile_us, starts = [], []
    for s in range(args.steps):
        on = s >= args.steps // 2
        _lib.check(lib.rg_diag_set_ncf_stamps(buf.data_ptr() if on else None), "stamps")
        e.train_step(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], plan=plans[s])
        torch.cuda.synchronize()
        if on:
            st = buf.view(e.blocks, 2, 8).cpu().numpy().astype(np.int64)
            t = (st - st[:, 0, 0].min()) * 0.01
            for k, p in enumerate(PHASES):
                res[p].append(float(np.median(t[:, :, k + 1] - t[:, :, k])))
            tile_us.append(float(np.median(t[:, :, 7] - t[:, :, 0])))
            starts.append(float(np.percentile(t[:, 0, 0], 90)))
    _lib.check(lib.rg_diag_set_ncf_stamps(None), "stamps")
    print(json.dumps({"dim": E, "mf_dim": M, "blocks": e.blocks, "tile_us_median": round(float(np.median(tile_us)), 2),
                      "block_start_p90_us": round(float(np.median(starts)), 2),
                      "phase_median_us": {p: round(float(np.median(v)), 2) for p, v in res.items()}}, indent=1))


def wave_main(lib, e, tu, ti, plans, args, B):
    nw = e.blocks * 4
    buf = torch.zeros(nw * 3 * 16, dtype=torch.int64, device=tu.device)
    res = {p: [] for p in WAVE_PHASES}
    tail = {p: [] for p in WAVE_PHASES}   # p95 over the waves of a phase
    tile_p = []                           # p50 / p90 / max over the waves of a whole tile
    tile_us, first_us, kern_us, pro, red_us, wr_us, tiles_done, bar_wait, ends = [], [], [], [], [], [], [], [], []
    for s in range(args.steps):
        on = s >= args.steps // 2
        buf.zero_()
        _lib.check(lib.rg_diag_set_ncf_stamps(buf.data_ptr() if on else None), "stamps")
        e.train_step(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], plan=plans[s])
        torch.cuda.synchronize()
        if on:
            st = buf.view(nw, 3, 16).cpu().numpy().astype(np.int64)
            t0 = st[:, 0, 0][st[:, 0, 0] > 0].min()
            t = (st - t0) * 0.01
            ok0 = st[:, 0, 13] > 0
            for k, p in enumerate(WAVE_PHASES):
                res[p].append(float(np.median(t[ok0, 0, k + 1] - t[ok0, 0, k])))
                tail[p].append(float(np.percentile(t[ok0, 0, k + 1] - t[ok0, 0, k], 95)))
            tw = t[ok0, 0, 13] - t[ok0, 0, 0]
            tile_p.append([float(np.percentile(tw, 50)), float(np.percentile(tw, 90)), float(tw.max())])
            tile_us.append(float(np.median(t[ok0, 0, 13] - t[ok0, 0, 0])))
            first_us.append(float(np.percentile(t[ok0, 0, 0], 90)))
            # record 2 (kernel level): 0 entry, 1 tiles done, 2 after the workgroup barrier,
            # 3 / 4 reduction rounds, 5 exit
            k2 = t[:, 2, :]
            kern_us.append(float(k2[:, 5].max() - k2[:, 0].min()))
            pro.append(float(np.median(t[ok0, 0, 0] - k2[ok0, 0])))
            tiles_done.append(float(np.median(k2[:, 1] - k2[:, 0])))
            bar_wait.append(float(np.median(k2[:, 2] - k2[:, 1])))
            red_us.append(float(np.median(k2[:, 4] - k2[:, 2])))
            wr_us.append(float(np.median(k2[:, 5] - k2[:, 4])))
            ends.append(float(np.max(k2[:, 1]) - np.min(k2[:, 0])))
    _lib.check(lib.rg_diag_set_ncf_stamps(None), "stamps")
    print(json.dumps({"kernel": "ncf_wave_kernel", "blocks": e.blocks, "waves": nw,
                      "tile_us_median": round(float(np.median(tile_us)), 2),
                      "wave_start_p90_us": round(float(np.median(first_us)), 2),
                      "kernel_entry_to_exit_us": round(float(np.median(kern_us)), 2),
                      "prologue_us_median": round(float(np.median(pro)), 2),
                      "entry_to_tiles_done_us_median": round(float(np.median(tiles_done)), 2),
                      "last_wave_tiles_done_us": round(float(np.median(ends)), 2),
                      "barrier_wait_us_median": round(float(np.median(bar_wait)), 2),
                      "reduction_us_median": round(float(np.median(red_us)), 2),
                      "partial_write_us_median": round(float(np.median(wr_us)), 2),
                      "tile_us_p50_p90_max": [round(float(np.median([x[i] for x in tile_p])), 2) for i in range(3)],
                      "phase_median_us": {p: round(float(np.median(v)), 2) for p, v in res.items()},
                      "phase_p95_us": {p: round(float(np.median(v)), 2) for p, v in tail.items()}}, indent=1))


if __name__ == "__main__":
    main()
