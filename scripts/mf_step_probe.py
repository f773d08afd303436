"""Decompose the overlapped MF step (rg_mf_step_front / rg_mf_step_hot) on one GPU.

    python scripts/mf_step_probe.py [--iters 30]

Times, with HIP events on the launch stream, at the bench configuration (ML-20M
shaped, d=64, B=8192, bpr, Adam):
  split   rg_mf_pairs alone, rg_mf_apply (all rows) alone
  front   rg_mf_step_front with the cold range full, and empty (= pair pass only)
  hot     rg_mf_step_hot by stamp scan and by owner flags
  two_stream  rg_mf_step_cold on a side stream beside rg_mf_pairs, then hot
  serial  cold, pairs, hot one after another (each alone on the GPU)
Run under rocprofv3 --kernel-trace --stats with one --variant for kernel durations.
Diagnostic only: the "empty cold range" variant skips the cold-row update, so the
tables it leaves are not a training state.
"""
import argparse
import ctypes
import json
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from recommendation_gans_amd import _lib  # noqa: E402
from recommendation_gans_amd._lib import check, ptr  # noqa: E402
from recommendation_gans_amd.mf_engine import MFEngine  # noqa: E402
from recommendation_gans_amd.synthetic import ML20M, movielens_like  # noqa: E402


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--variant", nargs="*")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    d, B, n = args.dim, args.batch, 5
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
    nb = 3 * args.iters + 10
    ins = [e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], B, e.make_plan(ti[s * B:(s + 1) * B]))
           for s in range(nb)]
    for s in range(5):                      # realistic optimizer state
        e.train_step_in(ins[s], ins[s + 1])
    torch.cuda.synchronize()
    stamps = [torch.zeros(U + I, dtype=torch.int32, device=dev) for _ in range(2)]
    serial = [1000]
    R = U + I
    res = {}

    def mark(k):
        serial[0] += 1
        m = _lib.MFMark()
        m.stamp, m.num_users, m.serial = ptr(stamps[k]), U, serial[0]
        return m

    def run(name, body):
        ts = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(args.iters):
            x = ins[5 + it]
            batch, work = e._acquire(x)
            t = body(batch, work, x)
            e._release()
            e.finish_step()
            ts.append(t)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.iters * 1e6
        res[name] = {k: float(np.median([a.elapsed_time(b) * 1e3 for a, b in (t[k] for t in ts[3:])]))
                     for k in ts[0]}
        res[name]["wall_us_per_iter"] = wall
        print(name, json.dumps(res[name]), flush=True)

    stream = _lib.stream_handle

    def split(batch, work, x):
        a = ev()
        check(lib.rg_mf_pairs(stream(), e._tables[e.cur], ctypes.byref(batch), ctypes.byref(work), 1), "pairs")
        b = ev()
        o = e._opt_step(e.t + 1)
        check(lib.rg_mf_apply(stream(), e._tables[e.cur], ctypes.byref(work), ctypes.byref(o), 0, R,
                              e._loss(B, e.loss_out)), "apply")
        c = ev()
        return {"pairs_us": (a, b), "apply_us": (b, c)}

    def fused(cold_end, scan):
        def body(batch, work, x):
            m = mark(0)
            check(lib.rg_mf_prepare_marked(stream(), ctypes.byref(batch), ctypes.byref(work), ctypes.byref(m)),
                  "prep")
            o = e._opt_step(e.t + 1)
            a = ev()
            check(lib.rg_mf_step_front(stream(), e._tables[e.cur], ctypes.byref(batch), ctypes.byref(work),
                                       ctypes.byref(m), ctypes.byref(o), 0, cold_end, None, None, None), "front")
            b = ev()
            check(lib.rg_mf_step_hot(stream(), e._tables[e.cur], ctypes.byref(batch), ctypes.byref(work),
                                     ctypes.byref(m) if scan else None, ctypes.byref(o), 0, R,
                                     e._loss(B, e.loss_out)), "hot")
            c = ev()
            return {"front_us": (a, b), "hot_us": (b, c)}
        return body

    side = torch.cuda.Stream(device=dev)

    def two_stream(cold_first):
        def body(batch, work, x):
            m = mark(0)
            check(lib.rg_mf_prepare_marked(stream(), ctypes.byref(batch), ctypes.byref(work), ctypes.byref(m)),
                  "prep")
            o = e._opt_step(e.t + 1)
            a = ev()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                check(lib.rg_mf_step_cold(_lib.stream_handle(side), e._tables[e.cur], ctypes.byref(m),
                                          ctypes.byref(o), 0, R), "cold")
            check(lib.rg_mf_pairs(stream(), e._tables[e.cur], ctypes.byref(batch), ctypes.byref(work), 1), "pairs")
            torch.cuda.current_stream().wait_stream(side)
            b = ev()
            check(lib.rg_mf_step_hot(stream(), e._tables[e.cur], ctypes.byref(batch), ctypes.byref(work),
                                     ctypes.byref(m), ctypes.byref(o), 0, R, e._loss(B, e.loss_out)), "hot")
            c = ev()
            return {"pairs_cold_us": (a, b), "hot_us": (b, c)}
        return body

    def serial_body(batch, work, x):
        m = mark(0)
        check(lib.rg_mf_prepare_marked(stream(), ctypes.byref(batch), ctypes.byref(work), ctypes.byref(m)), "prep")
        o = e._opt_step(e.t + 1)
        a = ev()
        check(lib.rg_mf_step_cold(stream(), e._tables[e.cur], ctypes.byref(m), ctypes.byref(o), 0, R), "cold")
        b = ev()
        check(lib.rg_mf_pairs(stream(), e._tables[e.cur], ctypes.byref(batch), ctypes.byref(work), 1), "pairs")
        c = ev()
        check(lib.rg_mf_step_hot(stream(), e._tables[e.cur], ctypes.byref(batch), ctypes.byref(work),
                                 ctypes.byref(m), ctypes.byref(o), 0, R, e._loss(B, e.loss_out)), "hot")
        d_ = ev()
        return {"cold_us": (a, b), "pairs_us": (b, c), "hot_us": (c, d_)}

    variants = {"split": split, "fused_scan": fused(R, True), "fused_owner": fused(R, False),
                "front_pairs_only": fused(0, True), "two_stream": two_stream(False), "serial": serial_body}
    for v in (args.variant or list(variants)):
        run(v, variants[v])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
