"""Timing probe (scripts only; results are not parity-checked): how much of the MF pair pass
(rg_mf_pairs) hides when it runs beside the dense pass (rg_mf_apply_prepare) on another stream,
at C2 (ML-20M-shaped, d = 64, B = 8192, n = 5, BPR).  Prints us per iteration for:
  serial      pair -> dense on one stream (today's step shape)
  dense only  / pair only
  overlapped  pair on stream A beside dense on stream B, joined every iteration by events
  free        the same without the joins (throughput bound of the pair)
The kernels run on the same buffers every iteration (the numbers are timing only)."""
import ctypes
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from recommendation_gans_amd import _lib  # noqa: E402
from recommendation_gans_amd.mf_engine import MFEngine  # noqa: E402
from recommendation_gans_amd.synthetic import ML20M, movielens_like  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    data = movielens_like(ML20M, seed=0)
    U, I, d, B, n = data.num_users, data.num_items, 64, 8192, 5
    torch.manual_seed(0)
    Uw, Iw = torch.empty(U, d).normal_(0, 1 / d), torch.empty(I, d).normal_(0, 1 / d)
    random.seed(0)
    mt = np.asarray(random.getstate()[1], dtype=np.uint32)
    e = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), data.pool_u, data.pool_i, mt, loss="bpr",
                 optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
    tu = torch.from_numpy(data.train_u[:4 * B].astype(np.int64)).to(dev)
    ti = torch.from_numpy(data.train_i[:4 * B].astype(np.int64)).to(dev)
    ins = [e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], B, e.make_plan(ti[s * B:(s + 1) * B]))
           for s in range(4)]
    for s in range(3):
        e.train_step_in(ins[s], ins[s + 1])
    torch.cuda.synchronize()
    batch, work = e._acquire(ins[3])
    e._release()
    lib = e.lib
    tables = e._tables[e.cur]
    opt = e._opt_step(e.t + 1)
    R = U + I
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def pair(s):
        _lib.check(lib.rg_mf_pairs(ctypes.c_void_p(s.cuda_stream), tables, ctypes.byref(batch), ctypes.byref(work), 1),
                   "pairs")

    def dense(s):
        _lib.check(lib.rg_mf_apply(ctypes.c_void_p(s.cuda_stream), tables, ctypes.byref(work), ctypes.byref(opt), 0, R,
                                   None), "apply")

    def timed(name, body, it=200):
        for _ in range(10):
            body()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            body()
        torch.cuda.synchronize()
        print(f"{name:12s} {(time.perf_counter() - t0) / it * 1e6:8.1f} us/iter", flush=True)

    def serial():
        pair(sa)
        dense(sa)

    ea, eb = torch.cuda.Event(), torch.cuda.Event()

    def overlapped():
        pair(sa)
        dense(sb)
        ea.record(sa)
        eb.record(sb)
        sa.wait_event(eb)
        sb.wait_event(ea)

    def free():
        pair(sa)
        dense(sb)

    for _ in range(2):
        timed("serial", serial)
        timed("dense only", lambda: dense(sa))
        timed("pair only", lambda: pair(sa))
        timed("overlapped", overlapped)
        timed("free", free)


if __name__ == "__main__":
    main()
