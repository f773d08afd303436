"""Diagnostic (scripts only): run a few MF steps (U=3000, I=400, B=1024, n=5, bpr, d=64, Zipf items
with plans) on the library RG_LIB / RG_PIPE select, and dump tables + optimizer state after every
step to an .npz, for bit-comparison of two runs (e.g. the lean dense pass vs the product one)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.test_pipe_gpu import _engine, _inputs, _state  # noqa: E402


def main(out, steps=3, pipe=False):
    U, I, B, n, d = 3000, 400, 1024, 5, 64
    e = _engine(pipe, "bpr", d, U, I, B, n)
    ins = _inputs(e, U, I, B, steps)
    res = {}
    for s in range(steps):
        nx = ins[s + 1] if s + 1 < steps else None
        nx2 = ins[s + 2] if s + 2 < steps else None
        loss = float(e.train_step_in(ins[s], nx, next2=nx2)[0]) if pipe else float(e.train_step_in(ins[s], nx)[0])
        t, st, mt = _state(e)
        res[f"loss{s}"] = np.array(loss)
        for k, x in enumerate(t + st):
            res[f"s{s}_{k}"] = x.numpy()
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1], pipe=len(sys.argv) > 2 and sys.argv[2] == "pipe")
