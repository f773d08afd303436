"""Driver entry points.

build(): compile librg_hip.so for gfx950 (hipcc, in-tree), compile the oracle's
         C restatement (oracle/Makefile), import the package.
smoke(): one small MF-BPR training step (+ one pointwise step) on cuda:0 through
         the HIP C-ABI, checked against the oracle (CPU restatement).
"""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def build() -> None:
    from recommendation_gans_amd import build as rg_build
    rg_build.build()
    from oracle import rng as orng
    orng.build()
    import recommendation_gans_amd  # noqa: F401
    from recommendation_gans_amd import _lib
    _lib.load()


def smoke() -> None:
    import numpy as np
    import torch

    from oracle import mf as omf
    from oracle import rng as orng
    from recommendation_gans_amd.mf_engine import MFEngine

    dev = torch.device("cuda:0")
    U, I, d, B, n = 500, 300, 64, 256, 5
    for loss in ("bpr", "pointwise"):
        g = torch.Generator().manual_seed(0)
        Uw, Iw = torch.randn(U, d, generator=g) / d, torch.randn(I, d, generator=g) / d
        ub, ib = torch.zeros(U, 1), torch.zeros(I, 1)
        rs = np.random.RandomState(0)
        pool_u, pool_i = rs.randint(0, U, 4000), rs.randint(0, I, 4000)
        pu, pi = rs.randint(0, U, B), rs.randint(0, I, B)
        st = orng.py_seed_state(0)
        o = omf.MFOracle(Uw.clone(), Iw.clone(), ub.clone(), ib.clone(), pool_u, pool_i, st.copy(), loss=loss,
                         optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
        o64 = omf.MFOracle(Uw.double(), Iw.double(), ub.double(), ib.double(), pool_u, pool_i, st.copy(),
                           loss=loss, optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
        o64.step(pu, pi)
        e = MFEngine(Uw, Iw, ub.reshape(-1), ib.reshape(-1), pool_u, pool_i, st.copy(), loss=loss,
                     optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
        ref = o.step(pu, pi)
        got = float(e.train_step(torch.from_numpy(pu).to(dev), torch.from_numpy(pi).to(dev))[0])
        torch.cuda.synchronize()
        assert abs(got - ref) <= 1e-5 * abs(ref), (loss, got, ref)
        for k in range(4):
            ok, msg = omf.tensor_parity(e.params()[k], o.params[k], o64.params[k])
            assert ok, (loss, k, msg)
        assert (e.mt_state() == o.state).all(), "MT state"
    print("smoke ok")


if __name__ == "__main__":
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "smoke":
        smoke()
