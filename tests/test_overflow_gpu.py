"""Heavily overflowed hot rows: a batch whose positives all name a handful of items, so
those item rows take thousands of contributions -- far past the RG_MF_LIST_CAP list slots -- and
sum the surplus in int64 fixed point (rg_common.h: fix_add at 2^48).  At the reference init
(mf_spotlight.py's BilinearNet: ScaledEmbedding N(0, 1/d), zero biases) and Adam, where
g / (|g| + eps) exposes a gradient that nearly cancels, three native steps must stay inside the
fp64 oracle's per-element rounding-noise band (oracle/mf.py elementwise_parity with
MFOracle(noise=True)), the hot rows included; and the fixed-point range must hold the largest
partial sum with room to spare (|sum| * 2^48 well below 2^63)."""
import numpy as np
import pytest
import torch

from oracle import mf as omf
from oracle import rng as orng

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("loss", ["bpr", "pointwise"])
def test_overflowed_hot_rows_match_float64(loss):
    from recommendation_gans_amd.mf_engine import MFEngine
    dev = torch.device("cuda:0")
    U, I, d, B, n, steps = 3000, 300, 64, 4096, 5, 3
    torch.manual_seed(0)
    tabs = omf.init_tables(U, I, d)
    rs = np.random.RandomState(3)
    pool_u, pool_i = rs.randint(0, U, 20000), rs.randint(0, I, 20000)
    # 90 % of the positives on items 0..3 (about 920 contributions each per step), the rest spread
    users = [rs.randint(0, U, B) for _ in range(steps)]
    items = [np.where(rs.rand(B) < 0.9, rs.randint(0, 4, B), rs.randint(0, I, B)) for _ in range(steps)]
    st = orng.py_seed_state(11)
    kw = dict(loss=loss, optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
    o = omf.MFOracle(*[t.clone() for t in tabs], pool_u, pool_i, st.copy(), **kw)
    o64 = omf.MFOracle(*[t.clone().double() for t in tabs], pool_u, pool_i, st.copy(), noise=True, **kw)
    e = MFEngine(tabs[0], tabs[1], tabs[2].reshape(-1), tabs[3].reshape(-1), pool_u, pool_i, st.copy(), device=dev,
                 **kw)
    tu = [torch.from_numpy(u.astype(np.int64)).to(dev) for u in users]
    ti = [torch.from_numpy(i.astype(np.int64)).to(dev) for i in items]
    ins = [e.step_input(tu[s], ti[s], B, e.make_plan(ti[s])) for s in range(steps)]
    for s in range(steps):
        got = e.train_step_in(ins[s], ins[s + 1] if s + 1 < steps else None)
        lo = o.step(users[s], items[s])
        o64.step(users[s], items[s])
        torch.cuda.synchronize()
        assert abs(float(got[0]) - lo) <= 1e-5 * abs(lo), (s, float(got[0]), lo)
        for k in range(4):
            ok, st_ = omf.elementwise_parity(e.params()[k], o.params[k], o64.params[k], noise=o64.noise[k])
            assert ok, (loss, s, k, st_)
        # the hot item rows themselves, element by element against float64 within the band
        hot = e.params()[1][:4].double().cpu()
        ref = o64.params[1][:4]
        band = 1e-5 * ref.abs() + 2.0 * o64.noise[1][:4] + 1e-8 * float(ref.abs().max())
        assert bool(((hot - ref).abs() <= band).all()), (loss, s, float((hot - ref).abs().max()))
    # fixed-point headroom: a step's surplus sum of a hot row is at most its contributions' |dz x|
    # summed; at this init that is orders of magnitude below 2^63 / 2^48 = 32768
    assert float(o64.params[1].abs().max()) < 1.0
