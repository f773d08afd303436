"""The overlapped MF step (rg_mf_step_front + rg_mf_step_hot, the stepper's default)
against the split step (rg_mf_pairs + rg_mf_apply, RG_FUSED=0) and the oracle.

Both compute every row's update with the same device code; the fused step only
reorders WHEN rows are updated: rows no pair of the step touches are updated in the
same grid as the pair pass (weight decay only), touched rows afterwards through the
owner flags the marked prepare leaves in the pairs buffer.  So:
* rows never touched by any step are bit-identical between the two paths;
* touched rows agree to the run-to-run noise of the contribution lists' order
  (list slots are claimed by atomics in either path): 1e-6 relative, tensor norm;
* negative pairs and the MT state are bit-exact (ownership flags masked);
* the scratch (row lists, overflow accumulators) is left zero.
"""
import numpy as np
import pytest
import torch

from oracle import mf as omf
from oracle import rng as orng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from recommendation_gans_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()
    if not _lib.ab_build():
        # the overlapped step (RG_FUSED) is a measured-slower alternative carried only by the A/B build
        # (DESIGN.md §9): scripts/gpu_ab_tests.sh runs this file with RG_LIB pointing at it
        pytest.skip("A/B build only (RG_LIB=recommendation_gans_amd/_variants/librg_hip_ab.so)")
    return torch.device("cuda:0")


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _problem(U, I, d, B, n_batches, seed, P=200_000):
    g = torch.Generator().manual_seed(seed)
    tabs = [torch.randn(U, d, generator=g) / d, torch.randn(I, d, generator=g) / d,
            torch.randn(U, generator=g) * 0.1, torch.randn(I, generator=g) * 0.1]
    rs = np.random.RandomState(seed)
    pool_u, pool_i = rs.randint(0, U, P), rs.randint(0, I, P)
    # Zipf-ish items so some rows overflow the lists, users spread
    items = np.minimum(rs.zipf(1.3, size=n_batches * B) - 1, I - 1)
    users = rs.randint(0, U, n_batches * B)
    return tabs, pool_u, pool_i, users, items


def _engine(dev, tabs, pool_u, pool_i, st, loss, opt, B, n, fused, monkeypatch, **kw):
    from recommendation_gans_amd.mf_engine import MFEngine
    monkeypatch.setenv("RG_FUSED", "1" if fused else "0")
    return MFEngine(tabs[0], tabs[1], tabs[2], tabs[3], pool_u, pool_i, st.copy(), loss=loss, optimizer=opt,
                    lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev, **kw)


def _run(e, dev, users, items, B, steps, plan, val_at=None, last_partial=False):
    tu = torch.from_numpy(users).to(dev)
    ti = torch.from_numpy(items).to(dev)
    spans = [(s * B, (s + 1) * B) for s in range(steps)]
    if last_partial:
        spans[-1] = (spans[-1][0], spans[-1][1] - 37)
    ins = []
    for a, b in spans:
        p = e.make_plan(ti[a:b]) if plan else None
        ins.append(e.step_input(tu[a:b], ti[a:b], None, p))
    losses, vals = [], []
    for s in range(steps):
        got = e.train_step_in(ins[s], ins[s + 1] if s + 1 < steps else None)
        losses.append(float(got[0]))
        if s == val_at:   # a validation draw between steps discards the prefetched pairs
            a, b = spans[0]
            vals.append(float(e.val_loss(tu[a:b], ti[a:b])[0]))
    torch.cuda.synchronize()
    return losses, vals


@pytest.mark.parametrize("loss,opt,plan", [("bpr", "adam", True), ("pointwise", "adam", False),
                                           ("hinge", "rms", True), ("pointwise", "sgd", True)])
def test_fused_matches_split(dev, loss, opt, plan, monkeypatch):
    U, I, d, B, n, steps = 30_000, 4_000, 64, 4096, 5, 7
    tabs, pool_u, pool_i, users, items = _problem(U, I, d, B, steps, seed=1)
    st = orng.py_seed_state(42)
    res = {}
    for fused in (1, 0):
        e = _engine(dev, tabs, pool_u, pool_i, st, loss, opt, B, n, fused, monkeypatch)
        losses, vals = _run(e, dev, users, items, B, steps, plan, val_at=2, last_partial=True)
        res[fused] = (losses, vals, [t.clone() for t in e.params()], [t.clone() for t in e.v if t is not None],
                      e.mt_state())
        assert int(e.row_count.abs().sum()) == 0
        assert float(e.hot_grad.abs().sum()) == 0.0 and float(e.hot_bias.abs().sum()) == 0.0
        del e
    (lf, vf, pf, sf, mf), (ls, vs, ps, ss, ms) = res[1], res[0]
    np.testing.assert_allclose(lf, ls, rtol=1e-6)
    np.testing.assert_allclose(vf, vs, rtol=1e-6)
    assert (mf == ms).all()
    # rows that no step touched: identical code path (zero data gradient) -> bit-identical
    touched = [np.zeros(U, bool), np.zeros(I, bool)]
    st2 = st.copy()
    for s in range(steps):
        b = B if s < steps - 1 else B - 37
        idx = orng.py_choices_indices(st2, len(pool_u), n * B)
        if s == 2:
            orng.py_choices_indices(st2, len(pool_u), n * B)       # the validation draw
        touched[0][pool_u[idx]] = True
        touched[1][pool_i[idx]] = True
        touched[0][users[s * B:s * B + b]] = True
        touched[1][items[s * B:s * B + b]] = True
    assert (st2 == mf).all()
    for k, side in enumerate((0, 1, 0, 1)):
        cold = torch.from_numpy(~touched[side])
        assert torch.equal(pf[k].cpu()[cold], ps[k].cpu()[cold]), f"cold rows of table {k} differ"
        assert _rel(pf[k], ps[k]) <= 1e-6, f"table {k}: {_rel(pf[k], ps[k]):.2e}"
    for a, b in zip(sf, ss):
        assert _rel(a, b) <= 1e-6


def test_fused_oracle_trajectory_prefetch(dev, monkeypatch):
    """Fused steps with the next step prepared inside the front grid, a ring slot
    boundary every 4 steps (RG_MT_UNITS default), and an export in the middle of a slot:
    loss / tables against the oracle, MT state exact after every step."""
    U, I, d, B, n, steps = 2_000, 700, 32, 512, 5, 9
    tabs, pool_u, pool_i, users, items = _problem(U, I, d, B, steps, seed=2, P=5_000)
    st = orng.py_seed_state(7)
    st[624] = 100
    o = omf.MFOracle(*[t.clone().reshape(t.shape[0], -1) for t in tabs], pool_u, pool_i, st.copy(), loss="bpr",
                     optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    o64 = omf.MFOracle(*[t.clone().double().reshape(t.shape[0], -1) for t in tabs], pool_u, pool_i, st.copy(),
                       loss="bpr", optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    e = _engine(dev, tabs, pool_u, pool_i, st, "bpr", "adam", B, n, 1, monkeypatch)
    tu, ti = torch.from_numpy(users).to(dev), torch.from_numpy(items).to(dev)
    ins = [e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], None, e.make_plan(ti[s * B:(s + 1) * B]))
           for s in range(steps)]
    for s in range(steps):
        ref = o.step(users[s * B:(s + 1) * B], items[s * B:(s + 1) * B])
        o64.step(users[s * B:(s + 1) * B], items[s * B:(s + 1) * B])
        got = e.train_step_in(ins[s], ins[s + 1] if s + 1 < steps else None)
        torch.cuda.synchronize()
        np.testing.assert_allclose(float(got[0]), ref, rtol=1e-5)
        assert (e.mt_state() == o.state).all(), f"MT state after step {s}"
        for k in range(4):
            shp = e.params()[k].shape
            ok, msg = omf.tensor_parity(e.params()[k], o.params[k].reshape(shp), o64.params[k].reshape(shp),
                                        rtol=1e-5)
            assert ok, f"step {s} table {k}: {msg}"
