"""The lazy dense pass (rg_mf_pairs_prepare + rg_mf_apply_lazy +
rg_mf_lazy_flush) against the eager dense pass it replaces (RG_LAZY=0: every row every
step, the reference's dense optimizer, optimizers.py:10-16 over sparse=False tables).

Deferring a row's cold updates and applying them later, in step order with each step's
constants, is the same operation sequence, so the two runs must agree BIT FOR BIT: the
loss of every step, every table and the optimizer state after a flush, the MT state --
across prefetched steps (the lazy path proper), a validation pass in the middle (which
flushes), a partial last batch, plans, every optimizer and loss.  The eager pass itself is
pinned to the oracle and the reference goldens by test_mf_gpu.py / test_configs_gpu.py."""
import os

import numpy as np
import pytest
import torch

from oracle import rng as orng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from recommendation_gans_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()
    if not _lib.ab_build():
        # the lazy dense pass is a measured-slower alternative carried only by the A/B build
        # (DESIGN.md §9): scripts/gpu_ab_tests.sh runs this file with RG_LIB pointing at it
        pytest.skip("A/B build only (RG_LIB=recommendation_gans_amd/_variants/librg_hip_ab.so)")
    return torch.device("cuda:0")


def _case(U, I, d, B, nsteps, pool_len, seed, partial_last=True):
    g = torch.Generator().manual_seed(seed)
    tabs = [torch.randn(U, d, generator=g) / d, torch.randn(I, d, generator=g) / d,
            torch.randn(U, generator=g) * 1e-3, torch.randn(I, generator=g) * 1e-3]
    rs = np.random.RandomState(seed)
    pool_u, pool_i = rs.randint(0, U, pool_len), rs.randint(0, I, pool_len)
    # Zipf-ish items (hot rows overflow their lists), users concentrated on a subset so
    # many users stay cold for several steps (long lags)
    steps = []
    for s in range(nsteps):
        m = B if not (partial_last and s == nsteps - 1) else B // 3
        pu = rs.randint(0, U // 3, m)
        pi = np.minimum(rs.zipf(1.3, m) - 1, I - 1)
        steps.append((pu.astype(np.int64), pi.astype(np.int64)))
    return tabs, pool_u, pool_i, steps


def _run(dev, lazy, tabs, pool_u, pool_i, steps, loss, opt, n, B, mt, plan=True, val_at=None, count=False):
    from recommendation_gans_amd.mf_engine import MFEngine
    old = os.environ.get("RG_LAZY")
    os.environ["RG_LAZY"] = "1" if lazy else "0"
    try:
        e = MFEngine(tabs[0], tabs[1], tabs[2], tabs[3], pool_u, pool_i, mt.copy(), loss=loss, optimizer=opt,
                     lr=1e-2, weight_decay=1e-4, n_neg=n, batch_size=B, device=dev)
    finally:
        if old is None:
            del os.environ["RG_LAZY"]
        else:
            os.environ["RG_LAZY"] = old
    tu = [torch.from_numpy(pu).to(dev) for pu, _ in steps]
    ti = [torch.from_numpy(pi).to(dev) for _, pi in steps]
    plans = [e.make_plan(x) if plan else None for x in ti]
    ins = [e.step_input(u, i, None, p) for u, i, p in zip(tu, ti, plans)]
    if count:
        e.lazy_rows(enable=True)
    losses, vals = [], []
    for s in range(len(steps)):
        out = torch.zeros(1, dtype=torch.float32, device=dev)
        e.train_step_in(ins[s], ins[s + 1] if s + 1 < len(steps) else None, loss_out=out)
        losses.append(out)
        if val_at is not None and s == val_at:
            vals.append(e.val_loss(tu[0], ti[0]))
    rows = e.lazy_rows() if count else None
    torch.cuda.synchronize()
    state = [t.clone() for t in e.params()] + [x.clone() for x in e.m if x is not None] + \
        [x.clone() for x in e.v if x is not None]
    return e, torch.cat(losses).cpu(), [float(v) for v in vals], state, e.mt_state(), rows


def _same(a, b, what):
    assert a.shape == b.shape, what
    diff = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
    assert not bool(diff.any()), f"{what}: {int(diff.sum())} of {a.numel()} elements differ"


@pytest.mark.parametrize("loss,opt,d", [("bpr", "adam", 64), ("pointwise", "adam", 32), ("hinge", "rms", 64),
                                        ("adaptive_hinge", "adam", 64), ("bpr", "sgd", 128),
                                        ("pointwise", "adam", 50), ("bpr", "adam", 8),
                                        ("adaptive_hinge", "adam", 8)])
def test_lazy_equals_eager_bitwise(dev, loss, opt, d):
    U, I, B, n = 3000, 400, 256, 5
    tabs, pool_u, pool_i, steps = _case(U, I, d, B, 14, 20000, seed=d + len(loss))
    mt = orng.py_seed_state(3)
    _, le, ve, se, mte, _ = _run(dev, False, tabs, pool_u, pool_i, steps, loss, opt, n, B, mt, val_at=6)
    el, ll, vl, sl, mtl, rows = _run(dev, True, tabs, pool_u, pool_i, steps, loss, opt, n, B, mt, val_at=6,
                                     count=True)
    _same(ll, le, "per-step losses")
    assert vl == ve, (vl, ve)
    for k, (a, b) in enumerate(zip(sl, se)):
        _same(a.cpu(), b.cpu(), f"state tensor {k}")
    assert (mtl == mte).all()
    # the lazy path really skipped rows: fewer user rows than U per step
    assert rows is not None and 0 < rows < U * len(steps), rows


def _fit_like(dev, lazy, loss, epochs=3, val=True):
    """implicit.py's fit loop on the fit golden's problem (U 30, I 20, d 8, B 32): the step
    inputs built once and replayed every epoch, the last step of an epoch without a next
    step, validation batches and a params() snapshot between epochs."""
    from recommendation_gans_amd.mf_engine import MFEngine
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "mf_fit_golden.npz"))
    U, I, d, B, n = (int(x) for x in z["meta"])
    key = loss if f"{loss}_init_U" in z else "pointwise"
    tabs = [torch.from_numpy(z[f"{key}_init_U"]), torch.from_numpy(z[f"{key}_init_I"]), torch.zeros(U),
            torch.zeros(I)]
    old = os.environ.get("RG_LAZY")
    os.environ["RG_LAZY"] = "1" if lazy else "0"
    try:
        e = MFEngine(*tabs, z["pool_u"], z["pool_i"], z[f"{key}_mt_state"].copy(), loss=loss, optimizer="adam",
                     lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
    finally:
        if old is None:
            del os.environ["RG_LAZY"]
        else:
            os.environ["RG_LAZY"] = old
    tu, ti = (torch.from_numpy(z[k].astype(np.int64)).to(dev) for k in ("train_u", "train_i"))
    vu, vi = (torch.from_numpy(z[k].astype(np.int64)).to(dev) for k in ("valid_u", "valid_i"))
    nb = (len(tu) + B - 1) // B
    plans = e.make_plans(ti)
    ins = [e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], None, plans[s]) for s in range(nb)]
    losses, vals, snaps = [], [], []
    for _ in range(epochs):
        for s in range(nb):
            out = torch.zeros(1, dtype=torch.float32, device=dev)
            e.train_step_in(ins[s], ins[s + 1] if s + 1 < nb else None, loss_out=out)
            losses.append(out)
        if val:
            vals += [float(e.val_loss(vu[s:s + B], vi[s:s + B])[0]) for s in range(0, len(vu), B)]
        snaps.append([t.clone().cpu() for t in e.params()])
    return torch.cat(losses).cpu(), vals, snaps, e.mt_state()


@pytest.mark.parametrize("loss", ["pointwise", "adaptive_hinge"])
def test_lazy_fit_loop_equals_eager(dev, loss):
    le, ve, se, mte = _fit_like(dev, False, loss)
    ll, vl, sl, mtl = _fit_like(dev, True, loss)
    bad = [k for k in range(len(le)) if le[k] != ll[k]]
    assert not bad, f"steps {bad} differ: eager {le.tolist()} lazy {ll.tolist()}"
    assert vl == ve, (vl, ve)
    for ep, (a, b) in enumerate(zip(sl, se)):
        for k in range(4):
            _same(a[k], b[k], f"epoch {ep} table {k}")
    assert (mtl == mte).all()


def test_lazy_without_plan_and_two_flushes(dev):
    """No plans, a flush (params()) between prefetched steps, then more lazy steps."""
    from recommendation_gans_amd.mf_engine import MFEngine  # noqa: F401
    U, I, d, B, n = 2000, 300, 64, 128, 3
    tabs, pool_u, pool_i, steps = _case(U, I, d, B, 10, 9000, seed=11, partial_last=False)
    mt = orng.py_seed_state(5)
    res = []
    for lazy in (False, True):
        e, losses, _, _, _, _ = _run(dev, lazy, tabs, pool_u, pool_i, steps[:5], "bpr", "adam", n, B, mt,
                                     plan=False)
        mid = [t.clone().cpu() for t in e.params()]
        # continue on the same engine with prefetched steps
        tu = [torch.from_numpy(pu).to(dev) for pu, _ in steps[5:]]
        ti = [torch.from_numpy(pi).to(dev) for _, pi in steps[5:]]
        ins = [e.step_input(u, i) for u, i in zip(tu, ti)]
        for s in range(len(ins)):
            e.train_step_in(ins[s], ins[s + 1] if s + 1 < len(ins) else ins[0])   # the last prefetch is unused
        e.flush()
        res.append((losses, mid, [t.clone().cpu() for t in e.params()], [x.clone().cpu() for x in e.m]))
    (l0, m0, p0, a0), (l1, m1, p1, a1) = res
    _same(l1, l0, "losses")
    for k in range(4):
        _same(m1[k], m0[k], f"mid params {k}")
        _same(p1[k], p0[k], f"final params {k}")
        _same(a1[k], a0[k], f"final m {k}")


def test_lazy_full_size_c2(dev):
    """ML-20M shape (U = 136,677, I = 20,108, d = 64, B = 8192, BPR, Adam): a run of
    prefetched lazy steps equals the eager pass bit for bit after the flush."""
    U, I, d, B, n = 136677, 20108, 64, 8192, 5
    g = torch.Generator().manual_seed(0)
    tabs = [torch.randn(U, d, generator=g) / d, torch.randn(I, d, generator=g) / d, torch.zeros(U), torch.zeros(I)]
    rs = np.random.RandomState(0)
    pool_u, pool_i = rs.randint(0, U, 2_000_000), rs.randint(0, I, 2_000_000)
    steps = [(rs.randint(0, U, B).astype(np.int64), np.minimum(rs.zipf(1.1, B) - 1, I - 1).astype(np.int64))
             for _ in range(6)]
    mt = orng.py_seed_state(0)
    _, le, _, se, mte, _ = _run(dev, False, tabs, pool_u, pool_i, steps, "bpr", "adam", n, B, mt)
    _, ll, _, sl, mtl, rows = _run(dev, True, tabs, pool_u, pool_i, steps, "bpr", "adam", n, B, mt, count=True)
    _same(ll, le, "losses")
    for k, (a, b) in enumerate(zip(sl, se)):
        _same(a.cpu(), b.cpu(), f"state tensor {k}")
    assert (mtl == mte).all()
    assert rows < U * len(steps)
