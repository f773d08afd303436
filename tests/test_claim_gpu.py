"""Claimed list slots (rg_mf_work_t claim_num_users; the stepper's default single-rank split
step): the prepare of step t + 1, inside step t's dense pass, claims every pair's list slots
and the pair pass writes its entries there without returning atomics.

The dense pass sums a row's entries in sorted order (and an overflowed row in fixed point),
so WHICH slot an entry lands in does not change the sum: the claimed step must equal the
pair pass's own atomics (RG_MF_CLAIM=0) BIT FOR BIT -- per-step losses, tables, optimizer
state, the MT state -- including validation passes between prefetched steps, a prefetched
step that never runs, a partial last batch, plans and no plans, overflowing hot items."""
import os

import numpy as np
import pytest
import torch

from oracle import rng as orng
from tests.test_lazy_gpu import _case, _same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from recommendation_gans_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _engine(dev, claim, tabs, pool_u, pool_i, mt, loss, opt, n, B):
    from recommendation_gans_amd.mf_engine import MFEngine
    old = os.environ.get("RG_MF_CLAIM")
    os.environ["RG_MF_CLAIM"] = "1" if claim else "0"
    try:
        return MFEngine(tabs[0], tabs[1], tabs[2], tabs[3], pool_u, pool_i, mt.copy(), loss=loss, optimizer=opt,
                        lr=1e-2, weight_decay=1e-4, n_neg=n, batch_size=B, device=dev)
    finally:
        if old is None:
            del os.environ["RG_MF_CLAIM"]
        else:
            os.environ["RG_MF_CLAIM"] = old


def _run(dev, claim, tabs, pool_u, pool_i, steps, loss, opt, n, B, mt, plan=True):
    e = _engine(dev, claim, tabs, pool_u, pool_i, mt, loss, opt, n, B)
    tu = [torch.from_numpy(pu).to(dev) for pu, _ in steps]
    ti = [torch.from_numpy(pi).to(dev) for _, pi in steps]
    plans = [e.make_plan(x) if plan else None for x in ti]
    ins = [e.step_input(u, i, None, p) for u, i, p in zip(tu, ti, plans)]
    losses, vals = [], []
    for s in range(len(steps)):
        out = torch.zeros(1, dtype=torch.float32, device=dev)
        if s == 7:
            # a prefetched step that never runs: its claims must not leak into the next one
            e.train_step_in(ins[s], ins[0], loss_out=out)
        else:
            e.train_step_in(ins[s], ins[s + 1] if s + 1 < len(steps) else None, loss_out=out)
        losses.append(out)
        if s in (3, 7):
            vals.append(e.val_loss(tu[1], ti[1]))          # validation after a prefetching step
    torch.cuda.synchronize()
    state = [t.clone().cpu() for t in e.params()] + [x.clone().cpu() for x in e.m if x is not None] + \
        [x.clone().cpu() for x in e.v if x is not None]
    return torch.cat(losses).cpu(), [float(v) for v in vals], state, e.mt_state()


@pytest.mark.parametrize("loss,opt,d,plan", [("bpr", "adam", 64, True), ("pointwise", "adam", 32, True),
                                             ("hinge", "rms", 64, False), ("bpr", "sgd", 128, True),
                                             ("pointwise", "adam", 50, False), ("bpr", "adam", 8, True)])
def test_claimed_slots_equal_pair_pass_atomics(dev, loss, opt, d, plan):
    U, I, B, n = 3000, 400, 256, 5
    tabs, pool_u, pool_i, steps = _case(U, I, d, B, 12, 20000, seed=d + len(loss))
    mt = orng.py_seed_state(7)
    la, va, sa, ma = _run(dev, False, tabs, pool_u, pool_i, steps, loss, opt, n, B, mt, plan)
    lc, vc, sc, mc = _run(dev, True, tabs, pool_u, pool_i, steps, loss, opt, n, B, mt, plan)
    _same(lc, la, "per-step losses")
    assert vc == va, (vc, va)
    for k, (a, b) in enumerate(zip(sc, sa)):
        _same(a, b, f"state tensor {k}")
    assert (mc == ma).all()


def test_claimed_slots_full_size_c2(dev):
    """ML-20M shape (C2: U = 136,677, I = 20,108, d = 64, B = 8192, BPR, Adam), Zipf items
    (hot rows overflow their 8-entry lists): claimed == atomics, bit for bit."""
    U, I, d, B, n = 136677, 20108, 64, 8192, 5
    g = torch.Generator().manual_seed(1)
    tabs = [torch.randn(U, d, generator=g) / d, torch.randn(I, d, generator=g) / d, torch.zeros(U), torch.zeros(I)]
    rs = np.random.RandomState(1)
    pool_u, pool_i = rs.randint(0, U, 2_000_000), rs.randint(0, I, 2_000_000)
    steps = [(rs.randint(0, U, B).astype(np.int64), np.minimum(rs.zipf(1.1, B) - 1, I - 1).astype(np.int64))
             for _ in range(9)]
    mt = orng.py_seed_state(0)
    la, va, sa, ma = _run(dev, False, tabs, pool_u, pool_i, steps, "bpr", "adam", n, B, mt)
    lc, vc, sc, mc = _run(dev, True, tabs, pool_u, pool_i, steps, "bpr", "adam", n, B, mt)
    _same(lc, la, "losses")
    assert vc == va
    for k, (a, b) in enumerate(zip(sc, sa)):
        _same(a, b, f"state tensor {k}")
    assert (mc == ma).all()
