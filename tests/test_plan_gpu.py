"""rg_mf_plans_build (rg_plan.hip) against a NumPy restatement of the plan contract
(include/rg_hip.h): planned positives sorted by (item, column), a new partial slot where
the item changes or a block of units_per_block positions starts, item -> first slot.

Covers single batches (full, partial, empty), a whole epoch in one launch (offset /
stride of the replicated data-parallel layout), the owner filter of the owner-sharded
layout (u % world == rank), and batches of more than 16,384 planned positives (the
device-scratch path).  Integer work: bit-exact."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def plan_ref(users, items, lo, m, cols, upb, num_items, world=1, rank=0):
    j = np.arange(m)
    it = items[lo:lo + m]
    keep = np.ones(m, bool) if world == 1 else (users[lo:lo + m] % world == rank)
    j, it = j[keep], it[keep]
    order = np.lexsort((j, it))
    j, it = j[order], it[order]
    n_own = len(j)
    s = np.arange(n_own)
    head = np.ones(n_own, bool)
    if n_own > 1:
        head[1:] = (it[1:] != it[:-1]) | (s[1:] % upb == 0)
    slot = np.cumsum(head) - 1
    perm = np.full(cols, -1, np.int64)
    perm[:n_own] = j
    if world == 1:
        perm[n_own:] = np.arange(n_own, cols)
    pos_slot = np.full(cols, -1, np.int64)
    pos_slot[:n_own] = slot
    seg_items = it[head]
    off = np.searchsorted(seg_items, np.arange(num_items + 1), side="left")
    return perm, pos_slot, off, n_own, int(head.sum())


def _check(plans, users, items, offset, stride, batch_len, cols, upb, num_items, world=1, rank=0):
    n = len(items)
    for k, p in enumerate(plans):
        lo = offset + k * stride
        m = max(0, min(batch_len, n - lo))
        perm, ps, off, n_own, _ = plan_ref(users, items, lo, m, cols, upb, num_items, world, rank)
        assert p.n_planned == n_own, (k, p.n_planned, n_own)
        np.testing.assert_array_equal(p.perm.cpu().numpy(), perm, err_msg=f"perm batch {k}")
        np.testing.assert_array_equal(p.pos_slot.cpu().numpy(), ps, err_msg=f"pos_slot batch {k}")
        np.testing.assert_array_equal(p.item_slot_off.cpu().numpy(), off, err_msg=f"item_slot_off batch {k}")


def _zipf_items(rs, n, num_items):
    w = 1.0 / np.arange(1, num_items + 1)
    return rs.choice(num_items, n, p=w / w.sum()).astype(np.int64)


@pytest.mark.parametrize("n,B,upb", [(8192, 8192, 16), (5000, 8192, 16), (1, 256, 32), (1000, 1024, 8)])
def test_single_batch(n, B, upb):
    from recommendation_gans_amd.mf_engine import build_plan
    rs = np.random.RandomState(n)
    I = 2000
    items = _zipf_items(rs, n, I)
    p = build_plan(torch.from_numpy(items).cuda(), B, upb, I)
    _check([p], None, items, 0, B, max(1, n), B, upb, I)


def test_empty_batch():
    from recommendation_gans_amd.mf_engine import build_plan
    p = build_plan(torch.zeros(0, dtype=torch.int64, device="cuda"), 64, 16, 10)
    assert p.n_planned == 0
    np.testing.assert_array_equal(p.perm.cpu().numpy(), np.arange(64))
    assert (p.pos_slot.cpu().numpy() == -1).all() and (p.item_slot_off.cpu().numpy() == 0).all()


def test_epoch_one_launch_with_offset_stride():
    """Every batch of an epoch, replicated-DP layout: rank 1 of 3 takes [g*3B + B, +B)."""
    from recommendation_gans_amd.mf_engine import build_plans
    rs = np.random.RandomState(1)
    I, B, n = 3000, 512, 40000
    items = _zipf_items(rs, n, I)
    plans = build_plans(torch.from_numpy(items).cuda(), B, 16, I, offset=B, stride=3 * B)
    assert len(plans) == -(-(n - B) // (3 * B))
    _check(plans, None, items, B, 3 * B, B, B, 16, I)


@pytest.mark.parametrize("world,rank", [(2, 1), (8, 3), (8, 0)])
def test_owner_filter(world, rank):
    from recommendation_gans_amd.mf_engine import build_plans
    rs = np.random.RandomState(world * 10 + rank)
    U, I, B = 5000, 4000, 1024
    GC = B * world
    n = GC * 3 + 777                                  # a partial last global batch
    users = rs.randint(0, U, n).astype(np.int64)
    items = _zipf_items(rs, n, I)
    plans = build_plans(torch.from_numpy(items).cuda(), GC, 16, I, users=torch.from_numpy(users).cuda(),
                        world=world, rank=rank, cols=GC)
    assert len(plans) == 4
    _check(plans, users, items, 0, GC, GC, GC, 16, I, world, rank)


def test_large_batch_scratch_path():
    """More than 16,384 planned positives: keys sorted in device scratch."""
    from recommendation_gans_amd.mf_engine import build_plans
    rs = np.random.RandomState(7)
    I, B = 20108, 40000
    items = _zipf_items(rs, 2 * B - 100, I)
    plans = build_plans(torch.from_numpy(items).cuda(), B, 16, I)
    _check(plans, None, items, 0, B, B, B, 16, I)
