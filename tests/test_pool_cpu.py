"""rg_pool_build (native, host) against the NumPy restatement of the reference's
get_negative_samples (spotlight/sampling.py:37-70) on random interactions: the same
pool, and NumPy's global generator left in the same state (the next draws agree).
The reference's own golden pools are checked in test_dropin_cpu.py."""
import numpy as np
import pytest

from recommendation_gans_amd.spotlight.interactions import Interactions
from recommendation_gans_amd.spotlight.sampling import get_negative_samples


def numpy_pool(train, n):
    """sampling.py:46-70 with NumPy calls (vectorised draws, the has_key loop in order)."""
    users = np.random.choice(train.num_users, n)
    items = np.random.choice(train.num_items, n)
    csr = train.csr_matrix
    hit = np.flatnonzero(np.asarray(csr[users, items]).ravel() == 1)
    for k in hit:
        pos = np.sort(csr[users[k], :].toarray().nonzero()[1])
        raw = np.random.randint(0, train.num_items - len(pos), size=1)
        items[k] = raw[0] + np.searchsorted(pos - np.arange(len(pos)), raw[0], side="right")
    return users, items


@pytest.mark.parametrize("U,I,nnz,n,rating,seed", [(50, 40, 600, 3000, 1.0, 0), (300, 1000, 20000, 50000, 1.0, 1),
                                                    (300, 1000, 20000, 50000, 4.0, 2), (7, 4, 10, 200, 1.0, 3),
                                                    (1, 70000, 5, 1000, 1.0, 4)])
def test_native_pool_matches_numpy(U, I, nnz, n, rating, seed):
    rs = np.random.RandomState(seed)
    r = np.full(nnz, rating, np.float32)
    r[::7] = 2.0                                  # mixed ratings: only exact 1s trigger has_key
    train = Interactions(rs.randint(0, U, nnz), rs.randint(0, I, nnz), ratings=r, num_users=U, num_items=I)
    np.random.seed(seed + 100)
    pool = get_negative_samples(train, n)
    after_native = np.random.randint(0, 1 << 30, 5)
    np.random.seed(seed + 100)
    ru, ri = numpy_pool(train, n)
    after_numpy = np.random.randint(0, 1 << 30, 5)
    assert (pool.user_ids == ru).all() and (pool.item_ids == ri).all()
    assert (after_native == after_numpy).all()


def test_user_with_every_item_positive_raises_like_numpy():
    """randint(0, 0) in the reference raises ValueError; so does the native builder."""
    u = np.array([0, 0, 0, 1]), np.array([0, 1, 2, 0])
    train = Interactions(u[0], u[1], ratings=np.ones(4, np.float32), num_users=2, num_items=3)
    np.random.seed(0)
    with pytest.raises(ValueError):
        numpy_pool(train, 500)
    np.random.seed(0)
    with pytest.raises(ValueError):
        get_negative_samples(train, 500)
