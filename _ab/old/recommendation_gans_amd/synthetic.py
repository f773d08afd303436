"""Synthetic MovieLens-shaped implicit-feedback data (no dataset download is possible).

Shapes follow SURVEY.md §8(d): ML-20M after the reference's own filter
(rating > 3.5, users with >= 5 ratings; spotlight/datasets/movielens.py:119-121)
has U = 136,677 users, I = 20,108 items and ~10.0 M positives.  The time split
mirrors utils/data_provider.py:77-78 (train_test_timebased_split twice, 10 % each:
train 81 %, valid 9 %, test 10 %; cutoff at spotlight/dataset_manilupation.py:210),
and the negative pool mirrors spotlight/sampling.py:46-70 on freshly processed
data, where ``has_key`` never fires: ``len(train)`` uniform
(user, item) pairs, users drawn first, then items.

Generator (seeded ``np.random.RandomState``):
  * per-user counts ~ lognormal(0, 1), floored at 5, rescaled to sum to N;
  * item ids ~ Zipf(s) over a random permutation of the items;
  * timestamps = a random permutation (all distinct, so the split is unambiguous).
"""
from dataclasses import dataclass

import numpy as np

ML20M = dict(num_users=136_677, num_items=20_108, num_interactions=10_000_000)
ML100K = dict(num_users=943, num_items=1_682, num_interactions=55_375)


@dataclass
class SyntheticSplit:
    num_users: int
    num_items: int
    train_u: np.ndarray
    train_i: np.ndarray
    valid_u: np.ndarray
    valid_i: np.ndarray
    test_u: np.ndarray
    test_i: np.ndarray
    pool_u: np.ndarray
    pool_i: np.ndarray
    item_popularity: np.ndarray


def _user_counts(rs, U, N, min_count=5):
    raw = rs.lognormal(0.0, 1.0, U)
    c = np.maximum(min_count, np.floor(raw / raw.sum() * N)).astype(np.int64)
    # fix the total to exactly N, taking from / giving to the heaviest users
    diff = N - int(c.sum())
    order = np.argsort(-c, kind="stable")
    k = 0
    while diff != 0:
        j = order[k % U]
        step = 1 if diff > 0 else -1
        if c[j] + step >= min_count:
            c[j] += step
            diff -= step
        k += 1
    return c


def make_implicit_dataset(num_users, num_items, num_interactions, seed=0, zipf_s=1.0):
    """Returns (user_ids, item_ids, timestamps) as int64 arrays."""
    rs = np.random.RandomState(seed)
    counts = _user_counts(rs, num_users, num_interactions)
    users = np.repeat(np.arange(num_users, dtype=np.int64), counts)
    w = 1.0 / np.power(np.arange(1, num_items + 1, dtype=np.float64), zipf_s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    ranks = np.searchsorted(cdf, rs.random_sample(num_interactions), side="right")
    ranks = np.minimum(ranks, num_items - 1)
    perm = rs.permutation(num_items)
    items = perm[ranks].astype(np.int64)
    ts = rs.permutation(num_interactions).astype(np.int64)
    return users, items, ts


def time_split(users, items, ts, test_percentage):
    """spotlight/dataset_manilupation.py:177-236 on distinct timestamps."""
    idx = np.argsort(ts, kind="stable")
    cut = int((1.0 - test_percentage) * len(ts))
    a, b = idx[:cut], idx[cut:]
    return (users[a], items[a], ts[a]), (users[b], items[b], ts[b])


def movielens_like(shape=ML20M, seed=0, zipf_s=1.0, pool_seed=None):
    U, I, N = shape["num_users"], shape["num_items"], shape["num_interactions"]
    u, i, t = make_implicit_dataset(U, I, N, seed=seed, zipf_s=zipf_s)
    (tu, ti, tt), (su, si, _) = time_split(u, i, t, 0.1)
    (tu, ti, _), (vu, vi, _) = time_split(tu, ti, tt, 0.1)
    prs = np.random.RandomState(seed + 1 if pool_seed is None else pool_seed)
    pool_u = prs.randint(0, U, len(tu)).astype(np.int64)
    pool_i = prs.randint(0, I, len(tu)).astype(np.int64)
    pop = np.bincount(i, minlength=I).astype(np.int64)
    return SyntheticSplit(U, I, tu, ti, vu, vi, su, si, pool_u, pool_i, pop)
