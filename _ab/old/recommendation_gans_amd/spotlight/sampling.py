"""Negative pool (spotlight/sampling.py:46-70 of the reference).

``get_negative_samples(train, n)`` draws exactly what the reference draws from
NumPy's global legacy generator -- ``np.random.choice(U, n)``, then
``np.random.choice(I, n)``, then, in index order, one
``np.random.randint(0, I - len(pos_u), 1)`` for every pair whose raw rating is 1
(``has_key``), remapped past the user's positives by binary search
(sampling.py:37-44) -- but vectorised, and returns a ``NegativePool`` (two int64
arrays that behave like the reference's list of (user, item) tuples) instead of
n Python tuples."""
import logging
import time

import numpy as np


class NegativePool:
    """Sequence of (user, item) pairs backed by two arrays."""

    def __init__(self, user_ids, item_ids):
        self.user_ids = np.ascontiguousarray(user_ids, dtype=np.int64)
        self.item_ids = np.ascontiguousarray(item_ids, dtype=np.int64)
        if self.user_ids.shape != self.item_ids.shape:
            raise ValueError("pool user and item arrays differ in length")

    def __len__(self):
        return len(self.user_ids)

    def __getitem__(self, k):
        if isinstance(k, slice):
            return NegativePool(self.user_ids[k], self.item_ids[k])
        return (int(self.user_ids[k]), int(self.item_ids[k]))

    def __iter__(self):
        return zip(self.user_ids.tolist(), self.item_ids.tolist())

    @staticmethod
    def from_pairs(pairs):
        """Accepts a NegativePool, a (users, items) pair of arrays or a sequence of tuples."""
        if isinstance(pairs, NegativePool):
            return pairs
        if isinstance(pairs, tuple) and len(pairs) == 2 and hasattr(pairs[0], "__len__") \
                and not np.isscalar(pairs[0]) and len(pairs[0]) != 2:
            return NegativePool(pairs[0], pairs[1])
        a = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
        return NegativePool(a[:, 0], a[:, 1])


def sample_items(interaction, user_ids, num_items, shape, random_state=None):
    """Uniform item ids (sampling.py:9-35)."""
    if random_state is None:
        random_state = np.random.RandomState()
    return random_state.randint(0, num_items, shape, dtype=np.int64)


def get_negative_samples(train, num_samples):
    num_items, num_users = train.num_items, train.num_users
    logging.info("Generating %d Samples" % num_samples)
    start = time.time()
    users = np.random.choice(num_users, num_samples)
    items = np.random.choice(num_items, num_samples)
    csr = train.csr_matrix
    if csr.nnz:
        hit = np.flatnonzero(np.asarray(csr[users, items]).ravel() == 1)
        for k in hit:                       # in index order, as the reference loop draws
            pos = np.sort(csr[users[k], :].toarray().nonzero()[1])
            raw = np.random.randint(0, num_items - len(pos), size=1)
            adj = pos - np.arange(len(pos))
            items[k] = raw[0] + np.searchsorted(adj, raw[0], side="right")
    logging.info("Took %d seconds" % (time.time() - start))
    return NegativePool(users, items)
