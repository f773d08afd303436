"""Negative pool (spotlight/sampling.py:46-70 of the reference).

``get_negative_samples(train, n)`` draws exactly what the reference draws from
NumPy's global legacy generator -- ``np.random.choice(U, n)``, then
``np.random.choice(I, n)``, then, in index order, one
``np.random.randint(0, I - len(pos_u), 1)`` for every pair whose raw rating is 1
(``has_key``), remapped past the user's positives by binary search
(sampling.py:37-44) -- in native code (rg_pool_build, rg_pool.cpp) that continues and
stores back NumPy's generator state, and returns a ``NegativePool`` (two int64 arrays
that behave like the reference's list of (user, item) tuples) instead of n Python
tuples."""
import ctypes
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
    """The pool, drawn by rg_pool_build (native, librg_hip.so) from NumPy's global legacy
    generator, whose state it continues and stores back."""
    from .. import _lib
    num_items, num_users = train.num_items, train.num_users
    logging.info("Generating %d Samples" % num_samples)
    start = time.time()
    csr = train.csr_matrix.tocsr(copy=True)
    csr.sum_duplicates()
    csr.sort_indices()
    indptr = np.ascontiguousarray(csr.indptr, dtype=np.int64)
    indices = np.ascontiguousarray(csr.indices, dtype=np.int32)
    ratings = np.ascontiguousarray(csr.data, dtype=np.float32)
    name, key, pos, has_gauss, cached = np.random.get_state(legacy=True)
    key = np.array(key, dtype=np.uint32)
    mt_pos = np.array([pos], dtype=np.int32)
    users = np.empty(num_samples, dtype=np.int64)
    items = np.empty(num_samples, dtype=np.int64)
    c = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    has = csr.nnz > 0
    lib = _lib.load()
    rc = lib.rg_pool_build(c(key), c(mt_pos), int(num_samples), int(num_users), int(num_items),
                           c(indptr) if has else None, c(indices) if has else None, c(ratings) if has else None,
                           c(users), c(items))
    np.random.set_state((name, key, int(mt_pos[0]), has_gauss, cached))
    if rc != 0:
        msg = lib.rg_last_error().decode(errors="replace")
        if "no negative" in msg:    # the reference's np.random.randint(0, 0) -> ValueError
            raise ValueError("high <= 0: " + msg)
        _lib.check(rc, "rg_pool_build")
    logging.info("Took %d seconds" % (time.time() - start))
    return NegativePool(users, items)
