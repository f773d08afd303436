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


RG_MT_PAD = 1280   # include/rg_hip.h: words rg_mt_generate may write past the requested count


def sample_items(interaction, user_ids, num_items, shape, random_state=None, device=None):
    """Uniform item ids (sampling.py:9-35): ``random_state.randint(0, num_items, shape)``.

    ``device`` (additive): draw on that GPU instead (``sample_items_device``) and return an
    int64 tensor there; the values and the generator state afterwards are NumPy's."""
    if random_state is None:
        random_state = np.random.RandomState()
    if device is not None:
        return sample_items_device(num_items, shape, random_state, device)
    return random_state.randint(0, num_items, shape, dtype=np.int64)


def sample_items_device(num_items, shape, random_state=None, device="cuda"):
    """NumPy legacy ``RandomState.randint(0, num_items, shape)`` on the GPU, bit-exact, with
    ``random_state`` advanced exactly as NumPy advances it: the MT19937 words are generated
    from the RandomState's (key, pos) state (rg_mt_generate) and NumPy's masked rejection
    runs as an ordered compaction (rg_uniform_int64); the words the draw consumed advance
    the host state (rg_mt_advance_host).  Returns an int64 tensor of ``shape`` on
    ``device``."""
    import torch
    from .. import _lib
    if random_state is None:
        random_state = np.random.RandomState()
    num_items = int(num_items)
    if num_items <= 0:
        raise ValueError("high <= 0")
    if num_items - 1 > 0xFFFFFFFF:
        raise ValueError("sample_items_device: num_items above 2^32 is not supported")
    shape = (shape,) if np.isscalar(shape) else tuple(shape)
    n = int(np.prod(shape, dtype=np.int64))
    out = torch.zeros(n, dtype=torch.int64, device=device)
    if n == 0 or num_items == 1:   # NumPy draws no words for a one-value range
        return out.reshape(shape)
    lib = _lib.load()
    name, key, pos, has_gauss, gauss = random_state.get_state()
    state = np.empty(625, np.uint32)
    state[:624] = key
    state[624] = pos
    rng = num_items - 1
    mask = (1 << int(rng).bit_length()) - 1
    nwords = int(n * (mask + 1) / (rng + 1) * 1.05) + 4096   # expected words + margin
    stream = _lib.stream_handle(torch.cuda.current_stream(device))
    consumed = torch.zeros(1, dtype=torch.int64, device=device)
    while True:
        st = torch.from_numpy(state.view(np.int32).copy()).to(device)
        words = torch.empty(nwords + RG_MT_PAD, dtype=torch.int32, device=device)
        _lib.check(lib.rg_mt_generate(stream, _lib.ptr(st), _lib.ptr(words), nwords, None), "rg_mt_generate")
        scratch = torch.empty(int(lib.rg_uniform_scratch_len(nwords)) + 2, dtype=torch.int32, device=device)
        _lib.check(lib.rg_uniform_int64(stream, _lib.ptr(words), nwords, 0, num_items, n, _lib.ptr(out),
                                        _lib.ptr(scratch), _lib.ptr(consumed)), "rg_uniform_int64")
        c = int(consumed.item())
        if c > 0:
            break
        nwords *= 2   # fewer accepted words than outputs (far tail): redraw from the same state
    host = state.copy()
    _lib.check(lib.rg_mt_advance_host(host.ctypes.data, c), "rg_mt_advance_host")
    random_state.set_state((name, host[:624].copy(), int(host[624]), has_gauss, gauss))
    return out.reshape(shape)


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
