"""oracle/rng.py -- TEST INFRASTRUCTURE ONLY.

ctypes front-end for oracle/rng.c plus the glue between Python's
``random.getstate()`` tuple and the flat 625-word MT state (624 words + position)
that the C restatement and the product's device sampler both use.

Reference call sites restated here:
  * implicit.py:352 / :370  ``random.choices(self.neg_examples, k=n*batch_size)``
  * mf_spotlight.py:36      ``np.random.RandomState(0)``
  * implicit.py:146         ``set_seed(self._random_state.randint(-10**8, 10**8))``
  * implicit.py:262         ``shuffle(user_ids, item_ids, random_state)`` (torch_utils.py:38-55)
  * spotlight/sampling.py:46-70  ``get_negative_samples`` (np.random.choice x2 + has_key)
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_rng.so")
_lib = None


def build():
    """Compile oracle/rng.c with gcc (recipe: oracle/Makefile)."""
    subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle_rng.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or (
                os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "rng.c"))):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
        L.orc_mt_next.argtypes = [u32p]
        L.orc_mt_next.restype = ctypes.c_uint32
        L.orc_mt_init_genrand.argtypes = [u32p, ctypes.c_uint32]
        L.orc_mt_init_by_array.argtypes = [u32p, u32p, ctypes.c_int64]
        L.orc_py_random.argtypes = [u32p]
        L.orc_py_random.restype = ctypes.c_double
        L.orc_py_choices.argtypes = [u32p, ctypes.c_int64, ctypes.c_int64, i64p]
        L.orc_np_randint.argtypes = [u32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, i64p]
        L.orc_np_randint.restype = ctypes.c_int
        L.orc_np_shuffle_i64.argtypes = [u32p, i64p, ctypes.c_int64]
        _lib = L
    return _lib


# ---------------------------------------------------------------- state glue
def state_from_python(py_state):
    """random.getstate() -> np.uint32[625] (624 words + position)."""
    version, internal, gauss = py_state
    assert version == 3 and len(internal) == 625, "unexpected random.getstate() layout"
    return np.asarray(internal, dtype=np.uint32).copy()


def state_to_python(state, gauss_next=None):
    """np.uint32[625] -> tuple accepted by random.setstate()."""
    return (3, tuple(int(x) for x in state), gauss_next)


def py_seed_state(seed):
    """CPython random.seed(int) -> 625-word state."""
    s = abs(int(seed))
    key = []
    while True:
        key.append(s & 0xFFFFFFFF)
        s >>= 32
        if s == 0:
            break
    st = np.zeros(625, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    lib().orc_mt_init_by_array(st, k, len(key))
    return st


def np_seed_state(seed):
    """NumPy legacy RandomState(seed) -> 625-word state."""
    st = np.zeros(625, dtype=np.uint32)
    lib().orc_mt_init_genrand(st, int(seed) & 0xFFFFFFFF)
    return st


def state_from_numpy(rs):
    """np.random.RandomState -> 625-word state (copy)."""
    d = rs.get_state(legacy=False)
    st = np.zeros(625, dtype=np.uint32)
    st[:624] = d["state"]["key"]
    st[624] = d["state"]["pos"]
    return st


# ---------------------------------------------------------------- draws
def py_choices_indices(state, n, k):
    """Indices drawn by random.choices(pop, k) with len(pop) == n; advances state in place."""
    out = np.empty(int(k), dtype=np.int64)
    lib().orc_py_choices(state, int(n), int(k), out)
    return out


def np_randint(state, low, high, size):
    out = np.empty(int(size), dtype=np.int64)
    rc = lib().orc_np_randint(state, int(low), int(high), int(size), out)
    if rc != 0:
        raise ValueError("orc_np_randint: unsupported range")
    return out


def np_shuffle_indices(state, n):
    x = np.arange(int(n), dtype=np.int64)
    lib().orc_np_shuffle_i64(state, x, int(n))
    return x


def negative_pool(state, num_users, num_items, num_samples, positive_csr=None):
    """spotlight/sampling.py:46-70 get_negative_samples.

    ``users = np.random.choice(U, n); items = np.random.choice(I, n)``; a pair
    whose raw-rating CSR entry equals 1 (``Interactions.has_key``,
    spotlight/interactions.py:159-160) has its item replaced by
    ``negsamp_vectorized_bsearch_preverif`` (sampling.py:37-44), which draws one
    more ``np.random.randint(0, I - len(pos))`` from the same stream.
    ``positive_csr`` is a scipy CSR of the raw ratings (or None when no entry can
    equal 1, the normal case after make_implicit -- SURVEY.md §0.4).
    Returns int64 arrays (users, items).
    """
    users = np_randint(state, 0, num_users, num_samples)
    items = np_randint(state, 0, num_items, num_samples)
    if positive_csr is None:
        return users, items
    items = items.copy()
    for t in range(num_samples):
        u, i = int(users[t]), int(items[t])
        if positive_csr[u, i] == 1:
            row = positive_csr[u, :].toarray().nonzero()[1]
            raw = int(np_randint(state, 0, num_items - len(row), 1)[0])
            adj = row - np.arange(len(row))
            items[t] = raw + int(np.searchsorted(adj, raw, side="right"))
    return users, items
