"""Dataset splits and slate construction (spotlight/dataset_manilupation.py of the
reference; the module keeps the reference's spelling so imports carry over).

Same functions and semantics: random / user-hash / time-based splits of
Interactions, row deletion from CSR matrices, and ``create_slates`` (each user's
last n interactions by time become the target slate and leave the history; users
with fewer than n interactions lose theirs; all-zero slate rows are dropped),
vectorised over users instead of one ``np.where`` per user."""
import numpy as np
from scipy.sparse import coo_matrix, csr_matrix
from sklearn.utils import murmurhash3_32

from .interactions import Interactions


def _index_or_none(array, index):
    return None if array is None else array[index]


def _subset(inter, index):
    return Interactions(inter.user_ids[index], inter.item_ids[index],
                        ratings=_index_or_none(inter.ratings, index),
                        timestamps=_index_or_none(inter.timestamps, index),
                        weights=_index_or_none(inter.weights, index),
                        num_users=inter.num_users, num_items=inter.num_items)


def shuffle_interactions(interactions, random_state=None):
    """dataset_manilupation.py:20-55: one RandomState.shuffle of the row order."""
    random_state = random_state if random_state is not None else np.random.RandomState()
    order = np.arange(len(interactions.user_ids))
    random_state.shuffle(order)
    return _subset(interactions, order)


def random_train_test_split(interactions, test_percentage=0.2, random_state=None):
    """:57-111: shuffle, then the first (1 - p) fraction is train."""
    inter = shuffle_interactions(interactions, random_state=random_state)
    cut = int((1.0 - test_percentage) * len(inter))
    return _subset(inter, slice(None, cut)), _subset(inter, slice(cut, None))


def user_based_train_test_split(interactions, test_percentage=0.2, random_state=None):
    """:113-175: users hashed (murmur3, seed from the RandomState) into test with
    probability p, so a user's whole history lands on one side."""
    random_state = random_state if random_state is not None else np.random.RandomState()
    seed = random_state.randint(np.iinfo(np.uint32).min, np.iinfo(np.uint32).max, dtype=np.int64)
    in_test = (murmurhash3_32(interactions.user_ids, seed=seed, positive=True) % 100 / 100.0) < test_percentage
    return _subset(interactions, np.logical_not(in_test)), _subset(interactions, in_test)


def train_test_timebased_split(interactions, test_percentage=0.2):
    """:177-236: sort by timestamp (the input is re-ordered in place, as the reference
    does), the earliest (1 - p) fraction is train."""
    order = interactions.timestamps.argsort()
    interactions.user_ids = interactions.user_ids[order]
    interactions.item_ids = interactions.item_ids[order]
    interactions.timestamps = interactions.timestamps[order]
    # ratings / weights are not re-ordered (as in the reference, :203-208)
    cut = int((1.0 - test_percentage) * len(interactions))
    return _subset(interactions, slice(None, cut)), _subset(interactions, slice(cut, None))


def delete_rows_csr(mat, row_indices=[], col_indices=[]):
    """:238-268: drop rows / columns of a CSR matrix (indices of the kept axis reset)."""
    if not isinstance(mat, csr_matrix):
        raise ValueError("works only for CSR format -- use .tocsr() first")
    rows, cols = list(row_indices), list(col_indices)
    if rows:
        keep = np.ones(mat.shape[0], dtype=bool)
        keep[rows] = False
        mat = mat[keep]
    if cols:
        keep = np.ones(mat.shape[1], dtype=bool)
        keep[cols] = False
        mat = mat[:, keep]
    return mat


def create_slates(interactions, n=5, padding_value=0):
    """:270-316.  Returns (history CSR without the slates' rows, slates (users, n)):
    per user with >= n interactions the last n by timestamp (argsort order) form the
    slate and are removed; users with fewer lose all their interactions; users whose
    slate row is all zeros are removed from both outputs."""
    U = interactions.num_users
    slates = np.zeros((U, n))
    uid, ts = interactions.user_ids, interactions.timestamps
    order = np.lexsort((ts, uid))                     # by user, then time
    su = uid[order]
    starts = np.searchsorted(su, np.arange(U + 1))
    counts = np.diff(starts)
    delete = np.zeros(len(uid), dtype=bool)
    short = counts < n
    # users with 0 < count < n: every interaction deleted
    delete[order[short[su]]] = True
    full = np.flatnonzero(counts >= n)
    if len(full):
        last = (starts[full + 1][:, None] - n + np.arange(n)[None, :])     # positions of the last n
        idx = order[last]
        slates[full] = interactions.item_ids[idx]
        delete[idx.ravel()] = True
    keep = np.logical_not(delete)
    interactions.user_ids = interactions.user_ids[keep]
    interactions.item_ids = interactions.item_ids[keep]
    interactions.timestamps = interactions.timestamps[keep]
    if interactions.ratings is not None:
        interactions.ratings = interactions.ratings[keep]
    zero = np.flatnonzero(~slates.any(axis=1))
    slates = np.delete(slates, zero, axis=0)
    return delete_rows_csr(interactions.tocsr(), row_indices=list(zero)), slates


def train_test_split(interactions, test_percentage=0.2):
    """:318-360: per user, int(p * count) test items drawn (with replacement) by the
    global np.random; dense, as the reference (small datasets only)."""
    dense = np.asarray(interactions.tocsr().todense())
    test = np.zeros(dense.shape)
    train = dense.copy()
    for user in range(dense.shape[0]):
        nz = dense[user, :].nonzero()[0]
        pick = np.random.choice(nz, int(nz.shape[0] * test_percentage))
        train[user, pick] = 0
        test[user, pick] = dense[user, pick]
    assert np.all(np.multiply(train, test) == 0)
    tr, te = coo_matrix(train), coo_matrix(test)
    mk = lambda c: Interactions(c.row, c.col, c.data, num_users=dense.shape[0], num_items=dense.shape[1])  # noqa
    return mk(tr), mk(te)
