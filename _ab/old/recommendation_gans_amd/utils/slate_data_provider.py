"""Slate dataset provider for the cGAN (utils/slate_data_provider.py:20-328 of the
reference).

``slate_data_provider(path, variant, slate_size, min_movies, min_viewers,
movies_to_keep)`` with ``get_data()`` returning the reference's 9-tuple
(train_vec, train_slates, test_vec, test_set, num_users, num_items, valid_vec,
val_vec_cold_start, valid_set) and ``get_cold_start_users()``.

* Cache: the reference's files ``<S>_slate_movielens_<V>{_train_vec,_test_vec,
  _valid_vec,_train_cold_start,_val_cold_start,_test_set,_valid_set}_<k>``,
  ``_train_slates_<k>.pkl`` and ``_statistics_<k>.json`` load through an unpickler
  that admits only NumPy arrays and SciPy CSR matrices (what those files hold).
* Otherwise (the raw MovieLens files cannot be fetched here) synthetic data of the
  variant's shape go through the reference's pipeline (:97-150): time split 10 %
  test, then 10 % validation; ``create_slates`` on the training part; histories
  padded with N (``preprocess_train``); the validation future split 80/20 by time
  with its cold-start users; the test histories / targets as the reference's
  intended (and, in its own build branch, commented-out) split of the test part
  (:136-145), whose active lines reference undefined names.
"""
import io
import json
import logging
import os
import pickle

import numpy as np
import torch

from ..spotlight.dataset_manilupation import create_slates, delete_rows_csr, train_test_timebased_split
from ..spotlight.interactions import Interactions
from ..synthetic import make_implicit_dataset
from .data_provider import SHAPES


class _SlateUnpickler(pickle.Unpickler):
    _ALLOWED = {("numpy", "dtype"), ("numpy", "ndarray"), ("numpy.core.multiarray", "_reconstruct"),
                ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
                ("numpy._core.multiarray", "scalar"), ("scipy.sparse._csr", "csr_matrix"),
                ("scipy.sparse.csr", "csr_matrix"), ("scipy.sparse._arrays", "csr_array")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"slate cache file may not reference {module}.{name}")


def _load(path):
    with open(path, "rb") as f:
        return _SlateUnpickler(io.BufferedReader(f)).load()


def preprocess_train(interactions, num_users, num_items):
    """slate_data_provider.py:208-234: (rows with interactions, their item lists padded
    with num_items as a float tensor, users without interactions)."""
    row, col = interactions.nonzero()
    valid_rows = np.unique(row)
    cold = np.delete(np.arange(num_users), valid_rows)
    if len(row) == 0:
        return valid_rows, torch.zeros(0, 0), cold
    starts = np.flatnonzero(np.r_[True, row[1:] != row[:-1]])
    lens = np.diff(np.r_[starts, len(row)])
    out = np.full((len(starts), int(lens.max())), float(num_items), np.float32)
    pos = np.arange(len(row)) - np.repeat(starts, lens)
    out[np.repeat(np.arange(len(starts)), lens), pos] = col
    return valid_rows, torch.from_numpy(out), cold


def synthetic_slate_data(num_users, num_items, num_interactions, slate_size, seed=0, zipf_s=1.0):
    u, i, t = make_implicit_dataset(num_users, num_items, num_interactions, seed=seed, zipf_s=zipf_s)
    dataset = Interactions(u.astype(np.int32), i.astype(np.int32), ratings=np.ones(len(u), np.float32),
                           timestamps=t.astype(np.int64), num_users=num_users, num_items=num_items)
    U, N = num_users, num_items
    train_set, test_set = train_test_timebased_split(dataset, test_percentage=0.1)
    train_set, valid_set = train_test_timebased_split(train_set, test_percentage=0.1)
    train_split, train_slates = create_slates(train_set, n=slate_size, padding_value=N)
    valid_rows, train_vec, _ = preprocess_train(train_split, train_split.shape[0], N)
    train_slates = np.delete(train_slates, np.delete(np.arange(train_split.shape[0]), valid_rows), axis=0)
    # validation: earliest 80 % of the validation part is the history, the rest the target
    valid_history, valid_future = train_test_timebased_split(valid_set, test_percentage=0.2)
    valid_future = valid_future.tocsr()
    val_rows, valid_vec, valid_cold = preprocess_train(valid_history.tocsr(), U, N)
    val_vec_cold_start = valid_future[valid_cold, :]
    valid_set = delete_rows_csr(valid_future, row_indices=list(np.delete(np.arange(U), val_rows)))
    # test: the same split of the test part
    test_history, test_future = train_test_timebased_split(test_set, test_percentage=0.2)
    test_future = test_future.tocsr()
    test_rows, test_vec, test_cold = preprocess_train(test_history.tocsr(), U, N)
    test_vec_cold_start = test_future[test_cold, :]
    test_set = delete_rows_csr(test_future, row_indices=list(np.delete(np.arange(U), test_rows)))
    return dict(train_vec=train_vec, test_vec=test_vec, valid_vec=valid_vec, test_vec_cold_start=test_vec_cold_start,
                val_vec_cold_start=val_vec_cold_start, train_slates=train_slates, test_set=test_set,
                valid_set=valid_set, num_items=N, num_user=U)


class slate_data_provider:
    def __init__(self, path, variant, slate_size=3, min_movies=0, min_viewers=5, movies_to_keep=-1,
                 synthetic=None, zipf=1.0, seed=0):
        rel = path + str(slate_size) + "_slate_movielens_" + variant
        self.slate_size, self.min_movies, self.min_viewers, self.movies_to_keep = (slate_size, min_movies,
                                                                                 min_viewers, movies_to_keep)
        k = "_" + str(movies_to_keep)
        if synthetic is not True and self.exists(rel, movies_to_keep):
            logging.info("Data exists, loading from file ... ")
            with open(rel + "_statistics" + k + ".json") as f:
                self.statistics = json.load(f)
            self.config = {
                "train_slates": np.asarray(_load(rel + "_train_slates" + k + ".pkl")),
                "test_set": _load(rel + "_test_set" + k), "valid_set": _load(rel + "_valid_set" + k),
                "test_vec_cold_start": _load(rel + "_train_cold_start" + k),
                "val_vec_cold_start": _load(rel + "_val_cold_start" + k),
                "train_vec": torch.Tensor(_load(rel + "_train_vec" + k)),
                "test_vec": torch.Tensor(_load(rel + "_test_vec" + k)),
                "valid_vec": torch.Tensor(_load(rel + "_valid_vec" + k)),
                "num_items": self.statistics["num_items"], "num_user": self.statistics["num_users"]}
        else:
            if synthetic is False:
                raise FileNotFoundError(f"slate cache files {rel}_* not found (and --synthetic False)")
            if variant not in SHAPES:
                raise ValueError(f"unknown MovieLens variant {variant!r}; one of {sorted(SHAPES)}")
            U, I, Nint = SHAPES[variant]
            logging.info("Slate cache not found: synthetic MovieLens-%s-shaped data (%d users, %d items)", variant,
                         U, I)
            self.config = synthetic_slate_data(U, I, Nint, slate_size, seed=seed, zipf_s=zipf)
            self.statistics = {"num_users": U, "num_items": I, "interactions": Nint}
        logging.info("{} user and {} items".format(self.statistics["num_users"], self.statistics["num_items"]))

    @staticmethod
    def exists(rel, k="-1"):
        return all(os.path.exists(rel + s + "_" + str(k)) for s in
                   ("_train_vec", "_test_vec", "_valid_vec", "_train_cold_start", "_test_set"))

    def get_cold_start_users(self):
        return self.config["test_vec_cold_start"]

    def get_data(self):
        c = self.config
        return (c["train_vec"], c["train_slates"], c["test_vec"], c["test_set"], c["num_user"], c["num_items"],
                c["valid_vec"], c["val_vec_cold_start"], c["valid_set"])
