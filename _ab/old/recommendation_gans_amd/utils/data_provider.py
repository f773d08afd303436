"""Dataset provider (utils/data_provider.py:18-178 of the reference).

``data_provider(path, variant, negative_per_positive, movies_to_keep=-1)`` loads
the reference's cache files when present -- ``movielens_<V>_{train,valid,test}_<k>.csv``
(userId,movieId,rating,timestamp), ``_popularity_<k>.csv``, ``_statistics_<k>.json``
and the negative pool ``_ngt_<k>.npz`` (arrays ``user_ids``/``item_ids``) or the
reference's ``_ngt_<k>.pkl`` (read by an unpickler that only admits the list /
tuple / int / NumPy-scalar objects a pool consists of).  Without them (the raw
MovieLens files cannot be fetched here), it builds synthetic data of the
variant's shape with the reference's processing order: implicit ratings, time
split 10 % test then 10 % valid (data_provider.py:77-78), pool of len(train)
pairs from NumPy's global generator (sampling.py:46-70)."""
import io
import json
import logging
import os
import pickle
import time

import numpy as np
import pandas as pd

from ..spotlight.interactions import Interactions
from ..spotlight.sampling import NegativePool, get_negative_samples
from ..synthetic import make_implicit_dataset
from .helper_functions import make_implicit

SHAPES = {"100K": (943, 1682, 55_375), "1M": (6_038, 3_533, 575_281), "10M": (69_838, 10_066, 5_005_002),
          "20M": (136_677, 20_108, 10_000_000)}


class _PoolUnpickler(pickle.Unpickler):
    _ALLOWED = {("numpy", "dtype"), ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"negative pool file may not reference {module}.{name}")


def read_pool(path):
    if path.endswith(".npz"):
        z = np.load(path, allow_pickle=False)
        return NegativePool(z["user_ids"], z["item_ids"])
    with open(path, "rb") as f:
        pairs = _PoolUnpickler(io.BufferedReader(f)).load()
    return NegativePool.from_pairs(pairs)


def time_split(interactions, test_percentage):
    """train_test_timebased_split (spotlight/dataset_manilupation.py:177-236)."""
    order = interactions.timestamps.argsort()
    cut = int((1.0 - test_percentage) * len(interactions))
    cols = [interactions.user_ids[order], interactions.item_ids[order], interactions.ratings[order],
            interactions.timestamps[order]]
    mk = lambda sl: Interactions(*(c[sl] for c in cols[:2]), ratings=cols[2][sl], timestamps=cols[3][sl],
                                 num_users=interactions.num_users, num_items=interactions.num_items)
    return mk(slice(None, cut)), mk(slice(cut, None))


class data_provider:
    def __init__(self, path, variant, negative_per_positive, movies_to_keep=-1, synthetic=None, zipf=1.0,
                 seed=0):
        self.movies_to_keep = movies_to_keep
        rel = os.path.join(path, "movielens_" + variant)
        tag = "_" + str(movies_to_keep)
        start = time.time()
        have_cache = all(os.path.exists(rel + s + tag + ".csv") for s in ("_train", "_valid", "_test", "_popularity"))
        pool_file = next((rel + "_ngt" + tag + e for e in (".npz", ".pkl") if os.path.exists(rel + "_ngt" + tag + e)),
                         None)
        if have_cache and pool_file and not synthetic:
            logging.info("Data exists, loading from file ... ")
            stats = json.load(open(rel + "_statistics" + tag + ".json"))
            sets = [self._interactions(pd.read_csv(rel + s + tag + ".csv"), stats["num_users"], stats["num_items"])
                    for s in ("_train", "_valid", "_test")]
            train, valid, test = [make_implicit(s) for s in sets]
            item_popularity = pd.read_csv(rel + "_popularity" + tag + ".csv", header=None).iloc[:, 1]
            neg = read_pool(pool_file)
        else:
            if synthetic is False:
                raise FileNotFoundError(f"dataset cache {rel}{tag}*.csv / _ngt file not found")
            if variant not in SHAPES:
                raise ValueError(f"unknown MovieLens variant {variant!r}")
            logging.info("Dataset cache absent: synthetic MovieLens-%s-shaped data", variant)
            U, I, N = SHAPES[variant]
            u, i, t = make_implicit_dataset(U, I, N, seed=seed, zipf_s=zipf)
            dataset = Interactions(u, i, ratings=np.full(N, 4.0), timestamps=t, num_users=U, num_items=I)
            dataset = make_implicit(dataset)
            train, test = time_split(dataset, 0.1)
            train, valid = time_split(train, 0.1)
            neg = get_negative_samples(dataset, len(train))
            item_popularity = pd.Series(np.bincount(i, minlength=I))
        logging.info("Took %d seconds" % (time.time() - start))
        logging.info("{} user and {} items".format(train.num_users, train.num_items))
        self.config = {"train_set": train, "valid_set": valid, "test_set": test,
                       "item_popularity": item_popularity, "neg_examples": neg}

    @staticmethod
    def _interactions(df, num_users, num_items):
        return Interactions(df.userId.values, df.movieId.values, df.rating.values, df.timestamp.values,
                            num_users=num_users, num_items=num_items)

    def get_timebased_data(self):
        c = self.config
        return c["train_set"], c["valid_set"], c["test_set"], c["neg_examples"], c["item_popularity"]
