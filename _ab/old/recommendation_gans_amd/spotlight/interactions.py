"""Interaction sets (spotlight/interactions.py:38-178 of the reference).

Same constructor, attributes, ``__len__``, ``tocoo``/``tocsr`` and ``has_key``
(which, as in the reference, compares the RAW rating stored at construction
with 1: ``interactions.py:159-160``).  Validation raises the reference's
ValueError messages (``interactions.py:136-158``)."""
import numpy as np
import scipy.sparse as sp


class Interactions:
    def __init__(self, user_ids, item_ids, ratings=None, timestamps=None, weights=None,
                 num_users=None, num_items=None):
        self.num_users = num_users or int(user_ids.max() + 1)
        self.num_items = num_items or int(item_ids.max() + 1)
        self.user_ids = user_ids
        self.item_ids = item_ids
        self.ratings = ratings
        self.timestamps = timestamps
        self.weights = weights
        self.shape = (num_users, num_items)
        self.csr_matrix = self.tocsr()      # raw ratings, kept for has_key
        self._check()

    def __repr__(self):
        return "<Interactions dataset ({} users x {} items x {} interactions)>".format(
            self.num_users, self.num_items, len(self))

    def __len__(self):
        return len(self.user_ids)

    def _check(self):
        if self.user_ids.max() >= self.num_users:
            raise ValueError("Maximum user id greater than declared number of users.")
        if self.item_ids.max() >= self.num_items:
            raise ValueError("Maximum item id greater than declared number of items.")
        n = len(self.user_ids)
        for name, value in (("item IDs", self.item_ids), ("ratings", self.ratings),
                            ("timestamps", self.timestamps), ("weights", self.weights)):
            if value is not None and len(value) != n:
                raise ValueError("Invalid {} dimensions: length must be equal to number of "
                                 "interactions".format(name))

    def has_key(self, user, item):
        return self.csr_matrix[user, item] == 1

    def tocoo(self):
        data = self.ratings if self.ratings is not None else np.ones(len(self))
        return sp.coo_matrix((data, (self.user_ids, self.item_ids)), shape=(self.num_users, self.num_items))

    def tocsr(self):
        return self.tocoo().tocsr()
