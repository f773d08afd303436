"""make_implicit (utils/helper_functions.py:7-26 of the reference): ratings > 3.5 -> 1, else 0."""
import numpy as np


def make_implicit(interactions):
    interactions.ratings = (np.asarray(interactions.ratings) > 3.5).astype(np.int64)
    return interactions
