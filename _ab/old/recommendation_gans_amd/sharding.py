"""User-sharded data parallelism for the MF training step (host-side partition).

The reference trains on one device (implicit.py:238-345); this is the multi-GPU
layout of the same step, one process per GPU:

* user u is owned by rank ``u % R`` and lives there as local row ``u // R`` --
  its embedding row, bias, optimizer state, its training positives (kept in the
  order of the reference's one-time shuffle, implicit.py:262) and the negative-pool
  entries whose user it is (kept in pool order; the pool is uniform over
  (user, item) pairs, spotlight/sampling.py:46-70, so each rank's sub-pool is
  uniform over its own users);
* the item table is replicated; the item gradient is the only exchange (RCCL
  all-reduce, ``rg_mf_stepper_train`` with a communicator);
* rank r draws its negatives with ``random.choices`` semantics (implicit.py:352)
  from its own CPython MT19937 stream: rank 0 continues the caller's stream (so
  R = 1 is exactly the reference), rank r > 0 a stream seeded from it and r;
* loss means run over every rank's positives / negatives of the step.

With R = 1 every function here is the identity.
"""
import hashlib
import random

import numpy as np

from . import _mtstate


def owner(users, world):
    return np.asarray(users, dtype=np.int64) % world


def local_ids(users, world):
    return np.asarray(users, dtype=np.int64) // world


def global_ids(local, rank, world):
    return np.asarray(local, dtype=np.int64) * world + rank


def num_local_users(num_users, rank, world):
    return (num_users - rank + world - 1) // world


def shard_rows(table, rank, world):
    """Rows of a (num_users, ...) table owned by ``rank`` (local row order)."""
    return table[rank::world]


def unshard_rows(shards, num_users):
    """Inverse of shard_rows over all ranks: shards[r] holds rows r, r+R, ..."""
    world = len(shards)
    first = np.asarray(shards[0])
    out = np.empty((num_users,) + first.shape[1:], dtype=first.dtype)
    for r, s in enumerate(shards):
        out[r::world] = np.asarray(s)
    return out


def shard_interactions(users, items, rank, world):
    """This rank's (local user, item) positives in the given (already shuffled) order."""
    users = np.asarray(users, dtype=np.int64)
    keep = owner(users, world) == rank
    return local_ids(users[keep], world), np.asarray(items, dtype=np.int64)[keep]


def shard_pool(pool_u, pool_i, rank, world):
    """This rank's sub-pool (local user ids), pool order preserved."""
    return shard_interactions(pool_u, pool_i, rank, world)


def rank_mt_state(state0, rank):
    """625-word CPython MT state of ``rank``'s negative stream: rank 0 continues
    ``state0`` itself; rank r > 0 is ``random.seed(int)`` (init_by_array) with a
    seed hashed from state0 and r, so streams are fixed by the run's seed alone."""
    state0 = np.asarray(state0, dtype=np.uint32)
    if rank == 0:
        return state0.copy()
    digest = hashlib.sha256(state0.tobytes() + int(rank).to_bytes(4, "little")).digest()
    rnd = random.Random(int.from_bytes(digest, "little"))
    return _mtstate.from_python(rnd.getstate())


def steps_per_epoch(shard_sizes, batch_size):
    """Every rank runs the same number of steps (a collective per step): the
    largest shard's batch count; shorter shards run empty trailing steps."""
    return max((n + batch_size - 1) // batch_size for n in shard_sizes)


def batch_counts(shard_sizes, batch_size, step):
    """Positives of every rank in ``step`` (for global loss denominators)."""
    return [max(0, min(batch_size, n - step * batch_size)) for n in shard_sizes]
