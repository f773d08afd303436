"""Shared pieces of the data-parallel tests (CPU gloo and GPU).

``global_view`` restates the user-sharded step (recommendation_gans_amd/sharding.py)
on the GLOBAL tables with the oracle's primitives: every rank's positives and
draws (its own MT stream over its own sub-pool, mapped back to global user ids)
contribute gradients with loss means over all ranks; one optimizer step.  The
sharded runs must reproduce it."""
import numpy as np
import torch

from oracle import mf as omf
from oracle import rng as orng
from recommendation_gans_amd import sharding

U, I, D, B, N_NEG, STEPS = 37, 23, 8, 8, 5, 3


def problem(seed=0):
    g = torch.Generator().manual_seed(seed)
    tables = [torch.randn(U, D, generator=g) / D, torch.randn(I, D, generator=g) / D,
              torch.randn(U, 1, generator=g) * 0.01, torch.randn(I, 1, generator=g) * 0.01]
    rs = np.random.RandomState(seed)
    pool_u, pool_i = rs.randint(0, U, 300), rs.randint(0, I, 300)
    train_u, train_i = rs.randint(0, U, 400), rs.randint(0, I, 400)
    return tables, pool_u, pool_i, train_u, train_i, orng.py_seed_state(seed)


def rank_batches(train_u, train_i, rank, world, steps=STEPS, batch=B):
    lu, li = sharding.shard_interactions(train_u, train_i, rank, world)
    return [(lu[s * batch:(s + 1) * batch], li[s * batch:(s + 1) * batch]) for s in range(steps)]


def global_view(tables, pool_u, pool_i, train_u, train_i, state0, world, loss, optimizer="adam",
                lr=1e-2, wd=1e-5, steps=STEPS, dtype=torch.float32):
    params = [t.clone().to(dtype) for t in tables]
    opt = omf.Optim(optimizer, params, lr, wd)
    states = [sharding.rank_mt_state(state0, r) for r in range(world)]
    pools = [sharding.shard_pool(pool_u, pool_i, r, world) for r in range(world)]
    batches = [rank_batches(train_u, train_i, r, world, steps) for r in range(world)]
    losses = []
    for s in range(steps):
        P = sum(len(batches[r][s][0]) for r in range(world))
        den = (P, N_NEG * B * world)
        total = [torch.zeros_like(p) for p in params]
        lsum = 0.0
        for r in range(world):
            lu, li = batches[r][s]
            pu = torch.from_numpy(sharding.global_ids(lu, r, world))
            pi = torch.from_numpy(np.asarray(li, np.int64))
            idx = orng.py_choices_indices(states[r], len(pools[r][0]), N_NEG * B)
            nu = torch.from_numpy(sharding.global_ids(pools[r][0][idx], r, world))
            ni = torch.from_numpy(np.asarray(pools[r][1][idx], np.int64))
            Uw, Iw, ub, ib = params
            p_pos = omf.scores(Uw, Iw, ub, ib, pu, pi)
            p_neg = omf.scores(Uw, Iw, ub, ib, nu, ni)
            lv, dpp, dpn = omf.loss_and_dp(loss, p_pos, p_neg, N_NEG, B, den=den)
            dz = torch.cat([dpp * (1 - p_pos) * p_pos, dpn * (1 - p_neg) * p_neg])
            gr = omf.dense_grads(Uw, Iw, ub, ib, torch.cat([pu, nu]), torch.cat([pi, ni]), dz)
            total = [a + b for a, b in zip(total, gr)]
            lsum += float(lv)
        opt.step(params, total)
        losses.append(lsum)
    return params, losses, states
