"""User-sharded data-parallel MF step on the GPU, through the HIP C-ABI.

* world 2 on one GPU: two processes share cuda:0; each runs MFEngine on its user
  shard + replicated items, exchanging the item gradient with gloo
  (``train_step_sharded``) -- RCCL cannot place two ranks on one device;
* world 1 with an RCCL communicator: the native step (rg_mf_stepper_train with
  item_grad + comm) including the ncclAllReduce on the communicator stream.
Both against the global-view restatement (tests/dp_common.py), fp32 and fp64."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import mf as omf
from recommendation_gans_amd import sharding
from tests import dp_common as dc

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _engine(rank, world, loss, comm=None):
    from recommendation_gans_amd.mf_engine import MFEngine
    tables, pool_u, pool_i, train_u, train_i, state0 = dc.problem()
    pu, pi = sharding.shard_pool(pool_u, pool_i, rank, world)
    e = MFEngine(sharding.shard_rows(tables[0], rank, world), tables[1],
                 sharding.shard_rows(tables[2], rank, world).reshape(-1), tables[3].reshape(-1), pu, pi,
                 sharding.rank_mt_state(state0, rank), loss=loss, optimizer="adam", lr=1e-2, weight_decay=1e-5,
                 n_neg=dc.N_NEG, batch_size=dc.B, device="cuda:0", rank=rank, world_size=world,
                 dp="user_shard", comm=comm)
    return e, dc.rank_batches(train_u, train_i, rank, world), train_u, train_i


def _global_pos(train_u, train_i, world, s):
    return sum(len(dc.rank_batches(train_u, train_i, r, world)[s][0]) for r in range(world))


def _worker_gloo(rank, world, port, loss, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e, batches, tu, ti = _engine(rank, world, loss)
        losses = []
        for s, (lu, li) in enumerate(batches):
            lv = e.train_step_sharded(torch.from_numpy(lu).cuda(), torch.from_numpy(li).cuda(),
                                      _global_pos(tu, ti, world, s), dist.all_reduce)
            losses.append(float(lv[0]))
        torch.cuda.synchronize()
        out[rank] = ([p.cpu().clone() for p in e.params()], losses, e.mt_state())
    finally:
        dist.destroy_process_group()


def _worker_rccl(rank, world, port, loss, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommendation_gans_amd.comm import RcclComm
        comm = RcclComm("cuda:0")
        t = torch.arange(5, dtype=torch.float32, device="cuda:0")
        comm.allreduce_(t)
        e, batches, tu, ti = _engine(rank, world, loss, comm=comm)
        losses = []
        for s, (lu, li) in enumerate(batches):
            lv = e.train_step(torch.from_numpy(lu).cuda(), torch.from_numpy(li).cuda(), _global_pos(tu, ti, world, s))
            losses.append(float(lv[0]))
        torch.cuda.synchronize()
        out[rank] = ([p.cpu().clone() for p in e.params()], losses, e.mt_state(), t.cpu())
        del e
        comm.close()
    finally:
        dist.destroy_process_group()


def _check(out, world, loss):
    tables, pool_u, pool_i, train_u, train_i, state0 = dc.problem()
    ref, ref_losses, states = dc.global_view(tables, pool_u, pool_i, train_u, train_i, state0, world, loss)
    ref64, _, _ = dc.global_view(tables, pool_u, pool_i, train_u, train_i, state0, world, loss,
                                 dtype=torch.float64)
    got_u = torch.from_numpy(sharding.unshard_rows([out[r][0][0].numpy() for r in range(world)], dc.U))
    got_ub = torch.from_numpy(sharding.unshard_rows([out[r][0][2].numpy() for r in range(world)], dc.U))
    for k, got in ((0, got_u), (2, got_ub)):
        ok, msg = omf.tensor_parity(got, ref[k], ref64[k])
        assert ok, (k, msg)
    for r in range(world):
        for k in (1, 3):
            ok, msg = omf.tensor_parity(out[r][0][k], ref[k], ref64[k])
            assert ok, (r, k, msg)
        np.testing.assert_allclose(out[r][1], ref_losses, rtol=1e-5)
        assert (out[r][2] == states[r]).all(), f"rank {r} MT stream"
    if world > 1:
        assert torch.equal(out[0][0][1], out[1][0][1]), "replicated items diverged"


@pytest.mark.parametrize("loss", ["pointwise", "bpr"])
def test_sharded_engine_gloo_world2(loss):
    out = mp.Manager().dict()
    mp.spawn(_worker_gloo, args=(2, _free_port(), loss, out), nprocs=2, join=True)
    _check(out, 2, loss)


def test_native_rccl_step_world1():
    out = mp.Manager().dict()
    mp.spawn(_worker_rccl, args=(1, _free_port(), "bpr", out), nprocs=1, join=True)
    assert torch.equal(out[0][3], torch.arange(5, dtype=torch.float32))
    _check(out, 1, "bpr")
