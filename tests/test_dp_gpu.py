"""Data-parallel MF steps on the GPU, through the HIP C-ABI.

Replicated / global stream (the default layout, reference-exact):
* world 2 on one GPU: two processes share cuda:0, each runs MFEngine(dp="global_stream")
  natively in two halves (rg_mf_stepper_dp_begin / _dp_end) around gloo collectives on
  the device buffers -- the rank-major gradient reduce-scatter and the table all-gather
  (RCCL cannot place two ranks on one device);
* world 1 with an RCCL communicator: the whole native step (rg_mf_stepper_train ->
  ncclReduceScatter / ncclAllGather);
both against the single-process oracle at batch world*B: negative ids and MT state
bit-exact, losses within 1e-5, tables by tensor parity (fp32 and fp64 restatements).

User-sharded (opt-in, not the reference's sampling at R > 1):
* world 2 on one GPU with gloo (``train_step_sharded``) and world 1 with RCCL
  (item_grad + comm), against the global-view restatement (tests/dp_common.py)."""
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


def _ab_only(needed):
    """The sharded item update and the MT rank slices were measured slower or equal:
    the A/B build carries them (scripts/gpu_ab_tests.sh)."""
    from recommendation_gans_amd import _lib
    if needed and not _lib.ab_build():
        pytest.skip("A/B build only (RG_LIB=recommendation_gans_amd/_variants/librg_hip_ab.so)")


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


def _gs_engine(rank, world, loss, comm=None):
    from recommendation_gans_amd.mf_engine import MFEngine
    tables, pool_u, pool_i, train_u, train_i, state0 = dc.problem()
    e = MFEngine(tables[0], tables[1], tables[2].reshape(-1), tables[3].reshape(-1), pool_u, pool_i, state0.copy(),
                 loss=loss, optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=dc.N_NEG, batch_size=dc.B,
                 device="cuda:0", rank=rank, world_size=world, dp="global_stream", comm=comm)
    tu = torch.from_numpy(train_u.astype(np.int64)).cuda()
    ti = torch.from_numpy(train_i.astype(np.int64)).cuda()
    inputs = []
    for k, (a, b, gp) in enumerate(dc.rank_columns(world, rank)):
        plan = e.make_plan(ti[a:b]) if (k % 2 == 1 and b > a) else None    # odd steps with a plan
        inputs.append((e.step_input(tu[a:b], ti[a:b], gp, plan), plan is not None))
    return e, inputs


def _gs_collect(e, inputs, rank, step_fn):
    losses, states, negs = [], [], []
    for k, (cur, planned) in enumerate(inputs):
        nxt = inputs[k + 1][0] if k + 1 < len(inputs) else None
        lv = step_fn(cur, nxt)
        losses.append(float(lv[0]))
        states.append(e.mt_state())
        S = 8                                                    # pair_stride(5)
        if planned:
            negs.append(None)
        else:                                                    # the buffer this step consumed
            pr = e.pairs[k % 2].view(dc.B, S, 2)[:, 1:1 + dc.N_NEG].transpose(0, 1).cpu().numpy() & 0x07FFFFFF
            negs.append((pr[..., 0], pr[..., 1]))
    torch.cuda.synchronize()
    return [p.cpu().clone() for p in e.params()], losses, states, negs


def _worker_gs_gloo(rank, world, port, loss, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e, inputs = _gs_engine(rank, world, loss)

        def reduce_scatter(buf, chunk):          # every chunk summed; this rank reads its own
            dist.all_reduce(buf)

        def all_gather(bufs, counts):
            for b, c in zip(bufs, counts):
                flat = b.view(-1)
                full = torch.zeros_like(flat)
                full[rank * c:(rank + 1) * c] = flat[rank * c:(rank + 1) * c]
                dist.all_reduce(full)
                flat.copy_(full)

        out[rank] = _gs_collect(e, inputs, rank,
                                lambda cur, nxt: e.train_step_exchange(cur, nxt, reduce_scatter, all_gather))
    finally:
        dist.destroy_process_group()


def _worker_gs_rccl(rank, world, port, loss, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommendation_gans_amd.comm import RcclComm
        comm = RcclComm("cuda:0")
        e, inputs = _gs_engine(rank, world, loss, comm=comm)
        out[rank] = _gs_collect(e, inputs, rank, lambda cur, nxt: e.train_step_in(cur, nxt))
        del e
        comm.close()
    finally:
        dist.destroy_process_group()


def _gs_check(out, world, loss):
    tables, pool_u, pool_i, train_u, train_i, state0 = dc.problem()
    o, ref_losses, ref_states, ref_negs = dc.reference_run(tables, pool_u, pool_i, train_u, train_i, state0, world,
                                                           loss)
    o64, _, _, _ = dc.reference_run(tables, pool_u, pool_i, train_u, train_i, state0, world, loss,
                                    dtype=torch.float64)
    for r in range(world):
        params, losses, states, negs = out[r]
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
        for s in range(len(ref_losses)):
            assert (states[s] == ref_states[s]).all(), (r, s, "MT state")
            if negs[s] is not None:
                cols = slice(r * dc.B, (r + 1) * dc.B)
                assert (negs[s][0] == ref_negs[s][0][:, cols]).all(), (r, s, "negative users")
                assert (negs[s][1] == ref_negs[s][1][:, cols]).all(), (r, s, "negative items")
        for k in range(4):
            ok, msg = omf.tensor_parity(params[k].reshape(o.params[k].shape), o.params[k], o64.params[k])
            assert ok, (r, k, msg)
    if world > 1:
        assert all(torch.equal(a, b) for a, b in zip(out[0][0], out[1][0])), "replicas diverged"


@pytest.mark.parametrize("loss", ["pointwise", "bpr"])
def test_global_stream_engine_gloo_world2(loss):
    """Two ranks at batch B (native halves, gloo collectives) == one process at batch 2B."""
    out = mp.Manager().dict()
    mp.spawn(_worker_gs_gloo, args=(2, _free_port(), loss, out), nprocs=2, join=True)
    _gs_check(out, 2, loss)


def test_global_stream_native_rccl_world1():
    """The whole native replicated step with its RCCL reduce-scatter / all-gather."""
    out = mp.Manager().dict()
    mp.spawn(_worker_gs_rccl, args=(1, _free_port(), "bpr", out), nprocs=1, join=True)
    _gs_check(out, 1, "bpr")


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
    """User-sharded opt-in layout against its own restatement."""
    out = mp.Manager().dict()
    mp.spawn(_worker_gloo, args=(2, _free_port(), loss, out), nprocs=2, join=True)
    _check(out, 2, loss)


def test_native_rccl_step_world1():
    out = mp.Manager().dict()
    mp.spawn(_worker_rccl, args=(1, _free_port(), "bpr", out), nprocs=1, join=True)
    assert torch.equal(out[0][3], torch.arange(5, dtype=torch.float32))
    _check(out, 1, "bpr")


# ------------------------------------------------------------------ owner-sharded (default at R > 1)
def _own_engine(rank, world, loss, comm=None):
    from recommendation_gans_amd.mf_engine import MFEngine
    tables, pool_u, pool_i, train_u, train_i, state0 = dc.problem()
    e = MFEngine(tables[0], tables[1], tables[2].reshape(-1), tables[3].reshape(-1), pool_u, pool_i, state0.copy(),
                 loss=loss, optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=dc.N_NEG, batch_size=dc.B,
                 device="cuda:0", rank=rank, world_size=world, dp="owner", comm=comm)
    tu = torch.from_numpy(train_u[:dc.GS_TRAIN].astype(np.int64)).cuda()
    ti = torch.from_numpy(train_i[:dc.GS_TRAIN].astype(np.int64)).cuda()
    plans = e.make_plans(ti, users=tu)
    inputs = [e.step_input(tu[lo:hi], ti[lo:hi], hi - lo, plans[g])
              for g, (lo, hi) in enumerate(dc.global_batches(world))]
    return e, inputs


def _own_collect(e, inputs, step_fn):
    losses, states, recs = [], [], []
    for k, cur in enumerate(inputs):
        nxt = inputs[k + 1] if k + 1 < len(inputs) else None
        lv = step_fn(cur, nxt)
        losses.append(float(lv[0]))
        states.append(e.mt_state())
        counts = e.owner_seg[k % 2].cpu().numpy()
        rec = e.owner_rec[k % 2].view(-1, 256, 4).cpu().numpy()
        recs.append(np.concatenate([rec[s, :counts[s], :3] for s in range(len(counts))]))
    torch.cuda.synchronize()
    return [p.cpu().clone() for p in e.params()], losses, states, recs


def _worker_own_gloo(rank, world, port, loss, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e, inputs = _own_engine(rank, world, loss)
        out[rank] = _own_collect(e, inputs, lambda cur, nxt: e.train_step_owner_exchange(cur, nxt, dist.all_reduce))
    finally:
        dist.destroy_process_group()


def _worker_own_rccl(rank, world, port, loss, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommendation_gans_amd.comm import RcclComm
        comm = RcclComm("cuda:0")
        e, inputs = _own_engine(rank, world, loss, comm=comm)
        out[rank] = _own_collect(e, inputs, lambda cur, nxt: e.train_step_in(cur, nxt))
        del e
        comm.close()
    finally:
        dist.destroy_process_group()


def _worker_own_host(rank, world, port, loss, out, item_shard="0"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RG_OWNER_ITEM_SHARD=item_shard)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommendation_gans_amd.comm import HostComm
        comm = HostComm("cuda:0")
        e, inputs = _own_engine(rank, world, loss, comm=comm)
        assert e.shard_items == (-(-e.I // world) if item_shard == "1" else 0)

        def step(cur, nxt):
            lv = e.train_step_in(cur, nxt)
            comm.sync()            # the exchanges' host callbacks need the GIL: wait in a ctypes call
            return lv
        out[rank] = _own_collect(e, inputs, step)
        comm.sync()
        del e
        comm.close()
    finally:
        dist.destroy_process_group()


def _own_check(out, world, loss):
    """R owner-sharded ranks at batch B == one process at batch R*B (the oracle): losses 1e-5,
    MT state and every negative's ids bit-exact (each valid draw kept by exactly the rank
    owning its user), tables by tensor parity after unsharding the user rows."""
    tables, pool_u, pool_i, train_u, train_i, state0 = dc.problem()
    o, ref_losses, ref_states, ref_negs = dc.reference_run(tables, pool_u, pool_i, train_u, train_i, state0, world,
                                                           loss)
    o64, _, _, _ = dc.reference_run(tables, pool_u, pool_i, train_u, train_i, state0, world, loss,
                                    dtype=torch.float64)
    GC = dc.B * world
    batches = dc.global_batches(world)
    for s, (lo, hi) in enumerate(batches):
        seen = np.zeros((dc.N_NEG, GC), np.int64)
        for r in range(world):
            rec = out[r][3][s]
            k1, c = rec[:, 0] // GC, rec[:, 0] % GC
            assert (k1 >= 1).all()
            users = rec[:, 1].astype(np.int64) * world + r
            assert (users == ref_negs[s][0][k1 - 1, c]).all(), (r, s, "negative users")
            assert (rec[:, 2] == ref_negs[s][1][k1 - 1, c]).all(), (r, s, "negative items")
            np.add.at(seen, (k1 - 1, c), 1)
        valid_cols = GC if loss in ("pointwise", "adaptive_hinge") else hi - lo
        assert (seen[:, :valid_cols] == 1).all() and (seen[:, valid_cols:] == 0).all(), (s, "draw ownership")
    for r in range(world):
        params, losses, states, _ = out[r]
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
        for s in range(len(ref_losses)):
            assert (states[s] == ref_states[s]).all(), (r, s, "MT state")
        for k in (1, 3):
            ok, msg = omf.tensor_parity(params[k].reshape(o.params[k].shape), o.params[k], o64.params[k])
            assert ok, (r, k, msg)
    for k in (0, 2):
        full = torch.from_numpy(sharding.unshard_rows([out[r][0][k].numpy() for r in range(world)], dc.U))
        ok, msg = omf.tensor_parity(full.reshape(o.params[k].shape), o.params[k], o64.params[k])
        assert ok, (k, msg)
    if world > 1:
        assert torch.equal(out[0][0][1], out[1][0][1]), "replicated items diverged"


@pytest.mark.parametrize("loss", ["pointwise", "bpr", "hinge", "adaptive_hinge"])
def test_owner_engine_gloo_world2(loss):
    """Two owner-sharded ranks at batch B (native parts, gloo all-reduces) == one process at 2B."""
    out = mp.Manager().dict()
    mp.spawn(_worker_own_gloo, args=(2, _free_port(), loss, out), nprocs=2, join=True)
    _own_check(out, 2, loss)


def test_owner_native_rccl_world1():
    """The whole native owner-sharded step with its two RCCL all-reduces."""
    out = mp.Manager().dict()
    mp.spawn(_worker_own_rccl, args=(1, _free_port(), "bpr", out), nprocs=1, join=True)
    _own_check(out, 1, "bpr")


@pytest.mark.parametrize("loss,item_shard", [("bpr", "0"), ("adaptive_hinge", "0"), ("bpr", "1"),
                                              ("adaptive_hinge", "1")])
def test_owner_native_concurrent_step_world2(loss, item_shard):
    _ab_only(item_shard == "1")
    """The whole native owner step (rg_mf_stepper_train, train_owner's stream placement: the score
    all-reduce and the item-gradient all-reduce on the main stream, where RCCL takes them; the
    user update and the next owner prepare on the communicator stream beside the item exchange
    and update) at world 2 -- two processes on cuda:0, each all-reduce host-staged through gloo
    on the main stream in stream order (comm.HostComm: D2H, host callback, H2D on the caller's
    stream, as RCCL would be enqueued; RCCL refuses two ranks on one GPU) -- == one process at
    batch 2B.  item_shard "1" (RG_OWNER_ITEM_SHARD): the item update sharded -- reduce-scatter of the
    rank-major item gradient, each rank's half of the items' Adam, all-gather of the item rows and
    biases (host-staged as all-reduces of the chunks) -- with the same result."""
    out = mp.Manager().dict()
    mp.spawn(_worker_own_host, args=(2, _free_port(), loss, out, item_shard), nprocs=2, join=True)
    _own_check(out, 2, loss)



# ------------------------------------------------------------------ owner step: MT word slices
def _worker_own_slices(rank, world, port, loss, slice_flag, out):
    """Rank `rank` of the owner step with a host-staged communicator at a batch where one rank's
    slice of a step's words (2 n B) is longer than a jump's stream window, RG_OWNER_MT_SLICE as
    given; per step the loss and the exported CPython MT state, at the end the tables."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RG_OWNER_MT_SLICE=slice_flag,
                      RG_MT_UNITS="2")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import rng as orng
        from recommendation_gans_amd.comm import HostComm
        from recommendation_gans_amd.mf_engine import MFEngine
        comm = HostComm("cuda:0")
        U, I, d, B, n, steps = 5000, 700, 32, 4096, 5, 5
        rs = np.random.RandomState(3)
        torch.manual_seed(3)
        Uw, Iw = torch.empty(U, d).normal_(0, 1.0 / d), torch.empty(I, d).normal_(0, 1.0 / d)
        pool_u, pool_i = rs.randint(0, U, 60000), rs.randint(0, I, 60000)
        e = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), pool_u, pool_i, orng.py_seed_state(3), loss=loss,
                     optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B, device="cuda:0",
                     rank=rank, world_size=world, dp="owner", comm=comm)
        gb = B * world
        tu = torch.from_numpy(rs.randint(0, U, (steps + 1) * gb).astype(np.int64)).cuda()
        ti = torch.from_numpy(np.minimum(rs.zipf(1.3, (steps + 1) * gb) - 1, I - 1).astype(np.int64)).cuda()
        plans = e.make_plans(ti, users=tu)
        ins = [e.step_input(tu[g * gb:(g + 1) * gb], ti[g * gb:(g + 1) * gb], gb, plans[g]) for g in range(steps + 1)]
        losses, states = [], []
        for s in range(steps):
            lv = e.train_step_in(ins[s], ins[s + 1])
            comm.sync()
            losses.append(float(lv[0]))
            states.append(e.mt_state())
        comm.sync()
        out[rank] = ([p.cpu().clone() for p in e.params()], losses, states, e.mt_mode == 2)
        del e
        comm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("loss", ["bpr", "pointwise"])
def test_owner_mt_slices_match_the_full_walk(loss):
    _ab_only(True)
    """The owner step's MT words by rank slices (each rank walks 2 n B of every step's 2 n R B words
    and jumps the rest; the slices all-gathered; the exported state advanced by a jump per slot)
    against every rank walking the whole global draw (RG_OWNER_MT_SLICE=0): per-step losses, the
    exported CPython MT state after every step, and the tables, bit for bit, at world 2 over a
    host-staged communicator, across several word slots (RG_MT_UNITS=2)."""
    res = {}
    for flag in ("1", "0"):
        out = mp.Manager().dict()
        mp.spawn(_worker_own_slices, args=(2, _free_port(), loss, flag, out), nprocs=2, join=True)
        res[flag] = dict(out)
    for r in range(2):
        ps, ls, ss, sl = res["1"][r]
        pf, lf, sf, fl = res["0"][r]
        assert sl and not fl, (r, "slice mode on / off as asked")
        assert ls == lf, (r, ls, lf)
        for s in range(len(ss)):
            assert (ss[s] == sf[s]).all(), (r, s, "MT state")
        for k in range(4):
            assert torch.equal(ps[k], pf[k]), (r, k)
