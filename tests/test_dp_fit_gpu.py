"""Data-parallel ``ImplicitFactorizationModel.fit`` (the additive ``world_size``): two ranks at
batch B, owner-sharded (mf_engine.MFEngine dp="owner"), reproduce one process at batch 2B --
which is itself pinned to the reference's own fit (tests/test_dropin_gpu.py).

Two processes share cuda:0 with a gloo group (RCCL cannot put two ranks on one device), so
the exchanges run through torch.distributed (``train_step_owner_exchange``); the RCCL path of
the same native parts is covered by tests/test_dp_gpu.py.  Checked: summary.csv losses 1e-5,
best epoch, the module-level ``random`` state after fit (every training and validation draw)
bit-exact, the gathered best tables by tensor parity, predict(3)."""
import csv
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import mf as omf

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fit(z, loss, batch, world, workdir):
    from recommendation_gans_amd.implicit import ImplicitFactorizationModel
    from recommendation_gans_amd.spotlight import optimizers
    from recommendation_gans_amd.spotlight.factorization.representations import BilinearNet
    from recommendation_gans_amd.spotlight.interactions import Interactions
    U, I, d, _, n = (int(x) for x in z["meta"])
    train = Interactions(z["train_u"].astype(np.int32), z["train_i"].astype(np.int32),
                         ratings=np.ones(len(z["train_u"]), np.float32), num_users=U, num_items=I)
    valid = Interactions(z["valid_u"].astype(np.int32), z["valid_i"].astype(np.int32),
                         ratings=np.ones(len(z["valid_u"]), np.float32), num_users=U, num_items=I)
    pool = list(zip(z["pool_u"].tolist(), z["pool_i"].tolist()))
    net = BilinearNet(U, I, d)
    with torch.no_grad():
        net.user_embeddings.weight.copy_(torch.from_numpy(z["pointwise_init_U"]))
        net.item_embeddings.weight.copy_(torch.from_numpy(z["pointwise_init_I"]))
    random.seed(0)
    os.chdir(workdir)
    model = ImplicitFactorizationModel(loss=loss, embedding_dim=d, n_iter=2, batch_size=batch, l2=1e-5,
                                       learning_rate=1e-2, optimizer_func=optimizers.adam_optimizer,
                                       representation=net, random_state=np.random.RandomState(0),
                                       neg_examples=pool, num_negative_samples=n, use_cuda=True,
                                       world_size=world)
    model.fit(train, valid)
    summary = None
    path = os.path.join(model.experiment_logs, "summary.csv")
    if os.path.exists(path):
        summary = [[float(x) for x in row] for row in list(csv.reader(open(path)))[1:]]
    return (summary, model.best_epoch, [t.detach().cpu().clone() for t in model.best_model],
            np.array(random.getstate()[1], np.uint32), model.predict(3))


def _worker(rank, world, port, loss, batch, workdir, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = np.load(os.path.join(ROOT, "tests", "golden", "mf_fit_golden.npz"))
        os.makedirs(os.path.join(workdir, f"r{rank}"), exist_ok=True)
        out[rank] = _fit(z, loss, batch, world, os.path.join(workdir, f"r{rank}"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("loss", ["pointwise", "hinge"])
def test_fit_world2_equals_single_process_at_2B(tmp_path, loss):
    z = np.load(os.path.join(ROOT, "tests", "golden", "mf_fit_golden.npz"))
    B = int(z["meta"][3])
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(2, _free_port(), loss, B, str(tmp_path), out), nprocs=2, join=True)
    os.makedirs(tmp_path / "ref", exist_ok=True)
    cwd = os.getcwd()
    try:
        ref = _fit(z, loss, 2 * B, 1, str(tmp_path / "ref"))
    finally:
        os.chdir(cwd)
    ref_summary, ref_best, ref_tables, ref_state, ref_pred = ref
    assert out[0][0] is not None and out[1][0] is None, "rank 0 writes summary.csv, rank 1 does not"
    np.testing.assert_allclose(out[0][0], ref_summary, rtol=1e-5)
    for r in range(2):
        summary, best, tables, state, pred = out[r]
        assert best == ref_best
        assert (state == ref_state).all(), (r, "random state after fit")
        for k, (t, rt) in enumerate(zip(tables, ref_tables)):
            ok, msg = omf.tensor_parity(t.reshape(rt.shape), rt, rtol=1e-5)
            assert ok, (r, k, msg)
        np.testing.assert_allclose(pred, ref_pred, rtol=1e-5, atol=1e-7)
