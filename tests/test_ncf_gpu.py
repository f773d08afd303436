"""NCF MLP step on the GPU (rg_ncf.hip through the C-ABI) against the reference's
own NCF steps (tests/golden/mlp_*.npz, dropout masks recorded from the reference
and fed to the kernel): loss, MT stream, and every parameter after each Adam
step (tensor parity vs the fp32 reference; small tensors vs the fp64 restatement
as in oracle.mf.tensor_parity)."""
import os

import numpy as np
import pytest
import torch

from oracle import mf as omf
from oracle import ncf as oncf

pytestmark = pytest.mark.gpu

CASES = ["mlp_pointwise_e16", "mlp_pointwise_e64", "mlp_adaptive_hinge_e16", "mlp_bpr_e16"]


def masks_for(z, s, nl, B, n, dev):
    def cat(kind, rows):
        m = np.concatenate([z[f"s{s}_mask_{kind}{k}"] for k in range(nl)], axis=1)
        out = np.zeros((rows, m.shape[1]), np.uint8)
        out[:m.shape[0]] = m
        return torch.from_numpy(out).to(dev).contiguous()
    return cat("pos", B), cat("neg", n * B)


@pytest.mark.parametrize("case", CASES)
def test_ncf_steps_match_reference(golden_dir, case):
    from recommendation_gans_amd.ncf_engine import NCFEngine
    dev = torch.device("cuda:0")
    z = np.load(os.path.join(golden_dir, case + ".npz"))
    names = [str(x) for x in z["param_names"]]
    init = [torch.from_numpy(z["init_" + nm.replace(".", "_")].copy()) for nm in names]
    U, I, E, B, n = (int(x) for x in z["meta"])
    loss = case.split("_e")[0][len("mlp_"):]
    nl = len(z["layers"]) - 1
    e = NCFEngine(init[0], init[1], init[2:], z["pool_u"], z["pool_i"], z["s0_mt_state"].copy(), loss=loss,
                  optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
    o64 = oncf.NCFOracle([t.double() for t in init], names, z["pool_u"], z["pool_i"], z["s0_mt_state"].copy(),
                         loss=loss, lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    for s in range(3):
        pu = torch.from_numpy(z[f"s{s}_pos_u"]).to(dev)
        pi = torch.from_numpy(z[f"s{s}_pos_i"]).to(dev)
        masks = masks_for(z, s, nl, B, n, dev)
        got = e.train_step(pu, pi, masks=masks)
        mp = [torch.from_numpy(z[f"s{s}_mask_pos{k}"]) for k in range(nl)]
        mn = [torch.from_numpy(z[f"s{s}_mask_neg{k}"]) for k in range(nl)]
        o64.step(z[f"s{s}_pos_u"], z[f"s{s}_pos_i"], mp, mn)
        torch.cuda.synchronize()
        np.testing.assert_allclose(float(got[0]), float(z[f"s{s}_loss"][0]), rtol=1e-5, err_msg=f"{case} loss {s}")
        assert (e.mt_state() == (z[f"s{s + 1}_mt_state"] if s < 2 else z["end_mt_state"])).all(), f"{case} MT {s}"
        params = [e.user_w, e.item_w] + e.mlp_params()
        for nm, p, r64 in zip(names, params, o64.P.t):
            ref = torch.from_numpy(z[f"s{s}_after_" + nm.replace(".", "_")])
            ok, msg = omf.tensor_parity(p.reshape(ref.shape), ref, r64.reshape(ref.shape))
            assert ok, f"{case} step {s} {nm}: {msg}"
    assert int(e.row_count.abs().sum()) == 0 and float(e.hot_grad.abs().sum()) == 0.0


def test_ncf_device_dropout_trains():
    """Device dropout RNG: bit-reproducible for a seed -- these tiny tables overflow the
    per-row lists on every step, and the overflow accumulators are int64 fixed point (sums
    independent of the atomics' order) while list entries are summed in sorted order, so
    two runs agree exactly; and a fixed batch's loss falls."""
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from oracle import rng as orng
    dev = torch.device("cuda:0")
    U, I, E, B, n = 400, 300, 64, 512, 5
    torch.manual_seed(0)
    sizes = oncf.layer_sizes(E)
    params = [torch.randn(U, E), torch.randn(I, E)]
    for a_, b_ in zip(sizes[:-1] + [sizes[-1]], sizes[1:] + [1]):
        w = torch.empty(b_, a_)
        torch.nn.init.xavier_uniform_(w)
        params += [w, torch.full((b_,), 0.01)]
    rs = np.random.RandomState(0)
    pool_u, pool_i = rs.randint(0, U, 5000), rs.randint(0, I, 5000)
    pu, pi = torch.from_numpy(rs.randint(0, U, B)).to(dev), torch.from_numpy(rs.randint(0, I, B)).to(dev)
    losses = []
    for rep in range(2):
        e = NCFEngine(params[0], params[1], params[2:], pool_u, pool_i, orng.py_seed_state(0), loss="pointwise",
                      lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev, seed=7)
        ls = [float(e.train_step(pu, pi, plan=e.make_plan(pi))[0]) for _ in range(6)]
        losses.append(ls)
        assert all(np.isfinite(ls))
    assert losses[0] == losses[1], (losses[0], losses[1])
    assert losses[0][-1] < losses[0][0]


def test_prefetched_negatives_leave_the_trajectory_unchanged():
    """rg_mf_stepper_prefetch (next step's negatives prepared during this step's updates)
    draws the same negatives (MT stream bit-exact) and gives the unprefetched trajectory
    bit for bit: a row's listed contributions are summed in sorted order and the overflow in
    fixed point (round 2), so where the negatives were prepared cannot change a sum."""
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from oracle import rng as orng
    dev = torch.device("cuda:0")
    U, I, E, B, n = 40000, 30000, 16, 256, 5
    torch.manual_seed(1)
    sizes = oncf.layer_sizes(E)
    params = [torch.randn(U, E), torch.randn(I, E)]
    for a_, b_ in zip(sizes[:-1] + [sizes[-1]], sizes[1:] + [1]):
        w = torch.empty(b_, a_)
        torch.nn.init.xavier_uniform_(w)
        params += [w, torch.full((b_,), 0.01)]
    rs = np.random.RandomState(2)
    pool_u, pool_i = rs.randint(0, U, 40000), rs.randint(0, I, 40000)
    batches = [(torch.from_numpy(rs.choice(U, B, replace=False)).to(dev),
                torch.from_numpy(rs.choice(I, B, replace=False)).to(dev)) for _ in range(5)]
    out = []
    # mode 0: no prefetch; 1: the next step's batch prefetched; 2: a wrong batch prefetched
    # (the next acquire sees another input and prepares again)
    for mode in (0, 1, 2):
        e = NCFEngine(params[0], params[1], params[2:], pool_u, pool_i, orng.py_seed_state(4), loss="pointwise",
                      lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev, seed=3)
        plans = [e.make_plan(b[1]) for b in batches]
        ls = []
        for s, (u, i) in enumerate(batches):
            nxt = None
            if mode and s + 1 < len(batches):
                k = s + 1 if mode == 1 else 0
                nxt = (batches[k][0], batches[k][1], plans[k])
            ls.append(float(e.train_step(u, i, plan=plans[s], next_step=nxt)[0]))
        out.append((ls, [t.detach().cpu().clone() for t in e.params()], e.mt_state()))
    for m in (1, 2):
        assert (out[0][2] == out[m][2]).all()
        assert out[m][0] == out[0][0], (m, out[m][0], out[0][0])
        for a, b in zip(out[0][1], out[m][1]):
            assert torch.equal(a, b), (m, float((a - b).abs().max()))


@pytest.mark.parametrize("loss,optimizer,E,M,U,I", [("pointwise", "adam", 64, 0, 400, 300),
                                                    ("bpr", "adam", 64, 0, 40000, 30000),
                                                    ("adaptive_hinge", "sgd", 16, 0, 3000, 2000),
                                                    ("pointwise", "adam", 16, 50, 40000, 30000),
                                                    ("hinge", "rms", 32, 20, 60, 25)])
def test_fused_tail_matches_the_separate_calls(loss, optimizer, E, M, U, I):
    """rg_ncf_tail (the next step's prepare, the MLP update with the loss, the embedding update
    and, when due, the MT walk in one launch; NeuMF's GMF pass before it) against the calls it
    replaces (rg_ncf_update, rg_ncf_apply / rg_neumf_apply, rg_mf_stepper_prefetch_inline, the
    generator-stream walk): losses, every parameter and the MT state bit for bit over steps with
    and without a prefetched next batch -- small tables (every row's list overflows) and large
    ones (mostly single contributions); NCF towers (M = 0) and NeuMF (M > 0)."""
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from oracle import rng as orng
    dev = torch.device("cuda:0")
    B, n, steps = 512, 5, 4
    torch.manual_seed(5)
    sizes = oncf.layer_sizes(E)
    params = [torch.randn(U, E) / E, torch.randn(I, E) / E]
    extra = {}
    if M:
        extra = dict(mf_user_w=torch.randn(U, M) / M, mf_item_w=torch.randn(I, M) / M)
    for a_, b_ in zip(sizes[:-1] + [sizes[-1] + M], sizes[1:] + [1]):
        w = torch.empty(b_, a_)
        torch.nn.init.xavier_uniform_(w)
        params += [w, torch.full((b_,), 0.01)]
    rs = np.random.RandomState(6)
    pool_u, pool_i = rs.randint(0, U, 20000), rs.randint(0, I, 20000)
    batches = [(torch.from_numpy(rs.randint(0, U, B)).to(dev), torch.from_numpy(rs.randint(0, I, B)).to(dev))
               for _ in range(steps)]
    out = []
    for fused in (True, False):
        e = NCFEngine(params[0], params[1], params[2:], pool_u, pool_i, orng.py_seed_state(8), loss=loss,
                      optimizer=optimizer, lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev, seed=9,
                      **extra)
        e.fused_tail = fused
        plans = [e.make_plan(b[1]) for b in batches]
        ls = []
        for s, (u, i) in enumerate(batches):
            # steps 0 and 2 hand over the next batch (prepared in the tail), 1 and 3 do not
            nxt = (batches[s + 1][0], batches[s + 1][1], plans[s + 1]) if s % 2 == 0 else None
            ls.append(float(e.train_step(u, i, plan=plans[s], next_step=nxt)[0]))
        torch.cuda.synchronize()
        out.append((ls, [t.detach().cpu().clone() for t in e.params()], e.mt_state()))
    assert out[0][0] == out[1][0], (out[0][0], out[1][0])
    assert all(np.isfinite(out[0][0]))
    assert (out[0][2] == out[1][2]).all()
    for k, (a, b) in enumerate(zip(out[0][1], out[1][1])):
        assert torch.equal(a, b), (k, float((a - b).abs().max()))


def test_ncf_rejects_the_positives_only_loss(tmp_path, monkeypatch):
    """RG_LOSS_POINTWISE_POS (neg_examples=None, implemented for BilinearNet only) is refused by
    the NCF engine, and the drop-in refuses it before building any engine (round-3 advisor)."""
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from recommendation_gans_amd.implicit import ImplicitFactorizationModel
    from recommendation_gans_amd.spotlight.dnn_models.mlp import MLP
    from recommendation_gans_amd.spotlight.interactions import Interactions
    from oracle import rng as orng
    monkeypatch.chdir(tmp_path)                 # the drop-in writes experiments_results/ under the cwd
    dev = torch.device("cuda:0")
    U, I, E = 40, 30, 8
    sizes = oncf.layer_sizes(E)
    params = [torch.randn(U, E), torch.randn(I, E)]
    for a_, b_ in zip(sizes[:-1] + [sizes[-1]], sizes[1:] + [1]):
        params += [torch.zeros(b_, a_), torch.zeros(b_)]
    with pytest.raises(ValueError):
        NCFEngine(params[0], params[1], params[2:], np.zeros(4, np.int64), np.zeros(4, np.int64),
                  orng.py_seed_state(0), loss="pointwise_pos", n_neg=5, batch_size=16, device=dev)
    rs = np.random.RandomState(0)
    train = Interactions(rs.randint(0, U, 200), rs.randint(0, I, 200), num_users=U, num_items=I)
    net = MLP(layers=[2 * E, E], num_users=U, num_items=I, embedding_dim=E)
    m = ImplicitFactorizationModel(representation=net, n_iter=1, batch_size=16, use_cuda=True, neg_examples=None)
    with pytest.raises(NotImplementedError):
        m.fit(train, train)
