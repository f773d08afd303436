"""The E = 64 NCF kernel (one wave per 32-row tile, rg_ncf.hip ncf_wave_kernel) on every loss
and on tile shapes other than the bench's: BPR / hinge (pairwise, the positive's lane sums its
column), adaptive hinge (the scores phase, then the given-dp phase), pointwise, with 1 to 8
negatives (16, 8, 5, 4 or 3 columns per 32-row tile), with and without item plans, tables small
enough that hot rows overflow their per-row lists.  Two native steps with recorded dropout
masks against the oracle (oracle/ncf.py, spotlight/losses.py:20-172 + mlp.py:5-46 restated)
run in fp32 and fp64 from the same MLP(...) init: MT state bit-exact, loss 1e-5 relative,
every parameter by tensor parity (oracle.mf.tensor_parity: GPU-vs-fp64 no worse than the
fp32 restatement's own distance, as the golden and full-size NCF tests)."""
import numpy as np
import pytest
import torch

from oracle import mf as omf
from oracle import ncf as oncf
from oracle import rng as orng

pytestmark = pytest.mark.gpu

CASES = [("bpr", 5, True), ("bpr", 8, False), ("hinge", 3, True), ("adaptive_hinge", 5, True),
         ("adaptive_hinge", 1, False), ("pointwise", 1, True), ("pointwise", 7, False)]


@pytest.mark.parametrize("loss,n,planned", CASES)
def test_ncf_e64_kernel_losses_and_shapes(loss, n, planned):
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from recommendation_gans_amd.ncf_spotlight import mlp_layers
    from recommendation_gans_amd.spotlight.dnn_models.mlp import MLP
    dev = torch.device("cuda:0")
    U, I, E, B = 900, 700, 64, 600
    torch.manual_seed(3)
    net = MLP(layers=mlp_layers(E), num_users=U, num_items=I, embedding_dim=E)
    names = [k for k, _ in net.named_parameters()]
    params = [p.detach().clone() for p in net.parameters()]
    rs = np.random.RandomState(11 + n)
    pool_u, pool_i = rs.randint(0, U, 20000), rs.randint(0, I, 20000)
    mt = orng.py_seed_state(7)
    kw = dict(loss=loss, lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    e = NCFEngine(params[0], params[1], params[2:], pool_u, pool_i, mt.copy(), optimizer="adam", device=dev, **kw)
    o32 = oncf.NCFOracle([t.clone() for t in params], names, pool_u, pool_i, mt.copy(), **kw)
    o64 = oncf.NCFOracle([t.double() for t in params], names, pool_u, pool_i, mt.copy(), **kw)
    widths = oncf.layer_sizes(E)[1:]
    for s in range(2):
        # Zipf-ish positives: a few hot items and users overflow their lists
        pu = np.minimum(rs.zipf(1.3, B) - 1, U - 1).astype(np.int64)
        pi = np.minimum(rs.zipf(1.2, B) - 1, I - 1).astype(np.int64)
        mp = [torch.from_numpy((rs.rand(B, w) >= 0.5).astype(np.uint8)) for w in widths]
        mn = [torch.from_numpy((rs.rand(n * B, w) >= 0.5).astype(np.uint8)) for w in widths]
        masks = (torch.cat(mp, 1).to(dev).contiguous(), torch.cat(mn, 1).to(dev).contiguous())
        pi_d = torch.from_numpy(pi).to(dev)
        before = [t.clone() for t in o32.P.t]   # (pointwise's output bias steps from 0.01 to ~0 at init)
        got = e.train_step(torch.from_numpy(pu).to(dev), pi_d, plan=e.make_plan(pi_d) if planned else None,
                           masks=masks)
        l32 = o32.step(pu, pi, mp, mn)
        l64 = o64.step(pu, pi, mp, mn)
        torch.cuda.synchronize()
        assert abs(float(got[0]) - l32) <= 1e-5 * abs(l32) + 1e-7, (s, float(got[0]), l32, l64)
        assert (e.mt_state() == o32.state).all(), f"MT state after step {s}"
        for nm, p, r32, r64, b0 in zip(names, e.params(), o32.P.t, o64.P.t, before):
            ok, msg = omf.tensor_parity(p.reshape(r32.shape), r32, r64, before=b0)
            assert ok, f"{loss} n={n} step {s} {nm}: {msg}"
    assert int(e.row_count.abs().sum()) == 0 and float(e.hot_grad.abs().sum()) == 0.0


@pytest.mark.parametrize("loss", ["pointwise", "bpr", "hinge", "adaptive_hinge"])
def test_ncf_e64_validation_loss(loss):
    """run_val_iteration (implicit.py:366-379) through the E = 64 kernel's loss-only phase
    (eval mode: LeakyReLU without dropout) and, for adaptive hinge, its scores phase: the loss
    of a batch against a float64 eval-mode forward on the same negatives (1e-5 relative), and
    the MT stream advanced exactly as the reference's draw."""
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from recommendation_gans_amd.ncf_spotlight import mlp_layers
    from recommendation_gans_amd.spotlight.dnn_models.mlp import MLP
    dev = torch.device("cuda:0")
    U, I, E, B, n = 900, 700, 64, 700, 5
    torch.manual_seed(4)
    net = MLP(layers=mlp_layers(E), num_users=U, num_items=I, embedding_dim=E)
    params = [p.detach().clone() for p in net.parameters()]
    rs = np.random.RandomState(21)
    pool_u, pool_i = rs.randint(0, U, 20000), rs.randint(0, I, 20000)
    mt = orng.py_seed_state(9)
    e = NCFEngine(params[0], params[1], params[2:], pool_u, pool_i, mt.copy(), loss=loss, optimizer="adam",
                  lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
    P = [t.double() for t in params]

    def eval_p(u, i):
        a = torch.cat([P[0][u], P[1][i]], 1)
        for k in range(2, len(P) - 2, 2):
            z = a @ P[k].T + P[k + 1]
            a = torch.where(z > 0, z, z * 0.1)
        return torch.sigmoid(a @ P[-2].T + P[-1]).reshape(-1)
    state = mt.copy()
    for s in range(2):
        pu = torch.from_numpy(rs.randint(0, U, B))
        pi = torch.from_numpy(rs.randint(0, I, B))
        got = float(e.val_loss(pu.to(dev), pi.to(dev))[0])
        idx = torch.from_numpy(orng.py_choices_indices(state, len(pool_u), n * B)).long()
        nu, ni = torch.as_tensor(pool_u).long()[idx], torch.as_tensor(pool_i).long()[idx]
        ref, _, _ = omf.loss_and_dp(loss, eval_p(pu, pi), eval_p(nu, ni), n, B)
        torch.cuda.synchronize()
        assert abs(got - float(ref)) <= 1e-5 * abs(float(ref)), (loss, s, got, float(ref))
        assert (e.mt_state() == state).all(), f"MT state after validation batch {s}"
