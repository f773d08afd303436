"""NeuMF step on the GPU (rg_ncf.hip with the GMF branch + rg_neumf_apply through the
C-ABI) against the reference's own NeuMF steps (tests/golden/neumf_*.npz, recorded
dropout masks fed to the kernel): loss, MT stream and every parameter after each Adam
step (tensor parity vs the fp32 reference; vs the fp64 restatement as in
oracle.mf.tensor_parity).  Larger synthetic cases cover the planned positive
partials, the per-row list overflow path of the GMF tables and both LDS placements
of the GMF rows (M <= E: inside the dX region; M > E: the tail region)."""
import os

import numpy as np
import pytest
import torch

from oracle import mf as omf
from oracle import ncf as oncf
from oracle import rng as orng

pytestmark = pytest.mark.gpu

CASES = ["neumf_pointwise_e16_m10", "neumf_bpr_e8_m5", "neumf_adaptive_hinge_e16_m12"]


def dev_masks(mp, mn, B, n, dev):
    def cat(ms, rows):
        m = torch.cat([x.to(torch.uint8) for x in ms], 1)
        out = torch.zeros(rows, m.shape[1], dtype=torch.uint8)
        out[:m.shape[0]] = m
        return out.to(dev).contiguous()
    return cat(mp, B), cat(mn, n * B)


def engine_params(e):
    return [e.user_w, e.item_w] + e.mf_w + e.mlp_params()


@pytest.mark.parametrize("case", CASES)
def test_neumf_steps_match_reference(golden_dir, case):
    from recommendation_gans_amd.ncf_engine import NCFEngine
    dev = torch.device("cuda:0")
    z = np.load(os.path.join(golden_dir, case + ".npz"))
    names = [str(x) for x in z["param_names"]]
    init = [torch.from_numpy(z["init_" + nm.replace(".", "_")].copy()) for nm in names]
    U, I, E, B, n, M = (int(x) for x in z["meta"])
    loss = case[len("neumf_"):].rsplit("_e", 1)[0]
    nl = len(z["layers"]) - 1
    e = NCFEngine(init[0], init[1], init[4:], z["pool_u"], z["pool_i"], z["s0_mt_state"].copy(), loss=loss,
                  optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev,
                  mf_user_w=init[2], mf_item_w=init[3])
    assert e.M == M and e.P == sum(t.numel() for t in init[4:])
    o64 = oncf.NeuMFOracle([t.double() for t in init], names, z["pool_u"], z["pool_i"], z["s0_mt_state"].copy(),
                           loss=loss, lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    for s in range(3):
        prev = [t.detach().cpu().clone() for t in engine_params(e)]
        mp = [torch.from_numpy(z[f"s{s}_mask_pos{k}"]) for k in range(nl)]
        mn = [torch.from_numpy(z[f"s{s}_mask_neg{k}"]) for k in range(nl)]
        got = e.train_step(torch.from_numpy(z[f"s{s}_pos_u"]).to(dev), torch.from_numpy(z[f"s{s}_pos_i"]).to(dev),
                           masks=dev_masks(mp, mn, B, n, dev))
        o64.step(z[f"s{s}_pos_u"], z[f"s{s}_pos_i"], mp, mn)
        torch.cuda.synchronize()
        np.testing.assert_allclose(float(got[0]), float(z[f"s{s}_loss"][0]), rtol=1e-5, err_msg=f"{case} loss {s}")
        assert (e.mt_state() == (z[f"s{s + 1}_mt_state"] if s < 2 else z["end_mt_state"])).all(), f"{case} MT {s}"
        for nm, p, r64, b in zip(names, engine_params(e), o64.P.t, prev):
            ref = torch.from_numpy(z[f"s{s}_after_" + nm.replace(".", "_")])
            ok, msg = omf.tensor_parity(p.reshape(ref.shape), ref, r64.reshape(ref.shape), before=b)
            assert ok, f"{case} step {s} {nm}: {msg}"
    assert int(e.row_count.abs().sum()) == 0 and float(e.mf_hot_grad.abs().sum()) == 0.0


def random_neumf(U, I, E, M, seed):
    g = torch.Generator().manual_seed(seed)
    sizes = oncf.layer_sizes(E)
    t = [torch.randn(U, E, generator=g), torch.randn(I, E, generator=g), torch.randn(U, M, generator=g),
         torch.randn(I, M, generator=g)]
    names = ["embedding_user_mlp.weight", "embedding_item_mlp.weight", "embedding_user_mf.weight",
             "embedding_item_mf.weight"]
    for k, (a_, b_) in enumerate(zip(sizes[:-1], sizes[1:])):
        t += [(torch.rand(b_, a_, generator=g) - 0.5) * (2 * (6 / (a_ + b_)) ** 0.5), torch.full((b_,), 0.01)]
        names += [f"layers.{3 * k}.weight", f"layers.{3 * k}.bias"]
    t += [(torch.rand(1, 8 + M, generator=g) - 0.5) * 0.5, torch.full((1,), 0.01)]
    names += ["affine_output.weight", "affine_output.bias"]
    return t, names


@pytest.mark.parametrize("E,M,loss,U,I", [(64, 64, "pointwise", 3000, 2000), (16, 50, "bpr", 3000, 2000),
                                          (32, 20, "pointwise", 40, 30), (8, 100, "hinge", 60, 25)])
def test_neumf_planned_and_overflow_vs_oracle(E, M, loss, U, I):
    """B = 1024 with the plan (positives' item partials), random dropout masks given to
    both sides; the small tables (U, I < 100) push most rows past the per-row list cap."""
    from recommendation_gans_amd.ncf_engine import NCFEngine
    dev = torch.device("cuda:0")
    B, n = 1024, 4
    t, names = random_neumf(U, I, E, M, seed=E + M)
    rs = np.random.RandomState(E * M)
    pool_u, pool_i = rs.randint(0, U, 20000), rs.randint(0, I, 20000)
    st = orng.py_seed_state(3)
    e = NCFEngine(t[0], t[1], t[4:], pool_u, pool_i, st.copy(), loss=loss, lr=1e-2, weight_decay=1e-5, n_neg=n,
                  batch_size=B, device=dev, mf_user_w=t[2], mf_item_w=t[3])
    o = oncf.NeuMFOracle([x.double() for x in t], names, pool_u, pool_i, st.copy(), loss=loss, lr=1e-2,
                         weight_decay=1e-5, n_neg=n, batch_size=B)
    o32 = oncf.NeuMFOracle([x.clone() for x in t], names, pool_u, pool_i, st.copy(), loss=loss, lr=1e-2,
                           weight_decay=1e-5, n_neg=n, batch_size=B)
    units = oncf.layer_sizes(E)[1:]
    for s in range(2):
        prev = [x.detach().cpu().clone() for x in engine_params(e)]
        pu_h, pi_h = rs.randint(0, U, B), rs.randint(0, I, B)
        mp = [torch.from_numpy(rs.randint(0, 2, (B, h)).astype(np.uint8)) for h in units]
        mn = [torch.from_numpy(rs.randint(0, 2, (n * B, h)).astype(np.uint8)) for h in units]
        pi = torch.from_numpy(pi_h).to(dev)
        got = e.train_step(torch.from_numpy(pu_h).to(dev), pi, plan=e.make_plan(pi), masks=dev_masks(mp, mn, B, n, dev))
        o.step(pu_h, pi_h, mp, mn)
        l32 = o32.step(pu_h, pi_h, mp, mn)
        torch.cuda.synchronize()
        np.testing.assert_allclose(float(got[0]), l32, rtol=1e-5)
        for nm, p, r32, r64, b in zip(names, engine_params(e), o32.P.t, o.P.t, prev):
            ok, msg = omf.tensor_parity(p, r32, r64, before=b)
            assert ok, f"E={E} M={M} step {s} {nm}: {msg}"
    assert int(e.row_count.abs().sum()) == 0 and float(e.mf_hot_grad.abs().sum()) == 0.0


def test_neumf_val_loss_and_device_dropout():
    from recommendation_gans_amd.ncf_engine import NCFEngine
    dev = torch.device("cuda:0")
    U, I, E, M, B, n = 500, 400, 16, 50, 512, 5
    t, _ = random_neumf(U, I, E, M, seed=1)
    rs = np.random.RandomState(1)
    pool_u, pool_i = rs.randint(0, U, 5000), rs.randint(0, I, 5000)
    pu, pi = torch.from_numpy(rs.randint(0, U, B)).to(dev), torch.from_numpy(rs.randint(0, I, B)).to(dev)
    e = NCFEngine(t[0], t[1], t[4:], pool_u, pool_i, orng.py_seed_state(0), loss="pointwise", lr=1e-2,
                  weight_decay=1e-5, n_neg=n, batch_size=B, device=dev, seed=7, mf_user_w=t[2], mf_item_w=t[3])
    v0 = float(e.val_loss(pu, pi)[0])
    ls = [float(e.train_step(pu, pi, plan=e.make_plan(pi))[0]) for _ in range(8)]
    v1 = float(e.val_loss(pu, pi)[0])
    assert all(np.isfinite(ls)) and np.isfinite(v0) and ls[-1] < ls[0] and v1 < v0
