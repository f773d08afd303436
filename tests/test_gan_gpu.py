"""cGAN on the GPU (rg_gemm.hip, rg_gan.hip through the C-ABI).

* the fp32 MFMA GEMM against a float64 product of the same fp32 operands, every
  operand layout, split-K, ragged edges and the tanh epilogue (tolerance: 2e-6 of
  sum |a b| per element, the f32 fma-chain bound at these K);
* the discriminator / generator iterations against the reference's own steps
  (tests/golden/gan_*.npz, recorded z and dropout masks fed in): D outputs, G(z),
  losses, BatchNorm running stats, inference slates, and every parameter after
  every step with the criterion of tests/test_gan_oracle.param_ok (1e-5 relative,
  elements whose float64 gradient cancels to noise excepted);
* generation through the fused argmax epilogue (heads wider than a column tile)
  against the eval-mode forward of the float64 restatement;
* the device dropout / noise path trains and is reproducible."""
import os

import numpy as np
import pytest
import torch

from oracle import gan as og
from tests.test_gan_oracle import key, load, param_ok

pytestmark = pytest.mark.gpu


def gemm(A, B, a_km, b_km, M, N, K, post=0, splits=1, bias=None, ldc=None):
    from recommendation_gans_amd import _lib
    from recommendation_gans_amd.gan_engine import ptr
    import ctypes
    L = _lib.load()
    ldc = ldc or N
    C = torch.zeros(M, ldc, device="cuda")
    work = torch.zeros(max(1, splits) * M * N, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = L.rg_gemm_f32(st, ptr(A), A.shape[1], int(a_km), ptr(B), B.shape[1], int(b_km), M, N, K, ptr(C), ldc,
                       ptr(bias), post, splits, ptr(work))
    _lib.check(rc, "rg_gemm_f32")
    torch.cuda.synchronize()
    return C[:, :N].cpu()


@pytest.mark.parametrize("a_km,b_km", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K,splits", [(256, 512, 1000, 1), (250, 130, 64, 1), (64, 256, 2048, 7),
                                          (300, 40, 36, 3),
                                          (256, 512, 100544, 64)])   # C4's D layer 1 (S*N rounded to 4)
def test_gemm_matches_float64(a_km, b_km, M, N, K, splits):
    if (a_km or b_km) and K % 4:
        pytest.skip("K-major operands need K % 4 == 0")
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    a = torch.randn(M, K, generator=g)
    b = torch.randn(N, K, generator=g)
    m4, n4 = (M + 3) // 4 * 4, (N + 3) // 4 * 4
    A = (a if a_km else torch.cat([a.t(), torch.zeros(K, m4 - M)], 1)).contiguous().cuda()
    B = (b if b_km else torch.cat([b.t(), torch.zeros(K, n4 - N)], 1)).contiguous().cuda()
    got = gemm(A, B, a_km, b_km, M, N, K, splits=splits)
    ref = a.double() @ b.double().t()
    bound = 2e-6 * (a.double().abs() @ b.double().abs().t()) + 1e-30
    assert ((got.double() - ref).abs() <= bound).all()


def test_gemm_bias_tanh():
    g = torch.Generator().manual_seed(3)
    a, b, bias = torch.randn(200, 64, generator=g) * 0.2, torch.randn(300, 64, generator=g) * 0.2, torch.randn(300)
    got = gemm(a.cuda(), b.cuda(), True, True, 200, 300, 64, post=1, bias=bias.cuda(), ldc=304)
    ref = torch.tanh(a.double() @ b.double().t() + bias.double())
    assert (got.double() - ref).abs().max() < 2e-6


@pytest.fixture(params=[0, 1], ids=["epilogue", "wave_specialised"])
def gemm_ws(request):
    """Both forms of the optimizer GEMM (rg_gemm_ws_mode): the update in gemm_kernel's
    epilogue, and the wave-specialised persistent kernel."""
    from recommendation_gans_amd import _lib
    L = _lib.load()
    if request.param and not _lib.ab_build():
        assert L.rg_gemm_ws_mode(1) == -1     # the product refuses it
        pytest.skip("wave-specialised form: A/B build only (scripts/gpu_ab_tests.sh)")
    prev = L.rg_gemm_ws_mode(request.param)
    yield request.param
    L.rg_gemm_ws_mode(prev)


@pytest.mark.parametrize("M,N,K,ldp", [(512, 20000, 256, 20000),   # several tiles per workgroup (persistent)
                                       (300, 1001, 64, 1004),      # K < 8 steps, ragged float4 tail column
                                       (130, 5003, 640, 5003)])    # K > 8 steps, rows not float4-aligned
def test_gemm_rmsprop_matches_float64(M, N, K, ldp, gemm_ws):
    """The gradient GEMM fused with the RMSprop update (the cGAN's W1S / WH path,
    CGANs.py:440-457 RMSprop on D and G) against a float64 product + update of the
    same fp32 operands: P within the f32 GEMM bound propagated through the update."""
    from recommendation_gans_amd import _lib
    from recommendation_gans_amd.gan_engine import ptr
    import ctypes
    L = _lib.load()
    g = torch.Generator().manual_seed(M + N + K)
    a, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    m4, n4 = (M + 3) // 4 * 4, (N + 3) // 4 * 4
    A = torch.cat([a.t(), torch.zeros(K, m4 - M)], 1).contiguous().cuda()
    B = torch.cat([b.t(), torch.zeros(K, n4 - N)], 1).contiguous().cuda()
    p0 = torch.randn(M, ldp, generator=g) * 0.01
    v0 = torch.rand(M, ldp, generator=g) * 1e-3
    P, V = p0.clone().cuda(), v0.clone().cuda()
    lr, alpha, eps = 1e-3, 0.99, 1e-8
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.rg_gemm_f32_rms(st, ptr(A), m4, 0, ptr(B), n4, 0, M, N, K, ptr(P), ptr(V), ldp, lr, alpha, eps),
               "rg_gemm_f32_rms")
    torch.cuda.synchronize()
    gd = a.double() @ b.double().t()
    vd = alpha * v0[:, :N].double() + (1 - alpha) * gd * gd
    pd = p0[:, :N].double() - lr * gd / (vd.sqrt() + eps)
    gb = 2e-6 * (a.double().abs() @ b.double().abs().t())
    Pg, Vg = P.cpu().double(), V.cpu().double()
    assert ((Vg[:, :N] - vd).abs() <= 2 * gd.abs() * gb + 1e-6 * vd).all()
    # d(lr g / sqrt(v)) / dg <= lr * 2 / sqrt(v): the GEMM bound carried through, plus f32 rounding
    assert ((Pg[:, :N] - pd).abs() <= 2 * lr * gb / vd.sqrt() + 1e-6 * pd.abs() + 1e-9).all()
    assert torch.equal(P.cpu()[:, N:], p0[:, N:]) and torch.equal(V.cpu()[:, N:], v0[:, N:]), "pad columns touched"


@pytest.mark.parametrize("M,N,K", [(512, 100540, 256),   # C4's W1S: 3,144 tiles over 256 persistent workgroups
                                   (100540, 256, 256),   # C4's WH (the long dimension in M)
                                   (130, 5003, 640)])    # ragged rows and columns
def test_gemm_rmsprop_forms_bit_identical(M, N, K):
    """The wave-specialised optimizer GEMM (A/B build; measured slower) gives the
    same bits as the epilogue form: same per-lane K order, same update arithmetic
    (rg_gemm.hip gemm_opt_ws_kernel)."""
    from recommendation_gans_amd import _lib
    from recommendation_gans_amd.gan_engine import ptr
    import ctypes
    L = _lib.load()
    if not _lib.ab_build():
        pytest.skip("wave-specialised form: A/B build only (scripts/gpu_ab_tests.sh)")
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    m4, n4 = (M + 3) // 4 * 4, (N + 3) // 4 * 4
    A = torch.randn(K, m4, device="cuda", generator=g)
    B = torch.randn(K, n4, device="cuda", generator=g)
    p0 = torch.randn(M, n4, device="cuda", generator=g) * 0.01
    v0 = torch.rand(M, n4, device="cuda", generator=g) * 1e-3
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = []
    prev = L.rg_gemm_ws_mode(-1)
    try:
        for mode in (0, 1):
            L.rg_gemm_ws_mode(mode)
            P, V = p0.clone(), v0.clone()
            _lib.check(L.rg_gemm_f32_rms(st, ptr(A), m4, 0, ptr(B), n4, 0, M, N, K, ptr(P), ptr(V), n4,
                                         1e-3, 0.99, 1e-8), "rg_gemm_f32_rms")
            torch.cuda.synchronize()
            out.append((P, V))
    finally:
        L.rg_gemm_ws_mode(prev)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    assert not torch.equal(out[0][0], p0)


CASES = ["gan_rms_n50", "gan_adam_n50", "gan_sgd_n64"]


def make_engine(z, gp, gb, dn, g_init, d_init, dims, opt, lr):
    from recommendation_gans_amd.gan_engine import GANEngine
    N, S, H, E, B, L, Z, nb, dsteps = dims
    g_sd = {k: torch.from_numpy(np.asarray(v).copy()) for k, v in g_init.items()}
    d_sd = {k: torch.from_numpy(np.asarray(v).copy()) for k, v in d_init.items()}
    return GANEngine(g_sd, d_sd, N, S, H, E, Z, batch_max=B, optimizer=opt, lr=lr)


@pytest.mark.parametrize("case", CASES)
def test_gan_steps_match_reference(golden_dir, case):
    from recommendation_gans_amd.gan_engine import GANBatch
    z, dims, gp, gb, dn, g_init, d_init = load(golden_dir, case)
    N, S, H, E, B, L, Z, nb, dsteps = dims
    lr, opt = float(z["lr"][0]), case.split("_")[1]
    eng = make_engine(z, gp, gb, dn, g_init, d_init, dims, opt, lr)
    o = og.GANOracle(g_init, d_init, N, S, H, E, Z, opt=opt, lr=lr)
    scales = tuple(float(x) for x in z["drop_scale"])
    gat = int(z["g_step_at"][0])
    ill = {}
    for k in range(dsteps):
        b = int(z[f"d{k}_batch"][0])
        hist, sl = z["hist"][b * B:(b + 1) * B], z["slates"][b * B:(b + 1) * B]
        batch = GANBatch(hist, sl, N, S, "cuda")
        masks = [z[f"d{k}_mask{j}"] for j in range(8)]
        out = eng.d_step(batch, z=torch.from_numpy(z[f"d{k}_z"]), masks=masks).cpu().numpy()
        o.d_step(hist, sl, z[f"d{k}_z"].astype(np.float64), [m.astype(np.float64) for m in masks], scales)
        dval = eng.last_d_out(2 * B).cpu().numpy()
        np.testing.assert_allclose(dval[:B], z[f"d{k}_d_real"].ravel(), rtol=1e-5, err_msg=f"{case} D{k} real")
        np.testing.assert_allclose(dval[B:], z[f"d{k}_d_fake"].ravel(), rtol=1e-5, err_msg=f"{case} D{k} fake")
        # G(z): every element within 1e-5 of the tensor's scale (max |reference|), the bar
        # the C4 config test holds against the float64 oracle
        fk, fref = eng.last_fake(B).cpu().numpy(), z[f"d{k}_fake"]
        assert np.abs(fk - fref).max() <= 1e-5 * np.abs(fref).max(), f"{case} D{k} fake"
        assert abs(out[0] - z[f"d{k}_loss"][0]) <= 1e-5 * abs(z[f"d{k}_d_real"]).mean()
        dsd = eng.d_state_dict()
        for n in dn:
            ok, msg = param_ok(dsd[n].numpy(), z[key(f"d{k}_after_D_", n)], o.last_grads[n], lr,
                               prior=ill.setdefault("D" + n, np.zeros(o.D[n].shape, bool)))
            assert ok, f"{case} D{k} {n}: {msg}"
        gsd = eng.g_state_dict()
        for n in gb:
            np.testing.assert_allclose(gsd[n].numpy(), z[key(f"d{k}_after_G_", n)], rtol=1e-5, atol=1e-7,
                                       err_msg=f"{case} D{k} {n}")
        if k == gat:
            masks = [z[f"g{k}_mask{j}"] for j in range(5)]
            gl, slates = eng.g_step(batch, z=torch.from_numpy(z[f"g{k}_z"]), masks=masks)
            o.g_step(hist, z[f"g{k}_z"].astype(np.float64), [m.astype(np.float64) for m in masks], scales)
            np.testing.assert_allclose(float(gl[0]), z[f"g{k}_loss"][0], rtol=1e-5)
            np.testing.assert_allclose(eng.last_d_out(B).cpu().numpy(), z[f"g{k}_d_fake"].ravel(), rtol=1e-5)
            assert (slates.cpu().numpy() == z[f"g{k}_slates_after"]).all()
            gsd = eng.g_state_dict()
            for n in gp:
                ok, msg = param_ok(gsd[n].numpy(), z[key(f"g{k}_after_G_", n)], o.last_grads[n], lr,
                                   exempt=n in o.pre_bn_biases(),
                                   prior=ill.setdefault("G" + n, np.zeros(o.G[n].shape, bool)))
                assert ok, f"{case} G{k} {n}: {msg}"
            for n in gb:
                np.testing.assert_allclose(gsd[n].numpy(), z[key(f"g{k}_after_G_", n)], rtol=1e-5, atol=1e-7)


def test_gan_reference_init_clamp(golden_dir):
    """The reference's own D init (clamp-bound): step-0 forward values (D outputs, G(z))
    and that the step started from the clamped weights."""
    from recommendation_gans_amd.gan_engine import GANBatch
    z, dims, gp, gb, dn, g_init, d_init = load(golden_dir, "gan_rms_refinit")
    N, S, H, E, B, L, Z, nb, dsteps = dims
    lr = float(z["lr"][0])
    eng = make_engine(z, gp, gb, dn, g_init, d_init, dims, "rms", lr)
    batch = GANBatch(z["hist"][:B], z["slates"][:B], N, S, "cuda")
    eng.d_step(batch, z=torch.from_numpy(z["d0_z"]), masks=[z[f"d0_mask{j}"] for j in range(8)])
    dval = eng.last_d_out(2 * B).cpu().numpy()
    np.testing.assert_allclose(dval[:B], z["d0_d_real"].ravel(), rtol=1e-5)
    np.testing.assert_allclose(dval[B:], z["d0_d_fake"].ravel(), rtol=1e-5)
    fref = z["d0_fake"]
    assert np.abs(eng.last_fake(B).cpu().numpy() - fref).max() <= 1e-5 * np.abs(fref).max()
    dsd = eng.d_state_dict()
    for n in dn:
        before = np.clip(d_init[n], -og.CLAMP, og.CLAMP)
        assert np.abs(dsd[n].numpy() - before).max() <= 10 * lr * (1 + 1e-5), n


def random_gan(N, S, H, E, Z, seed):
    """Reference-shaped G / D state dicts (cGAN_models.py init: xavier weights, bias 0.01,
    N(0,1) embeddings with a zero padding row, BatchNorm gamma 1 / beta 0)."""
    g = torch.Generator().manual_seed(seed)
    H1 = H // 2

    def lin(o, i):
        b = (6.0 / (i + o)) ** 0.5
        return (torch.rand(o, i, generator=g) * 2 - 1) * b, torch.full((o,), 0.01)

    def emb():
        e = torch.randn(N + 1, E, generator=g)
        e[N] = 0
        return e

    gs = {"embedding_layer.weight": emb()}
    for pre, (o, i) in (("layers.0", (H1, Z + E)), ("layers.4", (H, H1))):
        gs[pre + ".weight"], gs[pre + ".bias"] = lin(o, i)
    for pre, w in (("layers.1", H1), ("layers.5", H)):
        gs.update({pre + ".weight": torch.ones(w), pre + ".bias": torch.zeros(w), pre + ".running_mean": torch.zeros(w),
                   pre + ".running_var": torch.ones(w), pre + ".num_batches_tracked": torch.tensor(0)})
    for s in range(S):
        gs[f"mult_heads.head_{s}.weight"], gs[f"mult_heads.head_{s}.bias"] = lin(N, H)
    ds = {"embedding_layer.weight": emb()}
    for pre, (o, i) in (("layers.0", (2 * H, S * N + E)), ("layers.3", (H, 2 * H)), ("layers.6", (H1, H)),
                        ("layers.9", (1, H1))):
        ds[pre + ".weight"], ds[pre + ".bias"] = lin(o, i)
    return gs, ds


def hist_and_slates(rs, rows, N, S, L):
    hist = np.full((rows, L), N, np.int64)
    for r in range(rows):
        ln = rs.randint(0, L + 1)
        hist[r, :ln] = rs.choice(N, ln, replace=False)
    slates = np.stack([rs.choice(N, S, replace=False) for _ in range(rows)])
    return hist, slates


def test_gan_generate_fused_argmax():
    """Heads of N = 300 > one column tile: the fused argmax epilogue (tiles straddling two
    heads) against the float64 eval-mode forward; a near-tie may pick either item, so the
    chosen item's tanh must be the maximum to 1e-5."""
    from recommendation_gans_amd.gan_engine import GANBatch, GANEngine
    N, S, H, E, Z, B, L = 300, 5, 32, 5, 100, 64, 12
    gs, ds = random_gan(N, S, H, E, Z, 5)
    gs["layers.1.running_mean"].uniform_(-0.1, 0.1)
    gs["layers.5.running_var"].uniform_(0.5, 2.0)
    eng = GANEngine(gs, ds, N, S, H, E, Z, batch_max=B)
    rs = np.random.RandomState(1)
    hist, _ = hist_and_slates(rs, B, N, S, L)
    zz = torch.rand(B, Z, generator=torch.Generator().manual_seed(2))
    got = eng.generate(GANBatch(hist, None, N, S, "cuda"), z=zz).cpu().numpy().astype(np.int64)
    o = og.GANOracle({k: v.numpy() for k, v in gs.items()}, {k: v.numpy() for k, v in ds.items()}, N, S, H, E, Z)
    heads, _ = o.g_forward(zz.double().numpy(), hist.astype(np.float64), train=False)
    for s in range(S):
        t = heads[s]
        chosen = t[np.arange(B), got[:, s]]
        assert (chosen >= t.max(1) - 1e-5).all()


def test_gan_device_noise_trains():
    """torch.rand z and the hash dropout: finite losses, reproducible for a seed, and the
    generator's loss responds to training."""
    from recommendation_gans_amd.gan_engine import GANBatch, GANEngine
    N, S, H, E, Z, B, L = 200, 5, 64, 5, 100, 128, 20
    gs, ds = random_gan(N, S, H, E, Z, 9)
    rs = np.random.RandomState(4)
    hist, slates = hist_and_slates(rs, B, N, S, L)
    runs = []
    for rep in range(2):
        eng = GANEngine(gs, ds, N, S, H, E, Z, batch_max=B, seed=3)
        batch = GANBatch(hist, slates, N, S, "cuda")
        torch.manual_seed(11)
        losses = []
        for k in range(10):
            losses.append(eng.d_step(batch).cpu().numpy())
            if (k + 1) % 5 == 0:
                losses.append(eng.g_step(batch)[0].cpu().numpy())
        runs.append(np.concatenate(losses))
        assert np.isfinite(runs[-1]).all()
    np.testing.assert_array_equal(runs[0], runs[1])


def test_gan_reference_init_full_cycle(golden_dir):
    """the reference's own D init (clamp-bound) at lr 1e-3 over a whole
    n_critic cycle -- five D iterations, the G iteration after the fifth, a sixth D iteration
    (tests/golden/gan_rms_refinit5.npz, the reference's steps with their z and dropout masks).
    Free-running from the same init, every D / G tensor after every step is held to
    tensor_parity's rule: 1e-5 relative to the reference's fp32 tensor, or -- where the
    clamped weights put pre-activations on the LeakyReLU kink and summation order picks the
    slope, for any fp32 implementation -- no further from the float64 restatement (oracle/gan.py
    with the same z and masks) than 3x an fp32 implementation's own distance to it: the
    reference's, or the same restatement run in fp32 NumPy (another summation order).  The
    second matters where an exact gradient is 0: a clamped layer's bias sums terms that cancel
    exactly, torch's CPU order leaves 0 and fp32 NumPy (and the GPU) a 1e-10 residue that
    RMSprop's g / (sqrt(v) + eps) turns into a 2.8e-5 step (D0 layers.6.bias, measured).
    Nothing is exempted; the fraction of elements off by more than 1e-5 of the tensor's scale
    is reported (stdout, and RG_REPORT_DIR/gan_refinit5_parity.json when set)."""
    import json
    from oracle import mf as omf
    from recommendation_gans_amd.gan_engine import GANBatch
    z, dims, gp, gb, dn, g_init, d_init = load(golden_dir, "gan_rms_refinit5")
    N, S, H, E, B, L, Z, nb, dsteps = dims
    lr = float(z["lr"][0])
    assert lr == 1e-3 and dsteps == 6 and int(z["g_step_at"][0]) == 4
    assert (np.abs(d_init["layers.0.weight"]) > og.CLAMP).mean() > 0.5, "the reference init binds the clamp"
    eng = make_engine(z, gp, gb, dn, g_init, d_init, dims, "rms", lr)
    o = og.GANOracle(g_init, d_init, N, S, H, E, Z, opt="rms", lr=lr)
    o32 = og.GANOracle(g_init, d_init, N, S, H, E, Z, opt="rms", lr=lr, dtype=np.float32)
    scales = tuple(float(x) for x in z["drop_scale"])
    sc32 = tuple(np.float32(x) for x in scales)
    report, worst = [], []
    for k in range(dsteps):
        b = int(z[f"d{k}_batch"][0])
        hist, sl = z["hist"][b * B:(b + 1) * B], z["slates"][b * B:(b + 1) * B]
        batch = GANBatch(hist, sl, N, S, "cuda")
        masks = [z[f"d{k}_mask{j}"] for j in range(8)]
        eng.d_step(batch, z=torch.from_numpy(z[f"d{k}_z"]), masks=masks)
        o.d_step(hist, sl, z[f"d{k}_z"].astype(np.float64), [m.astype(np.float64) for m in masks], scales)
        o32.d_step(hist, sl, z[f"d{k}_z"], [m.astype(np.float32) for m in masks], sc32)
        dgr = dict(o.last_grads)
        checks = [(f"D{k} D.{n}", eng.d_state_dict()[n].numpy(), z[key(f"d{k}_after_D_", n)], o.D[n], o32.D[n], dgr)
                  for n in dn]
        if k == int(z["g_step_at"][0]):
            masks = [z[f"g{k}_mask{j}"] for j in range(5)]
            gl, slates = eng.g_step(batch, z=torch.from_numpy(z[f"g{k}_z"]), masks=masks)
            o.g_step(hist, z[f"g{k}_z"].astype(np.float64), [m.astype(np.float64) for m in masks], scales)
            o32.g_step(hist, z[f"g{k}_z"], [m.astype(np.float32) for m in masks], sc32)
            np.testing.assert_allclose(float(gl[0]), z[f"g{k}_loss"][0], rtol=1e-5)
            gsd = eng.g_state_dict()
            ggr = dict(o.last_grads)
            checks += [(f"G{k} G.{n}", gsd[n].numpy(), z[key(f"g{k}_after_G_", n)], o.G[n], o32.G[n], ggr)
                       for n in gp + gb]
        for what, got, ref32, ref64, np32, grads in checks:
            t = lambda x: torch.from_numpy(np.asarray(x, np.float64).ravel())
            ok, msg = omf.tensor_parity(t(got), t(ref32), t(ref64))
            if not ok:                       # the band of the other fp32 implementation
                ok2, msg2 = omf.tensor_parity(t(got), t(np32), t(ref64))
                ok, msg = ok2, f"{msg}; vs fp32 NumPy: {msg2}"
            zero = np.zeros(np.asarray(got).size, bool)
            if not ok:
                # elements whose float64 gradient is EXACTLY zero (terms that cancel exactly, e.g.
                # a clamped layer's bias): an fp32 sum leaves 0 or a rounding residue depending on
                # its order, and RMSprop's g / (sqrt(v) + eps) turns a residue into a step of up to
                # lr -- counted and bounded by lr; every other element stays under the band rule
                name = what.split(".", 1)[1]
                zero = (np.asarray(grads[name]).ravel() == 0) if name in grads else zero
                keep = ~zero
                ok3, msg3 = omf.tensor_parity(t(got)[keep], t(ref32)[keep], t(ref64)[keep]) if keep.any() else \
                    (True, "no elements")
                if not ok3:
                    ok3, msg3 = omf.tensor_parity(t(got)[keep], t(np32)[keep], t(ref64)[keep])
                bound = bool(np.all(np.abs(np.asarray(got, np.float64).ravel() - np.asarray(ref64).ravel())[zero]
                                    <= lr * (1 + 1e-5)))
                ok = bool(zero.any()) and ok3 and bound
                msg = f"{msg}; {int(zero.sum())} exact-zero-gradient elements (|d| <= lr: {bound}), rest: {msg3}"
            scale = max(float(np.abs(ref32).max()), 1e-30)
            frac = float((np.abs(np.asarray(got, np.float64) - ref32) > 1e-5 * scale).mean())
            report.append({"tensor": what, "parity": msg, "frac_outside_1e-5_of_scale": frac,
                           "exact_zero_gradient_elements": int(zero.sum())})
            if not ok:
                detail = {}
                if np.asarray(got).size <= 16:
                    detail = {"gpu": np.asarray(got).ravel().tolist(), "ref32": np.asarray(ref32).ravel().tolist(),
                              "ref64": np.asarray(ref64).ravel().tolist()}
                    detail["grad64"] = np.asarray(grads.get(what.split(".", 1)[1], [])).ravel().tolist()
                report[-1]["detail"] = detail
                worst.append((what, msg))
    print(json.dumps(report, indent=0))
    if os.environ.get("RG_REPORT_DIR"):
        os.makedirs(os.environ["RG_REPORT_DIR"], exist_ok=True)
        with open(os.path.join(os.environ["RG_REPORT_DIR"], "gan_refinit5_parity.json"), "w") as fp:
            json.dump(report, fp, indent=1)
    assert not worst, worst
