"""GPU parity of the HIP MF path against the oracle (and the reference's goldens).

All calls go through the C-ABI (librg_hip.so via recommendation_gans_amd._lib).
Tolerance (north_star): fp32 results within 1e-5 relative; integer/index work
(negative-sample indices, MT state) bit-exact.
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import mf as omf
from oracle import rng as orng

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _np(x):
    return x.detach().double().cpu().numpy() if torch.is_tensor(x) else np.asarray(x, np.float64)


def close(got, ref, rtol=RTOL, what=""):
    """Elementwise: |got - ref| <= rtol * (|ref| + max|ref|).  Used where no step of
    the computation amplifies reduction-order noise (scores, losses, SGD)."""
    got, ref = _np(got), _np(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = float(np.max(np.abs(ref))) if ref.size else 0.0
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=rtol * max(scale, 1e-30), err_msg=what)


def close_adam(got, ref32, ref64, what="", small=False):
    """Adam/RMSprop trajectories, every table (the bias vectors included): 1e-5 relative
    (tensor norm), or -- where an element's gradient cancels to ~eps and its update
    g/(|g|+eps) is decided by summation order, for any fp32 implementation -- within
    the fp32 reference's own distance to the float64 result (oracle.mf.tensor_parity).
    The components are pinned tightly on their own: gradients elementwise
    (test_mf_gradients_elementwise), the optimizer update given identical gradients
    (test_optimizer_update_matches_torch).

    Bias vectors (small=True): the same 1e-5 relative, with a wider fp64 band (15x the fp32
    reference's own distance instead of 3x).  Measured need: test_mf_step_dims[200] step 0,
    user biases 1.26e-5 relative: a bias element whose gradient (a sum of a few dz) cancels
    to ~1e-9 takes Adam's first step g / (|g| + eps) ~ g / eps, which turns the 1-ulp
    differences of dz (the device expf vs torch's vectorised exp, FMA contraction) into
    ~1e-5 of the vector's norm, while the fp32 reference happens to sit 1.3e-6 from fp64."""
    ok, msg = omf.tensor_parity(got, ref32, ref64, rtol=1e-5, band=15.0 if small else 3.0)
    assert ok, f"{what}: {msg}"


def close_norm(got, ref, rtol=RTOL, what=""):
    """Tensor parity as a relative error: ||got - ref||_2 <= rtol * ||ref||_2.

    After an Adam/RMSprop step an element whose gradient sum nearly cancels has
    its update m/(sqrt(v)+eps) decided by the last bits of that sum, which depend
    on summation order (GPU list order vs CPU index_add order); such single
    elements legitimately differ by up to ~lr * 1e-3, so the embeddings are
    compared as tensors (the gradients themselves are checked elementwise against
    a condition-aware bound in test_mf_gradients_elementwise)."""
    got, ref = _np(got), _np(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = np.linalg.norm(got - ref)
    nrm = np.linalg.norm(ref)
    assert err <= rtol * max(nrm, 1e-30), f"{what}: rel err {err / max(nrm, 1e-30):.3e} > {rtol}"


@pytest.fixture(scope="module")
def dev():
    from recommendation_gans_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


# ------------------------------------------------------------------ sampler
def temper(y):
    """MT19937 output tempering (the device stores raw state words)."""
    y = y.astype(np.uint32)
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


@pytest.mark.parametrize("seed,skip,nwords", [(0, 0, 81920), (5, 3, 1), (7, 623, 624), (9, 624, 625),
                                              (11, 100, 0), (13, 5, 100_003), (2 ** 40 + 7, 0, 2 * 5 * 8192 * 8)])
def test_mt_generate_bit_exact(dev, seed, skip, nwords):
    from recommendation_gans_amd import _lib
    lib = _lib.load()
    st = orng.py_seed_state(seed)
    for _ in range(skip):
        lib_ref = orng.lib().orc_mt_next(st)   # advance the oracle state mid-block
    dstate = torch.from_numpy(st.view(np.int32).copy()).to(dev)
    out = torch.empty(nwords + _lib.RG_MT_PAD, dtype=torch.int32, device=dev)
    before = torch.empty(625, dtype=torch.int32, device=dev)
    _lib.check(lib.rg_mt_generate(_lib.stream_handle(), _lib.ptr(dstate), _lib.ptr(out), nwords,
                                  _lib.ptr(before)), "rg_mt_generate")
    torch.cuda.synchronize()
    assert (before.cpu().numpy().view(np.uint32) == st).all()
    ref = np.array([orng.lib().orc_mt_next(st) for _ in range(nwords)], dtype=np.uint32)
    got = temper(out.cpu().numpy().view(np.uint32)[:nwords])
    assert (got == ref).all()
    assert (dstate.cpu().numpy().view(np.uint32) == st).all()


def test_sampler_indices_match_random_choices(dev):
    """Words -> indices exactly as random.choices(pool, k) (implicit.py:352)."""
    import random
    from recommendation_gans_amd.mf_engine import DeviceSampler
    random.seed(1234)
    s = DeviceSampler(orng.state_from_python(random.getstate()), dev)
    n = 8_100_000
    for _ in range(3):
        w = s.acquire(2 * 40960)
        torch.cuda.synchronize()
        words = temper(w.cpu().numpy().view(np.uint32)[: 2 * 40960])
        s.release()
        a = (words[0::2] >> 5).astype(np.float64)
        b = (words[1::2] >> 6).astype(np.float64)
        idx = np.floor((a * 67108864.0 + b) * (1.0 / 9007199254740992.0) * float(n)).astype(np.int64)
        ref = np.array(random.choices(range(n), k=40960), dtype=np.int64)
        assert (idx == ref).all()
    # prefetched words are not "drawn": the exported state equals Python's
    assert (s.export_state() == orng.state_from_python(random.getstate())).all()


# ------------------------------------------------------------------ MF step
def make_case(U, I, d, B, n, P, seed, hot_items=False):
    g = torch.Generator().manual_seed(seed)
    Uw = torch.randn(U, d, generator=g) / d
    Iw = torch.randn(I, d, generator=g) / d
    ub = torch.randn(U, 1, generator=g) * 0.1
    ib = torch.randn(I, 1, generator=g) * 0.1
    rs = np.random.RandomState(seed)
    pool_u, pool_i = rs.randint(0, U, P), rs.randint(0, I, P)
    if hot_items:
        pool_i[: P // 2] = 3                # half of all negatives hit item 3 -> list overflow
    steps = []
    for s in range(4):
        bp = B if s != 2 else max(1, B - 7)     # step 2 is a partial batch
        pu, pi = rs.randint(0, U, bp), rs.randint(0, I, bp)
        if hot_items:
            pi[: bp // 3] = 3
            pu[: bp // 4] = 5
        steps.append((pu, pi))
    return (Uw, Iw, ub, ib), pool_u, pool_i, steps


def run_parity(dev, U, I, d, B, n, loss, opt, wd=1e-5, seed=0, hot=False, P=5000, lr=1e-2, plan=False):
    from recommendation_gans_amd.mf_engine import MFEngine
    tabs, pool_u, pool_i, steps = make_case(U, I, d, B, n, P, seed, hot_items=hot)
    st = orng.py_seed_state(100 + seed)
    o = omf.MFOracle(*[t.clone() for t in tabs], pool_u, pool_i, st.copy(), loss=loss, optimizer=opt, lr=lr,
                     weight_decay=wd, n_neg=n, batch_size=B)
    o64 = omf.MFOracle(*[t.clone().double() for t in tabs], pool_u, pool_i, st.copy(), loss=loss, optimizer=opt,
                       lr=lr, weight_decay=wd, n_neg=n, batch_size=B)
    e = MFEngine(tabs[0], tabs[1], tabs[2].reshape(-1), tabs[3].reshape(-1), pool_u, pool_i, st.copy(), loss=loss,
                 optimizer=opt, lr=lr, weight_decay=wd, n_neg=n, batch_size=B, device=dev)
    for s, (pu, pi) in enumerate(steps):
        ref_loss = o.step(pu, pi)
        o64.step(pu, pi)
        du, di = torch.from_numpy(pu).to(dev), torch.from_numpy(pi).to(dev)
        got = e.train_step(du, di, plan=e.make_plan(di) if plan else None)
        torch.cuda.synchronize()
        tag = f"{loss}/{opt}/d{d}/step{s}{'/plan' if plan else ''}"
        close(got[0], np.float32(ref_loss), what=tag + " loss")
        for k, nm in enumerate(("user_w", "item_w", "user_b", "item_b")):
            shp = e.params()[k].shape
            if opt == "sgd":
                close(e.params()[k], o.params[k].reshape(shp), what=f"{tag} {nm}")
            else:
                close_adam(e.params()[k], o.params[k].reshape(shp), o64.params[k].reshape(shp), what=f"{tag} {nm}",
                           small=k >= 2)
            if opt == "adam":
                close_adam(e.m[k], o.opt.state[k][0].reshape(shp), o64.opt.state[k][0].reshape(shp),
                           what=f"{tag} m {nm}", small=k >= 2)
            if opt != "sgd":
                close_adam(e.v[k], o.opt.state[k][1].reshape(shp), o64.opt.state[k][1].reshape(shp),
                           what=f"{tag} v {nm}", small=k >= 2)
        assert (e.mt_state() == o.state).all(), tag + " MT state"
    # scratch left clean for the next step
    assert int(e.row_count.abs().sum()) == 0
    assert float(e.hot_grad.abs().sum()) == 0.0
    return e, o


@pytest.mark.parametrize("loss", ["pointwise", "bpr", "hinge", "adaptive_hinge"])
@pytest.mark.parametrize("opt", ["adam", "sgd", "rms"])
def test_mf_step_losses_optimizers(dev, loss, opt):
    run_parity(dev, 300, 200, 64, 128, 5, loss, opt)


@pytest.mark.parametrize("d", [8, 16, 32, 50, 64, 100, 128, 200, 256, 1, 7])
def test_mf_step_dims(dev, d):
    run_parity(dev, 200, 150, d, 64, 5, "bpr", "adam")
    run_parity(dev, 200, 150, d, 64, 3, "pointwise", "adam")


@pytest.mark.parametrize("n", [1, 2, 5, 8])
def test_mf_step_neg_counts(dev, n):
    run_parity(dev, 200, 150, 32, 96, n, "bpr", "adam")


@pytest.mark.parametrize("loss", ["pointwise", "bpr"])
@pytest.mark.parametrize("plan", [False, True])
def test_mf_step_hot_rows_overflow(dev, loss, plan):
    """Rows touched > RG_MF_LIST_CAP times take the overflow accumulators (no plan) or the
    planned per-block partial rows (positives' item side)."""
    run_parity(dev, 50, 40, 64, 256, 5, loss, "adam", hot=True, plan=plan)


@pytest.mark.parametrize("d", [8, 32, 50, 64, 128, 256])
@pytest.mark.parametrize("loss", ["pointwise", "bpr", "hinge", "adaptive_hinge"])
def test_mf_step_plan(dev, d, loss):
    """Item-sorted plan path (per-block partials for the positives' item side)."""
    run_parity(dev, 300, 200, d, 256, 5, loss, "adam", plan=True, hot=(d == 64))
    run_parity(dev, 300, 200, d, 256, 5, loss, "sgd", plan=True, hot=(d == 64))


def test_mf_step_batch_of_one(dev):
    run_parity(dev, 20, 10, 16, 1, 5, "pointwise", "adam")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "mf_*_*_d*.npz"))))
def test_mf_step_vs_reference_golden(dev, path):
    """The HIP path replays the reference's own steps (fixtures from make_golden.py)."""
    from recommendation_gans_amd.mf_engine import MFEngine
    g = np.load(path)
    U, I, d, B, n = (int(x) for x in g["meta"])
    base = os.path.basename(path)[3:-4]
    loss = "adaptive_hinge" if base.startswith("adaptive") else base.split("_")[0]
    opt = base.split("_")[-2] if not base.endswith("wd0") else base.split("_")[-3]
    names = ["user_embeddings_weight", "item_embeddings_weight", "user_biases_weight", "item_biases_weight"]
    init = [g["init_" + nm] for nm in names]
    e = MFEngine(init[0], init[1], init[2].reshape(-1), init[3].reshape(-1), g["pool_u"], g["pool_i"],
                 g["s0_mt_state"].copy(), loss=loss, optimizer=opt, lr=float(g["lr"][0]),
                 weight_decay=float(g["wd"][0]), n_neg=n, batch_size=B, device=dev)
    for s in range(3):
        got = e.train_step(torch.from_numpy(g[f"s{s}_pos_u"]).to(dev), torch.from_numpy(g[f"s{s}_pos_i"]).to(dev))
        torch.cuda.synchronize()
        close(got[0], g[f"s{s}_loss"][0], what=f"{path} step {s} loss")
        cmp = close if opt == "sgd" else close_norm
        for k, nm in enumerate(names):
            cmp(e.params()[k], g[f"s{s}_after_{nm}"].reshape(e.params()[k].shape), what=f"{path} {s} {nm}")


@pytest.mark.parametrize("loss,hot,d", [("pointwise", False, 64), ("bpr", False, 64), ("hinge", False, 64),
                                        ("adaptive_hinge", False, 64), ("bpr", True, 64), ("bpr", False, 8),
                                        ("bpr", False, 50), ("bpr", False, 200), ("pointwise", True, 256),
                                        ("bpr", True, 128)])
def test_mf_gradients_elementwise(dev, loss, hot, d):
    """The flat data gradient (rg_mf_grads) against the oracle, element by element,
    with a bound that follows each element's condition: |g - g_ref| <= 1e-5 * sum|terms|.
    Teacher-forced: the engine's tables are set to the oracle's before every step, so
    no earlier step's rounding feeds in."""
    from recommendation_gans_amd.mf_engine import MFEngine
    U, I, B, n = 300, 200, 128, 5
    tabs, pool_u, pool_i, steps = make_case(U, I, d, B, n, 5000, 3, hot_items=hot)
    st = orng.py_seed_state(7)
    o = omf.MFOracle(*[t.clone() for t in tabs], pool_u, pool_i, st.copy(), loss=loss, optimizer="adam", lr=1e-2,
                     weight_decay=1e-5, n_neg=n, batch_size=B)
    e = MFEngine(tabs[0], tabs[1], tabs[2].reshape(-1), tabs[3].reshape(-1), pool_u, pool_i, st.copy(), loss=loss,
                 optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
    for s, (pu, pi) in enumerate(steps):
        Uo, Io, ubo, ibo = [p.clone() for p in o.params]
        e.set_params(Uo, Io, ubo, ibo)
        out = o.step(pu, pi, return_all=True)
        du, di = torch.from_numpy(pu).to(dev), torch.from_numpy(pi).to(dev)
        g = e.grads(du, di, plan=e.make_plan(di) if s % 2 else None).cpu().double().numpy()
        u = torch.cat([torch.from_numpy(pu).long(), out["neg_u"]])
        i = torch.cat([torch.from_numpy(pi).long(), out["neg_i"]])
        p = torch.cat([out["p_pos"], out["p_neg"]])
        _, dpp, dpn = omf.loss_and_dp(loss, out["p_pos"], out["p_neg"], n, B)
        dz = (torch.cat([dpp, dpn]) * (1 - p) * p).abs()
        bU, bI, bub, bib = omf.dense_grads(Uo.abs(), Io.abs(), ubo, ibo, u, i, dz)
        ref = [x.double().numpy().reshape(-1) for x in out["grads"]]
        bound = [x.double().numpy().reshape(-1) for x in (bU, bI, bub, bib)]
        D = d
        got = [g[:U * D], g[U * D:(U + I) * D], g[(U + I) * D:(U + I) * D + U], g[(U + I) * D + U:(U + I) * (D + 1)]]
        for k in range(4):
            tol = 1e-5 * bound[k] + 1e-12
            bad = np.abs(got[k] - ref[k]) > tol
            assert not bad.any(), f"step {s} table {k}: {bad.sum()} elements, max err " \
                                  f"{np.max(np.abs(got[k] - ref[k])):.3e}"
        close(g[-1], np.float32(out["loss"]), what="loss slot")
        assert (e.mt_state() == o.state).all()


@pytest.mark.parametrize("loss", ["pointwise", "bpr"])
def test_mf_dense_update_path(dev, loss):
    """The replicated data-parallel step at world size 1 without a communicator
    (rg_mf_stepper_dp_begin: pairs -> rank-major rg_mf_grads_sharded; identity exchange;
    rg_mf_stepper_dp_end: rg_mf_apply_shard) tracks the oracle over several steps,
    optimizer state included."""
    from recommendation_gans_amd.mf_engine import MFEngine
    U, I, d, B, n = 300, 200, 64, 128, 5
    tabs, pool_u, pool_i, steps = make_case(U, I, d, B, n, 5000, 4)
    st = orng.py_seed_state(8)
    o = omf.MFOracle(*[t.clone() for t in tabs], pool_u, pool_i, st.copy(), loss=loss, optimizer="adam", lr=1e-2,
                     weight_decay=1e-5, n_neg=n, batch_size=B)
    e = MFEngine(tabs[0], tabs[1], tabs[2].reshape(-1), tabs[3].reshape(-1), pool_u, pool_i, st.copy(), loss=loss,
                 optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev,
                 dp="global_stream")
    for s, (pu, pi) in enumerate(steps):
        ref = o.step(pu, pi)
        got = e.train_step(torch.from_numpy(pu).to(dev), torch.from_numpy(pi).to(dev), len(pu))
        torch.cuda.synchronize()
        close(got[0], np.float32(ref), what=f"dense step {s} loss")
        for k in range(4):
            close_norm(e.params()[k], o.params[k].reshape(e.params()[k].shape), what=f"dense step {s} {k}")
            close_norm(e.m[k], o.opt.state[k][0].reshape(e.m[k].shape), what=f"dense step {s} m{k}")
            close_norm(e.v[k], o.opt.state[k][1].reshape(e.v[k].shape), what=f"dense step {s} v{k}")


def _torch_formula_step(opt, p, gr, m, v, t, lr, wd, cr_sqrt, betas=(0.5, 0.999), alpha=0.99, eps=1e-8):
    """torch.optim's single-tensor update written out op by op (torch/optim/adam.py,
    rmsprop.py, sgd.py), CPU tensor ops so each op keeps torch's own rounding; with
    cr_sqrt the sqrt is correctly rounded instead (ATen's CPU fp32 sqrt goes through
    MKL VML, which is 1 ulp off for small inputs such as v ~ 1e-21)."""
    sqrt = (lambda x: x.double().sqrt().float()) if cr_sqrt else torch.sqrt
    g = gr.add(p, alpha=wd)
    if opt == "sgd":
        return p.add(g, alpha=-lr), m, v
    if opt == "adam":
        b1, b2 = betas
        m = m.lerp(g, 1 - b1)
        v = v.mul(b2).addcmul(g, g, value=1 - b2)
        denom = (sqrt(v) / ((1 - b2 ** t) ** 0.5)).add(eps)
        return p.addcdiv(m, denom, value=-(lr / (1 - b1 ** t))), m, v
    v = v.mul(alpha).addcmul(g, g, value=1 - alpha)
    return p.addcdiv(g, sqrt(v).add(eps), value=-lr), m, v


def _ulps(a, b):
    return np.abs(a.numpy().view(np.int32).astype(np.int64) - b.numpy().view(np.int32).astype(np.int64))


@pytest.mark.parametrize("d", [64, 50])
@pytest.mark.parametrize("opt", ["adam", "sgd", "rms"])
def test_optimizer_update_matches_torch(dev, opt, d):
    """Given the same gradient, rg_mf_apply_dense's update is torch.optim's
    single-tensor CPU update, over 3 steps with evolving m/v and elements with
    |g| ~ eps.  Teacher-forced from the GPU's previous p/m/v, every element is within
    1 ulp of torch's op sequence (with torch's sqrt or a correctly rounded one), p, m
    and v; the trajectory stays within 2^-18 of the largest |p| + |update| each
    element has seen of torch.optim itself."""
    from recommendation_gans_amd.mf_engine import MFEngine
    U, I = 120, 70
    g = torch.Generator().manual_seed(1)
    params = [torch.randn(U, d, generator=g) / d, torch.randn(I, d, generator=g) / d,
              torch.randn(U, generator=g) * 0.1, torch.randn(I, generator=g) * 0.1]
    e = MFEngine(*params, np.zeros(4, np.int64), np.zeros(4, np.int64), orng.py_seed_state(0), loss="bpr",
                 optimizer=opt, lr=1e-2, weight_decay=1e-5, n_neg=5, batch_size=8, device=dev)
    tparams = [p.clone().requires_grad_(True) for p in params]
    topt = {"adam": lambda ps: torch.optim.Adam(ps, lr=1e-2, betas=(0.5, 0.999), weight_decay=1e-5),
            "sgd": lambda ps: torch.optim.SGD(ps, lr=1e-2, weight_decay=1e-5),
            "rms": lambda ps: torch.optim.RMSprop(ps, lr=1e-2, weight_decay=1e-5)}[opt](tparams)
    hist = [p.abs() for p in params]      # largest |p| + |update| each element has seen
    for step in range(3):
        grads = [torch.randn(p.shape, generator=g) * 10 ** float(torch.randint(-9, -2, (1,), generator=g))
                 for p in params]
        grads[0][0, :5] = torch.tensor([1e-8, -1e-8, 3e-9, 0.0, -2e-8])     # |g| ~ eps
        torch.cuda.synchronize()
        state = lambda x, k: torch.zeros_like(params[k]) if x is None else x.cpu().reshape(params[k].shape).clone()
        before = [(e.params()[k].cpu().clone(), state(e.m[k], k), state(e.v[k], k)) for k in range(4)]
        flat = torch.cat([grads[0].reshape(-1), grads[1].reshape(-1), grads[2], grads[3], torch.zeros(1)])
        e.apply_dense(flat.to(dev))
        prev = [p.detach().clone() for p in tparams]
        for p, gr in zip(tparams, grads):
            p.grad = gr.clone()
        topt.step()
        torch.cuda.synchronize()
        for k in range(4):
            got = e.params()[k].cpu()
            p0, m0, v0 = before[k]
            refs = [_torch_formula_step(opt, p0, grads[k], m0, v0, step + 1, lr=1e-2, wd=1e-5, cr_sqrt=cr)
                    for cr in (False, True)]
            ulps = np.minimum(_ulps(got, refs[0][0]), _ulps(got, refs[1][0]))
            assert ulps.max() <= 1, f"{opt} step {step} tensor {k}: {int((ulps > 0).sum())} differ, max {ulps.max()} ulp"
            for name, dev_state, ref_state in (("m", e.m[k], refs[0][1]), ("v", e.v[k], refs[0][2])):
                if dev_state is not None:
                    su = _ulps(dev_state.cpu().reshape(ref_state.shape), ref_state)
                    assert su.max() <= 1, f"{opt} step {step} tensor {k} {name}: max {su.max()} ulp"
            tref = tparams[k].detach()
            # an update that cancels p leaves the few-ulp error of the larger magnitudes
            hist[k] = torch.maximum(hist[k], prev[k].abs() + (tref - prev[k]).abs())
            scale = hist[k]
            err = (got - tref).abs()
            worst = int((err / scale).reshape(-1).argmax())
            assert bool((err <= 2.0 ** -18 * scale).all()), \
                (f"{opt} step {step} tensor {k}: vs torch.optim max err/scale {float((err / scale).max()):.3g} "
                 f"at {worst}: got {float(got.reshape(-1)[worst])!r} torch {float(tref.reshape(-1)[worst])!r} "
                 f"prev gpu {float(p0.reshape(-1)[worst])!r} prev torch {float(prev[k].reshape(-1)[worst])!r} "
                 f"g {float(grads[k].reshape(-1)[worst])!r}")


def test_scores_and_val_loss(dev):
    e, o = run_parity(dev, 300, 200, 64, 128, 5, "pointwise", "adam")
    rs = np.random.RandomState(1)
    u, i = rs.randint(0, 300, 1000), rs.randint(0, 200, 1000)
    got = e.scores(torch.from_numpy(u), torch.from_numpy(i))
    ref = omf.scores(*o.params, torch.from_numpy(u), torch.from_numpy(i))
    close(got, ref, what="scores")
    vu, vi = rs.randint(0, 300, 100), rs.randint(0, 200, 100)
    got = e.val_loss(torch.from_numpy(vu).to(dev), torch.from_numpy(vi).to(dev))
    ref = omf.val_loss(o, vu, vi)
    torch.cuda.synchronize()
    close(got[0], np.float32(ref), what="val loss")
    assert (e.mt_state() == o.state).all()


def test_large_full_size_properties(dev):
    """ML-20M-shaped step at full size: finite loss, scratch invariants, determinism of the
    sampler stream, and loss decreasing over a few steps on a fixed batch."""
    from recommendation_gans_amd.mf_engine import MFEngine
    U, I, d, B, n = 136_677, 20_108, 64, 8192, 5
    torch.manual_seed(0)
    Uw, Iw = torch.randn(U, d) / d, torch.randn(I, d) / d
    rs = np.random.RandomState(0)
    P = 1_000_000
    e = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), rs.randint(0, U, P), rs.randint(0, I, P),
                 orng.py_seed_state(0), loss="bpr", optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n,
                 batch_size=B, device=dev)
    pu = torch.from_numpy(rs.randint(0, U, B)).to(dev)
    pi = torch.from_numpy(rs.randint(0, I, B)).to(dev)
    losses = [float(e.train_step(pu, pi)[0]) for _ in range(5)]
    assert all(np.isfinite(losses))
    assert int(e.row_count.abs().sum()) == 0
    st = orng.py_seed_state(0)
    orng.py_choices_indices(st, P, 5 * n * B)
    assert (e.mt_state() == st).all()


@pytest.mark.parametrize("jump", [0, 1, "inline"])
@pytest.mark.parametrize("n", [5, 8])
def test_full_size_sampler_steps(dev, n, jump, monkeypatch):
    """Full-size steps through the stepper's word ring (chunks generated two steps
    ahead), with the plain walk or (RG_MT_JUMP=1) the jump-ahead sampler (head +
    XOR-of-windows jump + parallel tail segments; rg_mtjump.cpp).  With prefetch, a
    validation draw in between (takes the next chunk; the prepared pairs are redone),
    export and re-import of the state: negative pairs bit-exact, MT state exact,
    losses/tables as the oracle."""
    from recommendation_gans_amd.mf_engine import MFEngine
    # "inline": one-unit slots, unit t+2 walked inside step t's dense pass (forced at this size)
    monkeypatch.setenv("RG_MT_JUMP", "1" if jump == 1 else "0")
    monkeypatch.setenv("RG_MT_INLINE", "2" if jump == "inline" else "0")
    U, I, d, B = 300, 200, 16, 8192
    g = torch.Generator().manual_seed(3)
    tabs = [torch.randn(U, d, generator=g) / d, torch.randn(I, d, generator=g) / d,
            torch.zeros(U, 1), torch.zeros(I, 1)]
    rs = np.random.RandomState(3)
    pool_u, pool_i = rs.randint(0, U, 20000), rs.randint(0, I, 20000)
    st = orng.py_seed_state(9)
    st[624] = 300                                   # start mid-block
    o = omf.MFOracle(*[t.clone() for t in tabs], pool_u, pool_i, st.copy(), loss="bpr", optimizer="adam",
                     lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    o64 = omf.MFOracle(*[t.clone().double() for t in tabs], pool_u, pool_i, st.copy(), loss="bpr", optimizer="adam",
                       lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    e = MFEngine(tabs[0], tabs[1], tabs[2].reshape(-1), tabs[3].reshape(-1), pool_u, pool_i, st.copy(), loss="bpr",
                 optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
    batches = [(rs.randint(0, U, B), rs.randint(0, I, B)) for _ in range(5)]
    dbat = [(torch.from_numpy(u).to(dev), torch.from_numpy(i).to(dev)) for u, i in batches]
    for s in range(4):
        nxt = e.step_input(*dbat[s + 1]) if s < 3 else None
        out = o.step(*batches[s], return_all=True)
        o64.step(*batches[s])
        got = e.train_step(*dbat[s], next_input=nxt)
        torch.cuda.synchronize()
        close(got[0], np.float32(out["loss"]), what=f"jump step {s} loss")
        # the consumed pairs buffer of this step: negatives (q >= 1) in draw order
        found = False
        for buf in e.pairs:
            S = 8 if n + 2 <= 8 else 16                              # per-column records (rg_mf_pairs_len)
            pr = buf.view(B, S, 2)[:, :1 + n].transpose(0, 1).cpu().numpy() & 0x07FFFFFF   # minus ownership flags / claimed slots (bits 27-31)
            if (pr[1:, :, 0].reshape(-1) == out["neg_u"].numpy()).all() and \
               (pr[1:, :, 1].reshape(-1) == out["neg_i"].numpy()).all():
                found = True
        assert found, f"step {s}: negative pairs differ from random.choices"
        if s == 1:                                  # validation draw between steps (discards the prefetch)
            vu, vi = batches[4]
            vl = e.val_loss(torch.from_numpy(vu).to(dev), torch.from_numpy(vi).to(dev))
            ref = omf.val_loss(o, vu, vi)
            omf.val_loss(o64, vu, vi)
            torch.cuda.synchronize()
            close(vl[0], np.float32(ref), what="jump val loss")
        assert (e.mt_state() == o.state).all(), f"step {s}: MT state"
        if s == 2:
            e.set_mt_state(o.state)                 # import (back to CPython form)
    for k in range(4):
        ok, msg = omf.tensor_parity(e.params()[k], o.params[k], o64.params[k])
        assert ok, (k, msg)


@pytest.mark.parametrize("rank", [0, 5])
def test_dp_rank_slice_sampler_full_size(dev, rank):
    """Rank `rank` of 8 in the replicated DP layout at full size (B = 8192 per rank, global
    draw of 5 * 65,536 indices per step, the jump-ahead walk that layout defaults to at
    world > 1: 5.2 M words per 8-step slot in parallel segments): its prepared negatives
    are columns [rank*B, (rank+1)*B) of random.choices' global draw, bit-exact, and the MT
    state after each step is CPython's.  (Identity exchange: tables are not checked here.)"""
    from recommendation_gans_amd.mf_engine import MFEngine
    U, I, d, B, n, world = 300, 200, 16, 8192, 5, 8
    g = torch.Generator().manual_seed(5)
    tabs = [torch.randn(U, d, generator=g) / d, torch.randn(I, d, generator=g) / d, torch.zeros(U), torch.zeros(I)]
    rs = np.random.RandomState(5)
    pool_u, pool_i = rs.randint(0, U, 30000), rs.randint(0, I, 30000)
    st = orng.py_seed_state(11)
    e = MFEngine(*tabs, pool_u, pool_i, st.copy(), loss="bpr", optimizer="adam", lr=1e-2, weight_decay=1e-5,
                 n_neg=n, batch_size=B, device=dev, rank=rank, world_size=world, dp="global_stream")
    assert e.words_per_step == 2 * n * B * world
    ref = st.copy()
    none = lambda *a: None   # noqa: E731
    ins = [e.step_input(torch.from_numpy(rs.randint(0, U, B)).to(dev), torch.from_numpy(rs.randint(0, I, B)).to(dev),
                        B * world) for _ in range(10)]
    for s in range(9):
        e.train_step_exchange(ins[s], ins[s + 1], none, none)
        idx = orng.py_choices_indices(ref, len(pool_u), n * B * world).reshape(n, B * world)[:, rank * B:(rank + 1) * B]
        pr = e.pairs[s % 2].view(B, 8, 2)[:, 1:1 + n].transpose(0, 1).cpu().numpy() & 0x07FFFFFF
        assert (pr[..., 0] == pool_u[idx]).all() and (pr[..., 1] == pool_i[idx]).all(), f"step {s} negatives"
        assert (e.mt_state() == ref).all(), f"step {s} MT state"


def test_mf_steps_bit_reproducible(dev):
    """Two runs of the same MF steps give bit-identical tables: list entries are summed in
    (partner, dz) order, overflowed rows in int64 fixed point -- whatever order the slot
    atomics arrived in.  Small tables so that rows overflow their lists every step."""
    from recommendation_gans_amd.mf_engine import MFEngine
    U, I, d, B, n = 300, 200, 32, 1024, 5
    tabs, pool_u, pool_i, steps = make_case(U, I, d, B, n, 4000, 3, hot_items=True)
    st = orng.py_seed_state(7)
    out = []
    for rep in range(2):
        e = MFEngine(tabs[0], tabs[1], tabs[2].reshape(-1), tabs[3].reshape(-1), pool_u, pool_i, st.copy(),
                     loss="bpr", optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev)
        for k, (pu, pi) in enumerate(steps):
            di = torch.from_numpy(pi).to(dev)
            e.train_step(torch.from_numpy(pu).to(dev), di, plan=e.make_plan(di) if k % 2 else None)
        torch.cuda.synchronize()
        out.append([p.cpu().clone() for p in e.params()])
    for a, b in zip(*out):
        assert torch.equal(a, b)
