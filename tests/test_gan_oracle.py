"""oracle/gan.py against the reference's own cGAN steps (tests/golden/gan_*.npz):
five or six discriminator steps and the generator step after the fifth, with the
recorded z and dropout masks.  D outputs, fake slates, losses, BatchNorm running
stats and inference slates; every parameter after every step (see ``param_ok``).
``gan_rms_refinit`` keeps the reference's own D init (clamp-bound, see
make_golden.gan_case): step-0 forward values and the clamp only."""
import os

import numpy as np
import pytest

from oracle import gan as og

CASES = ["gan_rms_n50", "gan_adam_n50", "gan_sgd_n64"]


def load(golden_dir, case):
    z = np.load(os.path.join(golden_dir, case + ".npz"))
    N, S, H, E, B, L, Z, nb, dsteps = (int(x) for x in z["meta"])
    gp = [str(x) for x in z["g_param_names"]]
    gb = [str(x) for x in z["g_buffer_names"]]
    dn = [str(x) for x in z["d_param_names"]]
    g_init = {k: z["g_init_" + k.replace(".", "_")] for k in gp + gb}
    d_init = {k: z["d_init_" + k.replace(".", "_")] for k in dn}
    return z, (N, S, H, E, B, L, Z, nb, dsteps), gp, gb, dn, g_init, d_init


def key(prefix, name):
    return prefix + name.replace(".", "_")


def param_ok(got, ref, grad, lr, exempt=False, rtol=1e-5, prior=None):
    """||got - ref|| <= rtol ||ref||, or every element off by more than rtol * max|ref|
    is ill-conditioned: its float64 gradient cancelled to below 1e-3 of the
    tensor's largest, or to within 100 eps of zero (RMSprop/Adam then move it by
    lr * g / (|g| + eps), set by the last bits of the cancelled fp32 sum) — and such
    an element still moved by at most the step's bound.  ``prior``: elements found
    ill-conditioned at an earlier step (their optimizer state carries that noise);
    updated in place.  ``exempt`` (pre-BatchNorm biases, zero gradient) checks the bound only."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    err = np.linalg.norm(got - ref)
    if not exempt and err <= rtol * max(np.linalg.norm(ref), 1e-30):
        return True, f"rel {err / max(np.linalg.norm(ref), 1e-30):.1e}"
    bad = np.abs(got - ref) > rtol * max(np.abs(ref).max(), 1e-30)
    if exempt:
        return bool(np.all(np.abs(got - ref) <= 30 * lr)), "pre-BN bias bound"
    g = np.abs(np.asarray(grad, np.float64))
    ill = g < 1e-3 * max(g.max(), 1e-30) + 1e-6
    if prior is not None:
        ill |= prior
        prior |= ill
    ok = bool(np.all(ill[bad]) and np.all(np.abs(got - ref)[bad] <= 30 * lr))
    return ok, f"rel {err / max(np.linalg.norm(ref), 1e-30):.1e}, {int(bad.sum())} ill-conditioned of {bad.size}"


@pytest.mark.parametrize("case", CASES)
def test_gan_oracle_matches_reference(golden_dir, case):
    z, (N, S, H, E, B, L, Z, nb, dsteps), gp, gb, dn, g_init, d_init = load(golden_dir, case)
    lr = float(z["lr"][0])
    o = og.GANOracle(g_init, d_init, N, S, H, E, Z, opt=case.split("_")[1], lr=lr)
    scales = tuple(float(x) for x in z["drop_scale"])
    assert scales == (np.float32(1) / np.float32(0.9), np.float32(1) / np.float32(0.7))
    gat = int(z["g_step_at"][0])
    ill = {}
    for k in range(dsteps):
        b = int(z[f"d{k}_batch"][0])
        hist, sl = z["hist"][b * B:(b + 1) * B], z["slates"][b * B:(b + 1) * B]
        masks = [z[f"d{k}_mask{j}"].astype(np.float64) for j in range(8)]
        loss, dr, df, fake = o.d_step(hist, sl, z[f"d{k}_z"].astype(np.float64), masks, scales)
        np.testing.assert_allclose(dr, z[f"d{k}_d_real"], rtol=1e-5, err_msg=f"{case} D{k} real")
        np.testing.assert_allclose(df, z[f"d{k}_d_fake"], rtol=1e-5, err_msg=f"{case} D{k} fake")
        np.testing.assert_allclose(fake, z[f"d{k}_fake"], rtol=1e-4, atol=1e-5, err_msg=f"{case} D{k} G(z)")
        # d_loss is a difference of two near-equal means: absolute, at the means' scale
        assert abs(loss - z[f"d{k}_loss"][0]) <= 1e-5 * abs(dr).mean()
        for n in dn:
            ok, msg = param_ok(o.D[n], z[key(f"d{k}_after_D_", n)], o.last_grads[n], lr,
                               prior=ill.setdefault("D" + n, np.zeros(o.D[n].shape, bool)))
            assert ok, f"{case} D{k} {n}: {msg}"
        for n in gb:
            np.testing.assert_allclose(o.G[n], z[key(f"d{k}_after_G_", n)], rtol=1e-5, atol=1e-7,
                                       err_msg=f"{case} D{k} {n}")
        if k == gat:
            masks = [z[f"g{k}_mask{j}"].astype(np.float64) for j in range(5)]
            gl, dfk, slates = o.g_step(hist, z[f"g{k}_z"].astype(np.float64), masks, scales)
            np.testing.assert_allclose(gl, z[f"g{k}_loss"][0], rtol=1e-5)
            np.testing.assert_allclose(dfk, z[f"g{k}_d_fake"], rtol=1e-5)
            assert (slates == z[f"g{k}_slates_after"]).all()
            # the reference's training precision/recall: identity-hashed tensors, always 0
            assert not z[f"g{k}_precision"].any() and not z[f"g{k}_recall"].any()
            for n in gp:
                ok, msg = param_ok(o.G[n], z[key(f"g{k}_after_G_", n)], o.last_grads[n], lr,
                                   exempt=n in o.pre_bn_biases(),
                                   prior=ill.setdefault("G" + n, np.zeros(o.G[n].shape, bool)))
                assert ok, f"{case} G{k} {n}: {msg}"
            for n in gb:
                np.testing.assert_allclose(o.G[n], z[key(f"g{k}_after_G_", n)], rtol=1e-5, atol=1e-7)


def test_gan_oracle_reference_init_forward(golden_dir):
    z, (N, S, H, E, B, L, Z, nb, dsteps), gp, gb, dn, g_init, d_init = load(golden_dir, "gan_rms_refinit")
    o = og.GANOracle(g_init, d_init, N, S, H, E, Z, opt="rms", lr=float(z["lr"][0]))
    scales = tuple(float(x) for x in z["drop_scale"])
    masks = [z[f"d0_mask{j}"].astype(np.float64) for j in range(8)]
    loss, dr, df, fake = o.d_step(z["hist"][:B], z["slates"][:B], z["d0_z"].astype(np.float64), masks, scales)
    np.testing.assert_allclose(dr, z["d0_d_real"], rtol=1e-5)
    np.testing.assert_allclose(df, z["d0_d_fake"], rtol=1e-5)
    np.testing.assert_allclose(fake, z["d0_fake"], rtol=1e-4, atol=1e-5)
    assert abs(loss - z["d0_loss"][0]) <= 1e-5 * abs(dr).mean()
    # the clamp bound nearly every D weight: the step moved each by at most lr / sqrt(1 - alpha)
    for n in dn:
        before = np.clip(d_init[n], -og.CLAMP, og.CLAMP)
        assert np.abs(z["d0_after_D_" + n.replace(".", "_")] - before).max() <= 10 * float(z["lr"][0]) * (1 + 1e-5)
    assert (np.abs(d_init["layers.0.weight"]) > og.CLAMP).mean() > 0.5


def test_gan_oracle_reference_init_cycle(golden_dir):
    """gan_rms_refinit5: the reference's own init (the D clamp binding), lr
    1e-3, a whole n_critic cycle (5 D iterations, the G iteration after the 5th, a 6th D
    iteration).  Free-running from the same init, the float64 restatement tracks the
    reference's fp32 steps: D outputs, G(z) and losses at every step, and every D and G tensor
    after every step within 1e-5 relative (tensor norm) -- except the two Linear biases feeding
    a BatchNorm, whose gradient is analytically zero: there every implementation moves by its
    own rounding noise through RMSprop's g / (sqrt(v) + eps), so they are held to the step's
    bound and their distance is reported, not exempted silently."""
    z, (N, S, H, E, B, L, Z, nb, dsteps), gp, gb, dn, g_init, d_init = load(golden_dir, "gan_rms_refinit5")
    lr = float(z["lr"][0])
    assert lr == 1e-3 and dsteps == 6 and int(z["g_step_at"][0]) == 4
    assert (np.abs(d_init["layers.0.weight"]) > og.CLAMP).mean() > 0.5
    o = og.GANOracle(g_init, d_init, N, S, H, E, Z, opt="rms", lr=lr)
    scales = tuple(float(x) for x in z["drop_scale"])

    def rel(a, b):
        return np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30)
    for k in range(dsteps):
        b = int(z[f"d{k}_batch"][0])
        hist, sl = z["hist"][b * B:(b + 1) * B], z["slates"][b * B:(b + 1) * B]
        masks = [z[f"d{k}_mask{j}"].astype(np.float64) for j in range(8)]
        loss, dr, df, fake = o.d_step(hist, sl, z[f"d{k}_z"].astype(np.float64), masks, scales)
        np.testing.assert_allclose(dr, z[f"d{k}_d_real"], rtol=1e-5)
        np.testing.assert_allclose(df, z[f"d{k}_d_fake"], rtol=1e-5)
        assert np.abs(fake - z[f"d{k}_fake"]).max() <= 1e-5 * np.abs(z[f"d{k}_fake"]).max()
        assert abs(loss - z[f"d{k}_loss"][0]) <= 1e-5 * abs(dr).mean()
        for n in dn:
            assert rel(o.D[n], z[key(f"d{k}_after_D_", n)]) <= 1e-5, (k, n)
        if k == 4:
            masks = [z[f"g{k}_mask{j}"].astype(np.float64) for j in range(5)]
            gl, dfk, slates = o.g_step(hist, z[f"g{k}_z"].astype(np.float64), masks, scales)
            np.testing.assert_allclose(gl, z[f"g{k}_loss"][0], rtol=1e-5)
            assert (slates == z[f"g{k}_slates_after"]).all()
            for n in gp + gb:
                r = rel(o.G[n], z[key(f"g{k}_after_G_", n)])
                if n in o.pre_bn_biases():
                    assert np.abs(o.G[n] - z[key(f"g{k}_after_G_", n)]).max() <= lr, (n, r)
                else:
                    assert r <= 1e-5, (n, r)
