"""oracle.mf.elementwise_parity: the elementwise rule behind the full-size GPU tests."""
import torch

from oracle import mf as omf


def test_elementwise_catches_what_the_norm_hides():
    torch.manual_seed(0)
    r32 = torch.randn(1_000_000) / 64
    r64 = r32.double() + torch.randn(1_000_000).double() * 1e-9
    got = r32.clone()
    got[123] *= 1.003                         # one element 0.3 % off: the norm rule still passes
    ok_n, _ = omf.tensor_parity(got, r32, r64)
    ok_e, st = omf.elementwise_parity(got, r32, r64)
    assert ok_n and not ok_e
    assert st["n_out"] == 1 and st["n_fail"] == 1 and abs(st["frac_out"] - 1e-6) < 1e-12


def test_elementwise_band_and_operand_rules():
    r64 = torch.tensor([1.0, 2.0, 1e-3, 0.0], dtype=torch.float64)
    r32 = torch.tensor([1.0, 2.0, 1.2e-3, 0.0])          # the fp32 reference itself 20 % off on [2]
    got = torch.tensor([1.0 + 5e-6, 2.0, 0.85e-3, 1e-12])   # [2]: outside 1e-5 of r32, inside the band
    ok, st = omf.elementwise_parity(got, r32, r64)
    assert ok and st["n_out"] == 1 and st["n_fail"] == 0
    got[2] = 2e-3                                          # 5x the fp32 reference's distance from fp64
    assert not omf.elementwise_parity(got, r32, r64)[0]
    before = torch.tensor([1.0, 2.0, 1.0, 0.0])            # a cancelled step: judged on the operand
    got[2] = 1.2e-3 + 5e-6
    assert omf.elementwise_parity(got, r32, None, before=before)[0]


def test_mf_noise_band_covers_other_fp32_orders():
    """The float64 oracle's noise band (MFOracle(noise=True)) holds every element of two fp32
    restatements that sum the gradients in different orders (the reference's index order and
    the reverse), over three steps with Zipf-hot items overflowing any per-row list: the
    elementwise rule the full-size GPU tests apply cannot fail an fp32 result for its order."""
    import numpy as np
    from oracle import rng as orng
    torch.manual_seed(0)
    U, I, d, B, n = 3000, 400, 64, 1024, 5
    tabs = omf.init_tables(U, I, d)
    rs = np.random.RandomState(1)
    pool_u, pool_i = rs.randint(0, U, 20000), rs.randint(0, I, 20000)
    items = np.minimum((rs.zipf(1.3, 3 * B) - 1), I - 1)
    users = rs.randint(0, U, 3 * B)
    for loss in ("bpr", "pointwise"):
        kw = dict(loss=loss, optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
        st = orng.py_seed_state(0)
        fp32 = [omf.MFOracle(*[t.clone() for t in tabs], pool_u, pool_i, st.copy(), **kw) for _ in range(4)]
        r = omf.MFOracle(*[t.clone().double() for t in tabs], pool_u, pool_i, st.copy(), noise=True, **kw)
        for j, o in enumerate(fp32[1:]):          # the reverse and two random orders of the gradient sums
            g = torch.Generator().manual_seed(j)

            def perm_grads(U_, I_, ub, ib, u, i, dz, j=j, g=g):
                pr = torch.arange(len(u) - 1, -1, -1) if j == 0 else torch.randperm(len(u), generator=g)
                return omf.dense_grads(U_, I_, ub, ib, u[pr], i[pr], dz[pr])
            o.grads_fn = perm_grads
        for s in range(3):
            for o in fp32 + [r]:
                o.step(users[s * B:(s + 1) * B], items[s * B:(s + 1) * B])
            for k in range(4):
                r64, nz = r.params[k].reshape(-1), r.noise[k].reshape(-1)
                fl = 1e-8 * float(r64.abs().max())
                for o in fp32:
                    ok, st_ = omf.elementwise_parity(o.params[k], fp32[0].params[k], r.params[k], noise=r.noise[k])
                    assert ok, (loss, s, k, st_)
                    # and with room to spare: the deviation stays a quarter of the band
                    dev = (o.params[k].double().reshape(-1) - r64).abs()
                    assert float((dev / (1e-5 * r64.abs() + 2 * nz + fl)).max()) < 0.25, (loss, s, k)


def test_ncf_two_order_band_covers_a_third_order():
    """NCF / NeuMF (no noise model): the band is the larger distance from float64 of two fp32
    restatements that sum over the examples in different orders; a third order stays inside it."""
    import numpy as np
    from oracle import ncf as oncf
    from oracle import rng as orng
    torch.manual_seed(0)
    U, I, E, B, n = 2000, 300, 16, 512, 5
    sizes = oncf.layer_sizes(E)
    params = [torch.randn(U, E), torch.randn(I, E)]
    for a_, b_ in zip(sizes[:-1] + [sizes[-1]], sizes[1:] + [1]):
        w = torch.empty(b_, a_)
        torch.nn.init.xavier_uniform_(w)
        params += [w, torch.full((b_,), 0.01)]
    names = [f"p{k}" for k in range(len(params))]
    rs = np.random.RandomState(0)
    pool_u, pool_i = rs.randint(0, U, 20000), rs.randint(0, I, 20000)
    kw = dict(loss="pointwise", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
    st = orng.py_seed_state(0)
    a = oncf.NCFOracle([t.clone() for t in params], names, pool_u, pool_i, st.copy(), **kw)
    b = oncf.NCFOracle([t.clone() for t in params], names, pool_u, pool_i, st.copy(), order_seed=1, **kw)
    c = oncf.NCFOracle([t.clone() for t in params], names, pool_u, pool_i, st.copy(), order_seed=2, **kw)
    r = oncf.NCFOracle([t.double() for t in params], names, pool_u, pool_i, st.copy(), **kw)
    # the reordered restatement is the same function: in float64 it lands on the canonical one
    r2 = oncf.NCFOracle([t.double() for t in params], names, pool_u, pool_i, st.copy(), order_seed=3, **kw)
    widths = sizes[1:]
    for s in range(3):
        pu, pi = rs.randint(0, U, B), np.minimum(rs.zipf(1.3, B) - 1, I - 1)
        mp = [torch.from_numpy((rs.rand(B, w_) >= 0.5).astype(np.uint8)) for w_ in widths]
        mn = [torch.from_numpy((rs.rand(n * B, w_) >= 0.5).astype(np.uint8)) for w_ in widths]
        for o in (a, b, c, r, r2):
            o.step(pu, pi, mp, mn)
        for k in range(len(params)):
            ok, st_ = omf.elementwise_parity(c.P.t[k], a.P.t[k], r.P.t[k], alt32=b.P.t[k])
            assert ok, (s, k, st_)
            assert torch.allclose(r2.P.t[k], r.P.t[k], rtol=1e-9, atol=1e-12), (s, k)


def _neumf_small(E=8, M=6, U=1500, I=200):
    import numpy as np
    from oracle import ncf as oncf
    torch.manual_seed(1)
    sizes = oncf.layer_sizes(E)
    params = [torch.randn(U, E), torch.randn(I, E), torch.randn(U, M), torch.randn(I, M)]
    ins = sizes[:-1]
    outs = sizes[1:]
    for a_, b_ in zip(ins, outs):
        w = torch.empty(b_, a_)
        torch.nn.init.xavier_uniform_(w)
        params += [w, torch.full((b_,), 0.01)]
    w = torch.empty(1, sizes[-1] + M)
    torch.nn.init.xavier_uniform_(w)
    params += [w, torch.full((1,), 0.01)]
    rs = np.random.RandomState(3)
    return params, [f"p{k}" for k in range(len(params))], rs.randint(0, U, 8000), rs.randint(0, I, 8000), sizes[1:]


def test_neumf_unit_orders_and_kink_flips():
    """NeuMF's further fp32 samples (oracle/ncf.py): order_seed re-orders the examples, the
    tower's input features and hidden units (forward and backward inner sums) -- in float64 the
    same function as the canonical order; kink_flip decides the LeakyReLUs within rounding of the
    kink the other way -- with c = 0 it is the canonical restatement bit for bit, with c = 4 it
    flips a few decisions a step (counted in .flips) and moves only the rows they touch."""
    import numpy as np
    from oracle import ncf as oncf
    from oracle import rng as orng
    params, names, pool_u, pool_i, widths = _neumf_small()
    U, I = params[0].shape[0], params[1].shape[0]
    B, n = 512, 5
    kw = dict(loss="pointwise", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
    st = orng.py_seed_state(0)

    def mk(dtype, **k):
        return oncf.NeuMFOracle([t.to(dtype).clone() for t in params], names, pool_u, pool_i, st.copy(), **kw, **k)
    r, r2 = mk(torch.float64), mk(torch.float64, order_seed=3)
    a, a0, f = mk(torch.float32), mk(torch.float32, kink_flip=0.0), mk(torch.float32, kink_flip=4.0)
    f64 = mk(torch.float64, kink_flip=1e9)   # every kept decision flipped: a different function
    rs = np.random.RandomState(0)
    for s in range(3):
        pu, pi = rs.randint(0, U, B), np.minimum(rs.zipf(1.3, B) - 1, I - 1)
        mp = [torch.from_numpy((rs.rand(B, w_) >= 0.5).astype(np.uint8)) for w_ in widths]
        mn = [torch.from_numpy((rs.rand(n * B, w_) >= 0.5).astype(np.uint8)) for w_ in widths]
        for o in (r, r2, a, a0, f, f64):
            o.step(pu, pi, mp, mn)
        for k in range(len(params)):
            assert torch.allclose(r2.P.t[k], r.P.t[k], rtol=1e-9, atol=1e-12), (s, k)
            assert torch.equal(a0.P.t[k], a.P.t[k]), (s, k)
    assert a0.flips == [0, 0, 0]
    assert f64.flips[0] > 1000
    assert not torch.allclose(f64.P.t[4], r.P.t[4], rtol=1e-4)
    # the c = 4 sample: a handful of flips at most at this size, each moving its example's rows only
    assert sum(f.flips) <= 20
    moved = (f.P.t[0].double() - r.P.t[0]).abs().max(1).values > 1e-5
    assert int(moved.sum()) <= 2 * sum(f.flips) + 1


def test_kink_band_covers_seeded_orders():
    """kink_flip's c = 4: the distance of a seeded-order fp32 pre-activation from its exact value is
    within one band width (c = 1) on every decision of a batch; c = 4 leaves a 4x margin."""
    from oracle import ncf as oncf
    torch.manual_seed(2)
    K, N, H = 128, 4096, 64
    a = torch.randn(N, K)
    W = torch.empty(H, K)
    torch.nn.init.xavier_uniform_(W)
    b = torch.full((H,), 0.01)
    z64, band = oncf.kink_band(a, W, b, 1.0)
    for seed in range(3):
        p = torch.randperm(K, generator=torch.Generator().manual_seed(seed))
        z32 = a[:, p].mm(W[:, p].t()) + b
        assert float(((z32.double() - z64).abs() / band).max()) <= 1.0


def test_kink_envelope_covers_the_kink_flip_sample():
    """NCFOracle(kink_env=c) (float64): its per-element bound on what flipping any subset of the
    step's rounding-level LeakyReLU decisions moves after Adam covers the fp32 sample that flips
    ALL of them (kink_flip=c) on every element of every parameter, from the same state; without
    the envelope the same sample falls outside the two-order band.  NeuMF at a small size, one
    step from a state three steps in.  c = 200 (fifty times the tests' 4) so that this small batch
    has flips to check."""
    import numpy as np
    C = 200.0
    from oracle import ncf as oncf
    from oracle import rng as orng
    params, names, pool_u, pool_i, widths = _neumf_small(E=16, M=8, U=3000, I=400)
    B, n = 2048, 5
    kw = dict(loss="pointwise", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)
    rs = np.random.RandomState(4)

    def batch():
        pu, pi = rs.randint(0, 3000, B), np.minimum(rs.zipf(1.3, B) - 1, 399)
        mp = [torch.from_numpy((rs.rand(B, w_) >= 0.5).astype(np.uint8)) for w_ in widths]
        mn = [torch.from_numpy((rs.rand(n * B, w_) >= 0.5).astype(np.uint8)) for w_ in widths]
        return pu, pi, mp, mn
    run = oncf.NeuMFOracle([t.clone() for t in params], names, pool_u, pool_i, orng.py_seed_state(0), **kw)
    for _ in range(3):
        run.step(*batch())
    ps, st, t = [p.clone() for p in run.P.t], run.state.copy(), run.opt.t
    mom = [(m.clone(), v.clone()) for m, v in run.opt.state]

    def mk(dtype, **k):
        o = oncf.NeuMFOracle([p.to(dtype).clone() for p in ps], names, pool_u, pool_i, st.copy(), **kw, **k)
        o.opt.t, o.opt.state = t, [(m.to(dtype).clone(), v.to(dtype).clone()) for m, v in mom]
        return o
    r32, r64 = mk(torch.float32), mk(torch.float64, kink_env=C)
    alts = [mk(torch.float32, order_seed=k) for k in (1, 2)]
    flip = mk(torch.float32, kink_flip=C)
    b = batch()
    for o in [r32, r64, flip] + alts:
        o.step(*b)
    assert r64.kink_count[-1] == flip.flips[-1] > 0
    fail_env = fail_band = 0
    for k in range(len(names)):
        _, s1 = omf.elementwise_parity(flip.P.t[k], r32.P.t[k], r64.P.t[k], alt32=[a.P.t[k] for a in alts],
                                       kink=r64.kink_noise[k])
        _, s2 = omf.elementwise_parity(flip.P.t[k], r32.P.t[k], r64.P.t[k], alt32=[a.P.t[k] for a in alts])
        fail_env += s1["n_fail"]
        fail_band += s2["n_fail"]
    assert fail_env == 0 and fail_band > 0, (fail_env, fail_band)
