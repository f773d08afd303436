"""Pin the oracle (oracle/) against golden vectors produced by the reference itself.

CPU-only; no GPU.  The fixtures come from tests/golden/make_golden.py, which
imports the reference (Stamatios-Korres/recommendation_Gans) in the build container.
"""
import glob
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import mf as omf
from oracle import rng as orng

RTOL = 1e-5   # north_star: loss/embeddings within 1e-5 relative (fp32)


def _close(a, b, rtol=RTOL, atol=1e-7):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


# ------------------------------------------------------------------ RNG
def test_cpython_choices_bit_exact(golden_dir):
    g = np.load(os.path.join(golden_dir, "rng_golden.npz"))
    seeds = [0, 1, 12345, 2 ** 40 + 7]
    for si, s in enumerate(seeds):
        st = orng.py_seed_state(s)
        assert (st == g[f"py_state_seed{si}"]).all()
        for ni, n in enumerate(g["py_ns"]):
            idx = orng.py_choices_indices(st, int(n), 700)
            assert (idx == g[f"py_choices_s{si}_n{ni}"]).all(), (s, n)
        assert (st == g[f"py_state_end{si}"]).all()


def test_cpython_choices_mid_block(golden_dir):
    g = np.load(os.path.join(golden_dir, "rng_golden.npz"))
    st = g["py_mid_state"].copy()
    assert (orng.py_choices_indices(st, 40960, 5000) == g["py_mid_choices"]).all()


def test_numpy_legacy(golden_dir):
    g = np.load(os.path.join(golden_dir, "rng_golden.npz"))
    st = orng.np_seed_state(0)
    assert orng.np_randint(st, -10 ** 8, 10 ** 8, 1)[0] == g["np_seed0_randint"][0] == 30329135
    for n in [1, 2, 10, 1000, 100003]:
        assert (orng.np_shuffle_indices(orng.np_seed_state(0), n) == g[f"np_shuffle_{n}"]).all()
    st = orng.np_seed_state(7)
    assert (orng.np_randint(st, 0, 136677, 3000) == g["np_choice_u"]).all()
    assert (orng.np_randint(st, 0, 20108, 3000) == g["np_choice_i"]).all()
    st = orng.np_seed_state(0)
    assert orng.np_randint(st, -10 ** 8, 10 ** 8, 1)[0] == g["np_model_seed"][0]
    assert (orng.np_shuffle_indices(st, 5000) == g["np_model_shuffle_5000"]).all()


def test_negative_pool(golden_dir):
    g = np.load(os.path.join(golden_dir, "pool_golden.npz"))
    nu, ni, k = (int(x) for x in g["shape"])
    for tag, rating in (("raw4", 4.0), ("ones", 1.0)):
        csr = sp.coo_matrix((np.full(len(g["pos_u"]), rating), (g["pos_u"], g["pos_i"])),
                            shape=(nu, ni)).tocsr()
        st = orng.np_seed_state(11)
        u, i = orng.negative_pool(st, nu, ni, k, positive_csr=csr)
        ref = g[f"{tag}_pool"]
        assert (u == ref[:, 0]).all() and (i == ref[:, 1]).all(), tag
    # the has_key-True branch must actually have been exercised by the "ones" fixture
    assert not (g["ones_pool"] == g["raw4_pool"]).all()


# ------------------------------------------------------------------ MF steps
MF_FIXTURES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "mf_*_*_d*.npz")))


def _mf_cfg(path):
    base = os.path.basename(path)[3:-4]
    parts = base.split("_")
    if parts[0] == "adaptive":
        loss, rest = "adaptive_hinge", parts[2:]
    else:
        loss, rest = parts[0], parts[1:]
    return loss, rest[0]


def replay_mf(path, make_oracle):
    g = np.load(path)
    U, I, d, B, n = (int(x) for x in g["meta"])
    loss, opt = _mf_cfg(path)
    params = [torch.from_numpy(g[k].copy()) for k in
              ("init_user_embeddings_weight", "init_item_embeddings_weight",
               "init_user_biases_weight", "init_item_biases_weight")]
    st = g["s0_mt_state"].copy()
    o = make_oracle(params, g["pool_u"], g["pool_i"], st, loss, opt, float(g["lr"][0]),
                    float(g["wd"][0]), n, B)
    return g, o


@pytest.mark.parametrize("path", MF_FIXTURES, ids=[os.path.basename(p) for p in MF_FIXTURES])
def test_mf_step_oracle_vs_reference(path):
    def mk(params, pu, pi, st, loss, opt, lr, wd, n, B):
        return omf.MFOracle(*params, pu, pi, st, loss=loss, optimizer=opt, lr=lr,
                            weight_decay=wd, n_neg=n, batch_size=B)

    g, o = replay_mf(path, mk)
    names = ["user_embeddings_weight", "item_embeddings_weight", "user_biases_weight", "item_biases_weight"]
    for s in range(3):
        assert (o.state == g[f"s{s}_mt_state"]).all()
        out = o.step(g[f"s{s}_pos_u"], g[f"s{s}_pos_i"], return_all=True)
        assert (out["neg_idx"] == g[f"s{s}_neg_idx"]).all()
        _close(out["p_pos"], g[f"s{s}_p_pos"])
        _close(out["p_neg"], g[f"s{s}_p_neg"])
        _close(out["loss"], g[f"s{s}_loss"][0])
        for k, nm in enumerate(names):
            _close(out["grads"][k], g[f"s{s}_grad_{nm}"], atol=1e-8)
            _close(o.params[k], g[f"s{s}_after_{nm}"])


def test_mf_python_sampler_matches_c_sampler():
    """The timed CPU-baseline sampler (random.choices over a tuple list, as
    implicit.py:352) and the C restatement draw identical pairs."""
    rs = np.random.RandomState(0)
    pu, pi = rs.randint(0, 100, 5000), rs.randint(0, 50, 5000)
    st = orng.py_seed_state(3)
    a = omf.MFOracle(*omf.init_tables(100, 50, 4), pu, pi, st.copy(), python_sampler=True)
    b = omf.MFOracle(*omf.init_tables(100, 50, 4), pu, pi, st.copy())
    _, au, ai = a.draw(777)
    _, bu, bi = b.draw(777)
    assert torch.equal(au, bu) and torch.equal(ai, bi)


def test_mf_fit_oracle_vs_reference(golden_dir):
    g = np.load(os.path.join(golden_dir, "mf_fit_golden.npz"))
    U, I, d, B, n = (int(x) for x in g["meta"])
    for loss in ("pointwise", "adaptive_hinge"):
        params = [torch.from_numpy(g[f"{loss}_init_U"].copy()), torch.from_numpy(g[f"{loss}_init_I"].copy()),
                  torch.zeros(U, 1), torch.zeros(I, 1)]
        o = omf.MFOracle(*params, g["pool_u"], g["pool_i"], g[f"{loss}_mt_state"].copy(), loss=loss,
                         optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
        nps = orng.np_seed_state(0)
        orng.np_randint(nps, -10 ** 8, 10 ** 8, 1)       # implicit.py:146 set_seed draw
        rows, best, best_epoch = omf.fit(o, g["train_u"], g["train_i"], g["valid_u"], g["valid_i"], nps, 2)
        assert best_epoch == int(g[f"{loss}_best_epoch"][0])
        csv_rows = str(g[f"{loss}_summary_csv"]).strip().splitlines()
        assert csv_rows[0] == "train_loss,validation_loss,curr_epoch"
        for r, line in zip(rows, csv_rows[1:]):
            tl, vl, ep = line.split(",")
            _close(r[0], float(tl))
            _close(r[1], float(vl))
            assert r[2] == int(ep)
        _close(best[0], g[f"{loss}_best_user_embeddings_weight"])
        _close(best[1], g[f"{loss}_best_item_embeddings_weight"])
        _close(best[2], g[f"{loss}_best_user_biases_weight"])
        _close(best[3], g[f"{loss}_best_item_biases_weight"])
        _close(omf.scores(*best, torch.full((I,), 3, dtype=torch.long), torch.arange(I)),
               g[f"{loss}_predict_u3"])
        assert (o.state == g[f"{loss}_mt_state_end"]).all()
