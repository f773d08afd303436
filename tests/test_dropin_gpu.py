"""The drop-in model and CLI on the GPU.

* ``ImplicitFactorizationModel.fit`` reproduces the reference's own 2-epoch fit
  (tests/golden/mf_fit_golden.npz, made by importing the reference): summary.csv
  losses, best epoch, best tables, predict(3), and the module-level ``random``
  state after fit (the negative stream, implicit.py:352 + :370) bit-exact;
* ``python -m recommendation_gans_amd.mf_spotlight`` end to end on synthetic
  MovieLens-100K-shaped data: output files and a checkpoint loadable with
  torch.load(weights_only=True) under the reference's state_dict keys."""
import csv
import io
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import mf as omf

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("inline", ["1", "2"])
@pytest.mark.parametrize("loss", ["pointwise", "adaptive_hinge"])
def test_fit_matches_reference_golden(golden_dir, tmp_path, monkeypatch, loss, inline):
    """inline "2" forces the stepper's inline MT walk (words of step t+2 walked inside step t's
    dense pass) at this small size, mixed with the generator stream that validation uses."""
    monkeypatch.setenv("RG_MT_INLINE", inline)
    from recommendation_gans_amd.implicit import ImplicitFactorizationModel
    from recommendation_gans_amd.spotlight import optimizers
    from recommendation_gans_amd.spotlight.factorization.representations import BilinearNet
    from recommendation_gans_amd.spotlight.interactions import Interactions
    z = np.load(os.path.join(golden_dir, "mf_fit_golden.npz"))
    U, I, d, B, n = (int(x) for x in z["meta"])
    train = Interactions(z["train_u"].astype(np.int32), z["train_i"].astype(np.int32),
                         ratings=np.ones(len(z["train_u"]), np.float32), num_users=U, num_items=I)
    valid = Interactions(z["valid_u"].astype(np.int32), z["valid_i"].astype(np.int32),
                         ratings=np.ones(len(z["valid_u"]), np.float32), num_users=U, num_items=I)
    pool = list(zip(z["pool_u"].tolist(), z["pool_i"].tolist()))
    net = BilinearNet(U, I, d)
    with torch.no_grad():
        net.user_embeddings.weight.copy_(torch.from_numpy(z[f"{loss}_init_U"]))
        net.item_embeddings.weight.copy_(torch.from_numpy(z[f"{loss}_init_I"]))
    random.seed(0)
    assert (np.array(random.getstate()[1], np.uint32) == z[f"{loss}_mt_state"]).all()
    monkeypatch.chdir(tmp_path)
    model = ImplicitFactorizationModel(loss=loss, embedding_dim=d, n_iter=2, batch_size=B, l2=1e-5,
                                       learning_rate=1e-2, optimizer_func=optimizers.adam_optimizer,
                                       representation=net, random_state=np.random.RandomState(0),
                                       neg_examples=pool, num_negative_samples=n, use_cuda=True)
    model.fit(train, valid)
    # the negative stream after fit: every training and validation draw, bit-exact
    assert (np.array(random.getstate()[1], np.uint32) == z[f"{loss}_mt_state_end"]).all()
    assert model.best_epoch == int(z[f"{loss}_best_epoch"][0])
    got = list(csv.reader(open(os.path.join(model.experiment_logs, "summary.csv"))))
    ref = list(csv.reader(io.StringIO(str(z[f"{loss}_summary_csv"]))))
    assert got[0] == ref[0] and len(got) == len(ref)
    for g, r in zip(got[1:], ref[1:]):
        np.testing.assert_allclose([float(x) for x in g], [float(x) for x in r], rtol=1e-5)
    # best tables: 1e-5 relative (tensor norm) against the reference's own, or -- where Adam
    # amplifies a cancelled gradient's rounding -- as close to the float64 restatement of the
    # same fit (oracle.mf.fit) as the reference's fp32 tables are
    from oracle import rng as orng
    o64 = omf.MFOracle(torch.from_numpy(z[f"{loss}_init_U"].copy()).double(),
                       torch.from_numpy(z[f"{loss}_init_I"].copy()).double(), torch.zeros(U, 1, dtype=torch.float64),
                       torch.zeros(I, 1, dtype=torch.float64), z["pool_u"], z["pool_i"], z[f"{loss}_mt_state"].copy(),
                       loss=loss, optimizer="adam", lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    nps = orng.np_seed_state(0)
    orng.np_randint(nps, -10 ** 8, 10 ** 8, 1)
    _, best64, _ = omf.fit(o64, z["train_u"], z["train_i"], z["valid_u"], z["valid_i"], nps, 2)
    names = ["user_embeddings_weight", "item_embeddings_weight", "user_biases_weight", "item_biases_weight"]
    for t, nm, r64 in zip(model.best_model, names, best64):
        ref_t = torch.from_numpy(z[f"{loss}_best_{nm}"])
        ok, msg = omf.tensor_parity(t.reshape(ref_t.shape), ref_t, r64.reshape(ref_t.shape), rtol=1e-5)
        assert ok, (nm, msg)
    np.testing.assert_allclose(model.predict(3), z[f"{loss}_predict_u3"], rtol=1e-5, atol=1e-7)
    ck = torch.load(os.path.join(model.experiment_saved_models, "best_model"), weights_only=True)
    assert set(ck["network"]) == {"user_embeddings.weight", "item_embeddings.weight", "user_biases.weight",
                                  "item_biases.weight"}
    assert json.load(open(os.path.join(model.experiment_logs, "configuration.json")))["num_users"] == U


def test_fit_without_negatives_matches_reference(golden_dir, tmp_path, monkeypatch):
    """implicit.py:351-360's neg_examples=None branch (tests/golden/mf_fit_noneg_golden.npz, the
    reference's own 2-epoch fit): the pointwise loss on the positives only (RG_LOSS_POINTWISE_POS),
    summary.csv, best epoch, best tables, predict(3), and the `random` state untouched."""
    from recommendation_gans_amd.implicit import ImplicitFactorizationModel
    from recommendation_gans_amd.spotlight import optimizers
    from recommendation_gans_amd.spotlight.factorization.representations import BilinearNet
    from recommendation_gans_amd.spotlight.interactions import Interactions
    f = np.load(os.path.join(golden_dir, "mf_fit_golden.npz"))
    z = np.load(os.path.join(golden_dir, "mf_fit_noneg_golden.npz"))
    U, I, d, B, n = (int(x) for x in z["meta"])
    train = Interactions(f["train_u"].astype(np.int32), f["train_i"].astype(np.int32),
                         ratings=np.ones(len(f["train_u"]), np.float32), num_users=U, num_items=I)
    valid = Interactions(f["valid_u"].astype(np.int32), f["valid_i"].astype(np.int32),
                         ratings=np.ones(len(f["valid_u"]), np.float32), num_users=U, num_items=I)
    net = BilinearNet(U, I, d)
    with torch.no_grad():
        net.user_embeddings.weight.copy_(torch.from_numpy(z["init_U"]))
        net.item_embeddings.weight.copy_(torch.from_numpy(z["init_I"]))
    random.seed(0)
    monkeypatch.chdir(tmp_path)
    model = ImplicitFactorizationModel(loss="pointwise", embedding_dim=d, n_iter=2, batch_size=B, l2=1e-5,
                                       learning_rate=1e-2, optimizer_func=optimizers.adam_optimizer,
                                       representation=net, random_state=np.random.RandomState(0),
                                       neg_examples=None, num_negative_samples=n, use_cuda=True)
    model.fit(train, valid)
    assert (np.array(random.getstate()[1], np.uint32) == z["mt_state_end"]).all()
    assert (z["mt_state_end"] == z["mt_state"]).all()
    assert model.best_epoch == int(z["best_epoch"][0])
    got = list(csv.reader(open(os.path.join(model.experiment_logs, "summary.csv"))))
    ref = list(csv.reader(io.StringIO(str(z["summary_csv"]))))
    assert got[0] == ref[0] and len(got) == len(ref)
    for g, r in zip(got[1:], ref[1:]):
        np.testing.assert_allclose([float(x) for x in g], [float(x) for x in r], rtol=1e-5)
    names = ["user_embeddings_weight", "item_embeddings_weight", "user_biases_weight", "item_biases_weight"]
    for t, nm in zip(model.best_model, names):
        ref_t = torch.from_numpy(z[f"best_{nm}"])
        ok, msg = omf.tensor_parity(t.reshape(ref_t.shape), ref_t, rtol=1e-5)
        assert ok, (nm, msg)
    np.testing.assert_allclose(model.predict(3), z["predict_u3"], rtol=1e-5, atol=1e-7)
    # the pairwise losses need the negatives argument, as in the reference
    with pytest.raises(TypeError):
        ImplicitFactorizationModel(loss="hinge", embedding_dim=d, n_iter=1, batch_size=B, representation=BilinearNet(
            U, I, d), neg_examples=None, use_cuda=True).fit(train, valid)


def test_mf_spotlight_cli_synthetic(tmp_path, monkeypatch):
    from recommendation_gans_amd import mf_spotlight
    monkeypatch.chdir(tmp_path)
    np.random.seed(0)
    random.seed(0)
    model = mf_spotlight.main(["--use_gpu", "True", "--dataset", "100K", "--training_epochs", "2",
                               "--batch_size", "1024", "--mf_embedding_dim", "32", "--experiment_name", "cli",
                               "--k", "3", "--mf_loss", "pairwise_bpr"])
    logs = os.path.join("experiments_results", "cli", "result_outputs")
    rows = list(csv.reader(open(os.path.join(logs, "summary.csv"))))
    assert rows[0] == ["train_loss", "validation_loss", "curr_epoch"] and len(rows) == 3
    assert all(np.isfinite(float(x)) for x in rows[1][:2])
    res = json.load(open(os.path.join(logs, "test_summary.json")))
    assert {"k", "bce", "precision", "recall", "map"} <= set(res)
    ck = torch.load(os.path.join("experiments_results", "cli", "saved_models", "best_model"), weights_only=True)
    assert ck["network"]["user_embeddings.weight"].shape == (943, 32)
    assert 0 <= model.best_epoch <= 1


def test_ncf_fit_and_cli(tmp_path, monkeypatch):
    from recommendation_gans_amd import ncf_spotlight
    monkeypatch.chdir(tmp_path)
    np.random.seed(0)
    random.seed(0)
    model = ncf_spotlight.main(["--use_gpu", "True", "--dataset", "100K", "--training_epochs", "2",
                                "--batch_size", "1024", "--mlp_embedding_dim", "16", "--experiment_name", "ncf",
                                "--k", "3"])
    logs = os.path.join("experiments_results", "ncf", "result_outputs")
    rows = list(csv.reader(open(os.path.join(logs, "summary.csv"))))
    assert len(rows) == 3 and all(np.isfinite(float(x)) for x in rows[1][:2] + rows[2][:2])
    assert float(rows[2][0]) < float(rows[1][0])            # training loss falls over the epochs
    ck = torch.load(os.path.join("experiments_results", "ncf", "saved_models", "best_model"), weights_only=True)
    assert ck["network"]["embedding_user.weight"].shape == (943, 16)
    assert "layers.0.weight" in ck["network"]
    res = json.load(open(os.path.join(logs, "test_summary.json")))
    assert {"precision", "recall", "map"} <= set(res)
    p = model.predict(3)
    assert p.shape == (1682,) and np.all((p > 0) & (p < 1))


def test_neumf_fit_and_cli(tmp_path, monkeypatch):
    from recommendation_gans_amd import neuMF_spotlight
    monkeypatch.chdir(tmp_path)
    np.random.seed(0)
    random.seed(0)
    model = neuMF_spotlight.main(["--use_gpu", "True", "--dataset", "100K", "--training_epochs", "2",
                                  "--batch_size", "1024", "--mlp_embedding_dim", "16", "--mf_embedding_dim", "50",
                                  "--experiment_name", "neumf", "--k", "3"])
    logs = os.path.join("experiments_results", "neumf", "result_outputs")
    rows = list(csv.reader(open(os.path.join(logs, "summary.csv"))))
    assert len(rows) == 3 and all(np.isfinite(float(x)) for x in rows[1][:2] + rows[2][:2])
    assert float(rows[2][0]) < float(rows[1][0])
    ck = torch.load(os.path.join("experiments_results", "neumf", "saved_models", "best_model"), weights_only=True)
    assert ck["network"]["embedding_user_mf.weight"].shape == (943, 50)
    assert ck["network"]["affine_output.weight"].shape == (1, 58)
    res = json.load(open(os.path.join(logs, "test_summary.json")))
    assert {"precision", "recall", "map"} <= set(res)
    p = model.predict(3)
    assert p.shape == (1682,) and np.all((p > 0) & (p < 1))
    # the module's own forward (eval mode) scores as the engine does
    net = model._net.eval()
    u = torch.full((1682,), 3, dtype=torch.int64, device="cuda")
    with torch.no_grad():
        s = net(u, torch.arange(1682, device="cuda")).reshape(-1).cpu().numpy()
    np.testing.assert_allclose(s, p, rtol=1e-5, atol=1e-6)


def test_slate_generation_cli(tmp_path, monkeypatch):
    """python -m recommendation_gans_amd.slate_generation end to end on synthetic
    MovieLens-100K-shaped slates: summary.csv (the reference's columns; training
    precision 0 as in the reference), validation / test precision, and a generator
    checkpoint loadable with weights_only=True under the reference's names."""
    from recommendation_gans_amd import slate_generation
    monkeypatch.chdir(tmp_path)
    model, res = slate_generation.main(["--use_gpu", "True", "--dataset", "100K", "--training_epochs", "2",
                                        "--batch_size", "128", "--gan_hidden_layer", "16", "--slate_size", "3",
                                        "--experiment_name", "gan"])
    logs = os.path.join("experiments_results", "gan", "result_outputs")
    rows = list(csv.reader(open(os.path.join(logs, "summary.csv"))))
    assert rows[0] == ["G_loss", "D_loss", "G_pre", "G_rec", "curr_epoch", "Val_prec"] and len(rows) == 3
    for r in rows[1:]:
        g, d, pre, rec, ep, vp = (float(x) for x in r)
        assert np.isfinite(g) and np.isfinite(d) and pre == 0.0 and rec == 0.0 and 0.0 <= vp <= 1.0
    assert 0.0 <= res["precision"] <= 1.0 and res["at"] == 3
    assert json.load(open(os.path.join(logs, "test_results.json")))["at"] == 3
    ck = torch.load(os.path.join("experiments_results", "gan", "saved_models", "generator"), weights_only=True)
    assert ck["network"]["mult_heads.head_0.weight"].shape == (1682, 16)
    assert ck["network"]["layers.1.running_mean"].shape == (8,)
    assert model.chosen_epoch in (0, 1)
