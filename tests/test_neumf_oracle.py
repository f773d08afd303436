"""oracle/ncf.py's NeuMF restatement against the reference's own NeuMF steps
(tests/golden/neumf_*.npz): scores, loss, gradients and parameters after each Adam
step, with the recorded dropout masks of the tower."""
import os

import numpy as np
import pytest
import torch

from oracle import ncf as oncf

CASES = ["neumf_pointwise_e16_m10", "neumf_bpr_e8_m5", "neumf_adaptive_hinge_e16_m12"]


def load_case(golden_dir, name):
    z = np.load(os.path.join(golden_dir, name + ".npz"))
    names = [str(x) for x in z["param_names"]]
    tensors = [torch.from_numpy(z["init_" + nm.replace(".", "_")].copy()) for nm in names]
    return z, names, tensors


def step_masks(z, s, kind, n_layers):
    return [torch.from_numpy(z[f"s{s}_mask_{kind}{k}"]) for k in range(n_layers)]


def loss_of(case):
    return case[len("neumf_"):].rsplit("_e", 1)[0]


@pytest.mark.parametrize("case", CASES)
def test_neumf_oracle_matches_reference(golden_dir, case):
    z, names, tensors = load_case(golden_dir, case)
    U, I, E, B, n, M = (int(x) for x in z["meta"])
    assert list(z["layers"]) == oncf.layer_sizes(E)
    assert names[:4] == ["embedding_user_mlp.weight", "embedding_item_mlp.weight", "embedding_user_mf.weight",
                         "embedding_item_mf.weight"] and names[-2] == "affine_output.weight"
    o = oncf.NeuMFOracle(tensors, names, z["pool_u"], z["pool_i"], z["s0_mt_state"].copy(), loss=loss_of(case),
                         lr=1e-2, weight_decay=1e-5, n_neg=n, batch_size=B)
    nl = len(z["layers"]) - 1
    for s in range(3):
        assert (o.state == z[f"s{s}_mt_state"]).all()
        prev = [t.numpy().copy() for t in o.P.t]
        out = o.step(z[f"s{s}_pos_u"], z[f"s{s}_pos_i"], step_masks(z, s, "pos", nl), step_masks(z, s, "neg", nl),
                     return_all=True)
        np.testing.assert_allclose(out["p_pos"].numpy(), z[f"s{s}_p_pos"], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(out["p_neg"].numpy(), z[f"s{s}_p_neg"], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(out["loss"], z[f"s{s}_loss"][0], rtol=1e-6)
        for nm, g in zip(names, out["grads"]):
            ref = z[f"s{s}_grad_" + nm.replace(".", "_")]
            np.testing.assert_allclose(g.numpy(), ref, rtol=1e-5, atol=1e-6 * float(np.abs(ref).max() + 1e-30),
                                       err_msg=f"{case} step {s} grad {nm}")
        for nm, p, before in zip(names, o.P.t, prev):
            ref = z[f"s{s}_after_" + nm.replace(".", "_")]
            scale = max(float(np.linalg.norm(ref)), float(np.linalg.norm(before)))
            err = float(np.linalg.norm(p.numpy() - ref)) / max(scale, 1e-30)
            assert err <= 1e-5, f"{case} step {s} {nm}: rel {err:.2e}"
    assert (o.state == z["end_mt_state"]).all()
