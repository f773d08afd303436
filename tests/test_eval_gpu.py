"""Evaluation top-k on the GPU (rg_topk_rows through the C-ABI) against the host
ranking the reference uses, argsort(-scores) (spotlight/evaluation.py:115-185,
334-353), on continuous random scores (no ties: numpy's argsort order of equal keys
is unspecified), padded row strides, excluded (-inf) and NaN entries; and the
metrics computed from it through the drop-in evaluation module."""
import ctypes

import numpy as np
import pytest
import torch

from recommendation_gans_amd import _lib

pytestmark = pytest.mark.gpu


def device_topk(scores, k, ld=None):
    lib = _lib.load()
    rows, cols = scores.shape
    ld = cols if ld is None else ld
    buf = torch.full((rows, ld), 7.0, dtype=torch.float32, device="cuda:0")
    buf[:, :cols] = scores.to("cuda:0")
    out = torch.empty(rows, k, dtype=torch.int32, device="cuda:0")
    _lib.check(lib.rg_topk_rows(_lib.stream_handle(), _lib.ptr(buf), rows, cols, ld, k, _lib.ptr(out)), "topk")
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("rows,cols,k,ld", [(1, 40, 1, None), (100, 1000, 5, None), (300, 20108, 10, None),
                                            (64, 777, 17, 800), (50, 5000, 32, None), (3, 32, 32, None)])
def test_topk_matches_argsort(rows, cols, k, ld):
    g = torch.Generator().manual_seed(rows * 7 + k)
    s = torch.rand(rows, cols, generator=g)
    got = device_topk(s, k, ld)
    ref = np.argsort(-s.numpy(), axis=1, kind="stable")[:, :k]
    assert (got == ref).all()


def test_topk_excluded_and_nan_rank_last():
    g = torch.Generator().manual_seed(3)
    s = torch.rand(20, 300, generator=g)
    s[:, :250] = float("-inf")          # excluded items (train interactions)
    s[0, 260] = float("nan")
    got = device_topk(s, 32)
    x = s.numpy().copy()
    x[np.isnan(x)] = -np.inf
    ref = np.argsort(-x, axis=1, kind="stable")[:, :32]
    assert (got == ref).all()


def test_topk_bad_arguments_fail_loudly():
    lib = _lib.load()
    s = torch.rand(4, 10, device="cuda:0")
    out = torch.empty(4, 40, dtype=torch.int32, device="cuda:0")
    assert lib.rg_topk_rows(_lib.stream_handle(), _lib.ptr(s), 4, 10, 10, 11, _lib.ptr(out)) != 0
    assert lib.rg_topk_rows(_lib.stream_handle(), _lib.ptr(s), 4, 10, 10, 33, _lib.ptr(out)) != 0
    assert lib.rg_topk_rows(_lib.stream_handle(), _lib.ptr(s), 4, 10, 9, 5, _lib.ptr(out)) != 0


class _DeviceModel:
    """A model exposing both paths over the same device scores."""

    def __init__(self, scores):
        self.s = scores.to("cuda:0")

    def score_users(self, users):
        return self.s[torch.as_tensor(np.asarray(users), device="cuda:0")].cpu().numpy()

    def topk_users(self, users, k, exclude_csr=None):
        sub = self.s[torch.as_tensor(np.asarray(users), device="cuda:0")].clone()
        if exclude_csr is not None:
            for r, u in enumerate(users):
                sub[r, torch.as_tensor(exclude_csr[u].indices, device="cuda:0", dtype=torch.int64)] = float("-inf")
        return device_topk(sub.cpu(), k).astype(np.int64)


class _HostOnly:
    def __init__(self, m):
        self.score_users = m.score_users


def test_metrics_from_device_topk_match_host_ranking():
    from recommendation_gans_amd.spotlight import evaluation
    from recommendation_gans_amd.spotlight.interactions import Interactions
    rs = np.random.RandomState(0)
    U, I = 300, 2000
    m = _DeviceModel(torch.rand(U, I, generator=torch.Generator().manual_seed(1)))
    test = Interactions(rs.randint(0, U, 3000), rs.randint(0, I, 3000), num_users=U, num_items=I)
    train = Interactions(rs.randint(0, U, 9000), rs.randint(0, I, 9000), num_users=U, num_items=I)
    h = _HostOnly(m)
    for k in (1, 5, 10):
        assert evaluation.precision_recall_score(m, test, k=k) == evaluation.precision_recall_score(h, test, k=k)
        assert evaluation.precision_recall_score(m, test, train, k=k) == \
            evaluation.precision_recall_score(h, test, train, k=k)
        assert evaluation.map_at_k(m, test, k=k) == evaluation.map_at_k(h, test, k=k)
