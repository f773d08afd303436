"""The device top-k path of the ranking metrics, vectorised over the users
(recommendation_gans_amd/spotlight/evaluation.py _topk_hits), against the per-user loop over
the full argsort ranking (the reference's definitions, spotlight/evaluation.py:115-185,
334-353) on the CPU: the same means, to the bit, with and without train-item exclusion, for
several k at once, and apk's `not actual.any()` quirk (a user whose only test item is item 0)."""
import numpy as np


class _TopkModel:
    """Scores on the host; topk_users returns the first k ids of argsort(-score) with the
    excluded (train) items last -- the ranking the reference's argsort gives."""

    def __init__(self, scores):
        self.s = scores

    def score_users(self, users):
        return self.s[np.asarray(users)].copy()

    def topk_users(self, users, k, exclude_csr=None):
        sub = -self.s[np.asarray(users)].astype(np.float32)
        if exclude_csr is not None:
            for r, u in enumerate(users):
                sub[r, exclude_csr.indices[exclude_csr.indptr[u]:exclude_csr.indptr[u + 1]]] = np.finfo(np.float32).max
        return np.argsort(sub, axis=1, kind="stable")[:, :k].astype(np.int64)


class _HostOnly:
    def __init__(self, m):
        self.score_users = m.score_users


def test_vectorised_topk_metrics_match_the_loop():
    from recommendation_gans_amd.spotlight import evaluation
    from recommendation_gans_amd.spotlight.interactions import Interactions
    rs = np.random.RandomState(0)
    U, I = 400, 700
    m = _TopkModel(rs.rand(U, I).astype(np.float32))
    h = _HostOnly(m)
    tu, ti = rs.randint(0, U, 4000), rs.randint(0, I, 4000)
    tu, ti = np.append(tu, [U - 1]), np.append(ti, [0])              # a user whose only test item is 0
    keep = ~((tu == U - 1) & (ti != 0))
    test = Interactions(tu[keep], ti[keep], num_users=U, num_items=I)
    train = Interactions(rs.randint(0, U - 50, 9000), rs.randint(0, I, 9000), num_users=U, num_items=I)
    for k in (1, 5, 10, [1, 5, 10]):
        kk = max(k) if isinstance(k, list) else k
        assert evaluation.precision_recall_score(m, test, k=k) == evaluation.precision_recall_score(h, test, k=k)
        assert evaluation.precision_recall_score(m, test, train, k=k) == \
            evaluation.precision_recall_score(h, test, train, k=k)
        assert evaluation.map_at_k(m, test, k=kk) == evaluation.map_at_k(h, test, k=kk)
