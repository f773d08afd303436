"""Ranking metrics of spotlight/evaluation.py (reference :13-353).

Same definitions as the reference: per test user with at least one test item,
rank all items by -score (``argsort``), precision/recall@k over the top k,
average precision@k, hit ratio; popularity and random baselines.  The scores of a
block of users against every item come from one GEMM on the device
(``model.score_users``) instead of one ``predict`` call per user; the metrics that read
only the first k ranks (precision/recall@k, hit ratio, MAP@k) take them from the
device top-k (``model.topk_users`` -> rg_topk_rows) when the model has one and
k <= 32, so only users x k ids reach the host."""
import numpy as np
import scipy.stats as st

FLOAT_MAX = np.finfo(np.float32).max


def _get_precision_recall(predictions, targets, k):
    predictions = predictions[:k]
    num_hit = len(set(predictions).intersection(set(targets)))
    return float(num_hit) / k, float(num_hit) / len(targets)


def _row(csr, u):
    """csr[u].indices without building a row matrix (per-user slicing dominated the loop)."""
    return csr.indices[csr.indptr[u]:csr.indptr[u + 1]]


def _scored(model, test_csr, train_csr=None, block=4096):
    """Yields (user, row indices, -scores with train items at FLOAT_MAX) for every test
    user with items, in user order."""
    users = np.flatnonzero(np.diff(test_csr.indptr) > 0)
    for s in range(0, len(users), block):
        ub = users[s:s + block]
        scores = -model.score_users(ub)                      # (len(ub), I) float32, host
        for r, u in enumerate(ub):
            pred = scores[r]
            if train_csr is not None:
                pred[_row(train_csr, u)] = FLOAT_MAX
            yield u, _row(test_csr, u), pred


TOPK_MAX = 32


def _ranked(model, test_csr, train_csr=None, block=4096, k=None):
    """Yields (user, row indices, item ranking) for every test user with items; with k,
    the ranking may hold only its first k entries (the device top-k)."""
    if k is not None and k <= TOPK_MAX and hasattr(model, "topk_users"):
        users = np.flatnonzero(np.diff(test_csr.indptr) > 0)
        for s in range(0, len(users), block):
            ub = users[s:s + block]
            top = model.topk_users(ub, int(k), train_csr)      # (len(ub), k) int64, host
            for r, u in enumerate(ub):
                yield u, _row(test_csr, u), top[r]
        return
    for u, idx, pred in _scored(model, test_csr, train_csr, block):
        yield u, idx, pred.argsort(axis=0)


def _topk_hits(model, test_csr, train_csr, k, block=4096):
    """The device top-k path of the metrics (model.topk_users, k <= TOPK_MAX), vectorised over
    the users instead of a Python loop per user (the loop took 0.7 s per 125 k users): the users
    with test items, their top-k rankings, hits[u, j] = ranking j of user u is one of its test
    items (the rankings are distinct ids, so the count of hits in the first x ranks is the
    reference's |set(ranking[:x]) & set(targets)|), and each user's number of test items."""
    users = np.flatnonzero(np.diff(test_csr.indptr) > 0)
    if not len(users):
        return users, np.zeros((0, k), bool), np.zeros(0, np.int64)
    I = np.int64(test_csr.shape[1])
    rows = np.repeat(np.arange(test_csr.shape[0], dtype=np.int64), np.diff(test_csr.indptr))
    keys = np.sort(rows * I + test_csr.indices.astype(np.int64))
    hits = np.empty((len(users), k), bool)
    for s in range(0, len(users), block):
        ub = users[s:s + block]
        top = np.asarray(model.topk_users(ub, int(k), train_csr), dtype=np.int64)[:, :k]
        q = ub[:, None].astype(np.int64) * I + top
        pos = np.minimum(np.searchsorted(keys, q), len(keys) - 1)
        hits[s:s + len(ub)] = keys[pos] == q
    return users, hits, np.diff(test_csr.indptr)[users].astype(np.int64)


def _device_topk(model, k):
    return k <= TOPK_MAX and hasattr(model, "topk_users")


def mrr_score(model, test, train=None):
    """Mean reciprocal rank of each test user's items (evaluation.py:13-60): ranks of
    -score with ties averaged (scipy rankdata), train items pushed to the end."""
    test_csr = test.tocsr()
    train_csr = train.tocsr() if train is not None else None
    return np.array([(1.0 / st.rankdata(pred)[idx]).mean() for _, idx, pred in _scored(model, test_csr, train_csr)])


def sequence_mrr_score(model, test, exclude_preceding=False):
    """Reciprocal rank of each sequence's last item given the rest (evaluation.py:62-106)."""
    sequences, targets = test.sequences[:, :-1], test.sequences[:, -1:]
    mrrs = []
    for i in range(len(sequences)):
        pred = -model.predict(sequences[i])
        if exclude_preceding:
            pred[sequences[i]] = FLOAT_MAX
        mrrs.append((1.0 / st.rankdata(pred)[targets[i]]).mean())
    return np.array(mrrs)


def precision_recall_score(model, test, train=None, k=10):
    test_csr = test.tocsr()
    train_csr = train.tocsr() if train is not None else None
    ks = np.array([k]) if np.isscalar(k) else np.asarray(k)
    if _device_topk(model, int(ks.max())):
        users, hits, n_t = _topk_hits(model, test_csr, train_csr, int(ks.max()))
        if train_csr is not None:
            print("Cold start users: ", int((np.diff(train_csr.indptr)[users] == 0).sum()))
        else:
            print("Cold start users: ", 0)
        c = np.cumsum(hits, axis=1)
        num = np.stack([c[:, int(x) - 1] for x in ks], axis=1).astype(np.float64)
        return (np.mean((num / ks.astype(np.float64)[None, :]).squeeze()),
                np.mean((num / n_t[:, None].astype(np.float64)).squeeze()))
    precision, recall = [], []
    cold = 0
    for u, targets, ranking in _ranked(model, test_csr, train_csr, k=int(ks.max())):
        if train_csr is not None and not len(_row(train_csr, u)):
            cold += 1
        p, r = zip(*[_get_precision_recall(ranking, targets, x) for x in ks])
        precision.append(p)
        recall.append(r)
    print("Cold start users: ", cold)
    return np.mean(np.array(precision).squeeze()), np.mean(np.array(recall).squeeze())


def rmse_score(net, user_ids, item_ids):
    predictions = net(user_ids, item_ids)
    array = 1 - predictions.cpu().detach().numpy()
    return np.sum(array ** 2)


def hit_ratio(model, test, k=10):
    hits = users = 0
    for _, target, ranking in _ranked(model, test.tocsr(), k=k):
        users += 1
        if target in ranking[:k]:
            hits += 1
    return hits / users


def apk(actual, predicted, k=10):
    if len(predicted) > k:
        predicted = predicted[:k]
    score, num_hits = 0.0, 0.0
    for i, p in enumerate(predicted):
        if p in actual and p not in predicted[:i]:
            num_hits += 1.0
            score += num_hits / (i + 1.0)
    if not actual.any():
        return 0.0
    return score / min(len(actual), k)


def mapk(actual, predicted, k=10):
    return np.mean([apk(a, p, k) for a, p in zip(actual, predicted)])


def map_at_k(model, test, k=5):
    if _device_topk(model, k):
        # apk over every user at once, its sums in apk's order (one position at a time)
        test_csr = test.tocsr()
        users, hits, n_t = _topk_hits(model, test_csr, None, k)
        cum = np.cumsum(hits, axis=1).astype(np.float64)
        score = np.zeros(len(users))
        for i in range(k):
            score = np.where(hits[:, i], score + cum[:, i] / (i + 1.0), score)
        first = test_csr.indices[test_csr.indptr[users]]
        only_zero = (n_t == 1) & (first == 0)          # apk: `not actual.any()` -> 0
        vals = np.where(only_zero, 0.0, score / np.minimum(n_t, k).astype(np.float64))
        return np.mean(vals.squeeze())
    vals = [apk(targets, ranking, k=k) for _, targets, ranking in _ranked(model, test.tocsr(), k=k)]
    return np.mean(np.array(vals).squeeze())


def evaluate_popItems(item_popularity, test, k=10):
    test = test.tocsr()
    pop = np.asarray(getattr(item_popularity, "values", item_popularity))
    pop_top = pop.argsort()[::-1][:k]
    ks = np.array([k]) if np.isscalar(k) else np.asarray(k)
    precision, recall = [], []
    for row in test:
        if not len(row.indices):
            continue
        p, r = zip(*[_get_precision_recall(pop_top, row.indices, x) for x in ks])
        precision.append(p)
        recall.append(r)
    return np.mean(precision), np.mean(recall),


def evaluate_random(item_popularity, test, k=10):
    all_items = test.num_items
    test = test.tocsr()
    ks = np.array([k]) if np.isscalar(k) else np.asarray(k)
    precision, recall = [], []
    for row in test:
        if not len(row.indices):
            continue
        predictions = np.random.choice(all_items, len(row.indices))
        p, r = zip(*[_get_precision_recall(predictions, row.indices, x) for x in ks])
        precision.append(p)
        recall.append(r)
    return np.mean(np.array(precision).squeeze()), np.mean(np.array(recall).squeeze())


def precision_recall_score_slates(slates, test, k=3):
    """spotlight/evaluation.py:355-382: precision / recall@k of each test user's
    generated slate (row u of ``slates`` belongs to row u of the CSR ``test``)."""
    ks = np.array([k]) if np.isscalar(k) else np.asarray(k)
    test = test.tocsr()
    precision, recall = [], []
    for user_id in range(test.shape[0]):
        targets = test.indices[test.indptr[user_id]:test.indptr[user_id + 1]]
        if not len(targets):
            continue
        pred = slates[user_id].numpy() if hasattr(slates[user_id], "numpy") else np.asarray(slates[user_id])
        p, r = zip(*[_get_precision_recall(pred, targets, x) for x in ks])
        precision.append(p[0])
        recall.append(r[0])
    return precision, recall


def precision_recall_slates_atk(fake_slates, real_slates, k=3):
    """spotlight/evaluation.py:394-412, the generator's training precision / recall.
    The reference intersects sets of 0-d torch tensors (rows of the two slate
    tensors), which hash by identity, so every user scores 0; the same operations on
    the same tensor types are kept here so summary.csv matches the reference."""
    ks = np.array([k]) if np.isscalar(k) else np.asarray(k)
    precision, recall = [], []
    for user_id in range(fake_slates.shape[0]):
        p, r = zip(*[_get_precision_recall(fake_slates[user_id, :], real_slates[user_id, :], x) for x in ks])
        precision.append(p[0])
        recall.append(r[0])
    return precision, recall
