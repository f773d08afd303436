"""oracle/ncf.py -- TEST INFRASTRUCTURE ONLY.

CPU restatement (torch-CPU fp32, explicit formulas, no autograd) of the
reference's NCF training step:

  * MLP.__init__ / forward             spotlight/dnn_models/mlp.py:5-46
      layers [2E, E, ..., 8] -> 1      ncf_spotlight.py:53-56
      Linear -> LeakyReLU(0.1) -> Dropout(0.5) per hidden layer, Linear -> Sigmoid
  * losses on (N, 1) scores            spotlight/losses.py:20-172 (as oracle/mf.py)
  * autograd of the above              implicit.py:361 (linear / leaky_relu /
      dropout / sigmoid backward as ATen computes them, dense embedding grads)
  * Adam over every parameter          spotlight/optimizers.py:10-16, implicit.py:363
  * NeuMF.__init__ / forward           spotlight/dnn_models/neuMF.py:7-55
      the same tower (no output Linear inside), GMF branch U_mf[u] * I_mf[i],
      affine_output over cat([tower, gmf]) -> Sigmoid

Dropout masks are inputs (the reference draws them from torch's CPU generator;
tests/golden records them with forward hooks), scaled by 1 / (1 - 0.5) = 2.
Pinned by tests/golden/mlp_*.npz and neumf_*.npz (made by importing the reference).
"""
import torch

from . import mf as omf
from . import rng as orng

LRELU = 0.1
DROP_SCALE = 2.0


def layer_sizes(E):
    """ncf_spotlight.py:53-55: [2**x for x in reversed(range(3, log2(2E) + 1))]."""
    import math
    top = int(math.log2(E * 2))
    return [2 ** x for x in reversed(range(3, top + 1))]


class MLPParams:
    """Parameters in the reference's named_parameters() order."""

    NAMES_FMT = ("embedding_user.weight", "embedding_item.weight")

    def __init__(self, tensors, names):
        self.t = list(tensors)
        self.names = list(names)

    def emb(self):
        return self.t[0], self.t[1]

    def linears(self):
        return [(self.t[k], self.t[k + 1]) for k in range(2, len(self.t), 2)]


def forward(P, u, i, masks, xperm=None):
    """Returns p (N,1) and the cache for backward.  ``masks``: per hidden layer (N, out) 0/1.
    ``xperm``: the input features in that order (P's first layer permuted to match)."""
    Ue, Ie = P.emb()
    x = torch.cat([Ue[u], Ie[i]], dim=-1)
    if xperm is not None:
        x = x[:, xperm]
    lin = P.linears()
    cache = {"x": x, "z": [], "a": [x]}
    a = x
    for k, (W, b) in enumerate(lin[:-1]):
        z = a.mm(W.t()) + b
        r = torch.where(z > 0, z, z * LRELU)
        a = r * (masks[k].to(z.dtype) * DROP_SCALE)
        cache["z"].append(z)
        cache["a"].append(a)
    W, b = lin[-1]
    logit = a.mm(W.t()) + b
    p = torch.sigmoid(logit)
    cache["p"] = p
    return p, cache


def backward(P, u, i, masks, cache, dp, xperm=None):
    """dp: dL/dp (N,1).  Returns dense grads in parameter order."""
    p = cache["p"]
    dz = dp * (1 - p) * p
    lin = P.linears()
    grads_lin = []
    for k in range(len(lin) - 1, -1, -1):
        W, b = lin[k]
        a_prev = cache["a"][k]
        dW = dz.t().mm(a_prev)
        db = dz.sum(0)
        grads_lin.append((dW, db))
        da = dz.mm(W)
        if k > 0:
            z = cache["z"][k - 1]
            da = da * (masks[k - 1].to(z.dtype) * DROP_SCALE)
            dz = torch.where(z > 0, da, da * LRELU)
        else:
            dx = da
    grads_lin.reverse()
    Ue, Ie = P.emb()
    E = Ue.shape[1]
    if xperm is not None:
        dx = dx[:, torch.argsort(xperm)]
    dU = torch.zeros_like(Ue).index_add_(0, u, dx[:, :E])
    dI = torch.zeros_like(Ie).index_add_(0, i, dx[:, E:])
    out = [dU, dI]
    for dW, db in grads_lin:
        out += [dW, db]
    return out


class NCFOracle:
    """One run_train_iteration (implicit.py:347-364) of the NCF MLP per ``step``."""

    def __init__(self, tensors, names, pool_u, pool_i, mt_state, loss="pointwise", lr=1e-2, weight_decay=1e-5,
                 n_neg=5, batch_size=256, betas=(0.5, 0.999), order_seed=None):
        self.P = MLPParams(tensors, names)
        # order_seed (pointwise, test infrastructure): run the step over the examples, the input
        # features and every hidden layer's units in seeded orders -- the same arithmetic summed
        # in other fp32 orders (batch sums and every product's inner sum), a further sample of
        # the rounding noise for tests/parity_report.py's elementwise band
        assert order_seed is None or loss == "pointwise"
        self.order = None if order_seed is None else torch.Generator().manual_seed(order_seed)
        self.loss_kind = loss
        self.n, self.batch_size = n_neg, batch_size
        self.opt_lr, self.opt_wd, self.opt_betas = lr, weight_decay, betas
        self.opt = omf.Optim("adam", self.P.t, lr, weight_decay, betas=betas)
        self.pool_u = torch.as_tensor(pool_u).long()
        self.pool_i = torch.as_tensor(pool_i).long()
        self.state = mt_state

    def draw(self, k):
        idx = orng.py_choices_indices(self.state, len(self.pool_u), k)
        t = torch.from_numpy(idx)
        return idx, self.pool_u[t], self.pool_i[t]

    def _permuted(self, u, i, masks):
        if self.order is None:
            return u, i, masks
        pr = torch.randperm(len(u), generator=self.order)
        return u[pr], i[pr], [m[pr] for m in masks]

    def _unit_orders(self):
        """order_seed: the input features and every hidden layer's units in a seeded order (the
        same function; every product sums over its inner dimension in another order).  Returns
        (P', masks -> masks', grads' -> grads, xperm); identity without order_seed."""
        if self.order is None:
            return self.P, (lambda m: m), (lambda g: g), None
        lin = self.P.linears()
        E2 = lin[0][0].shape[1]
        xperm = torch.randperm(E2, generator=self.order)
        hperm = [torch.randperm(W.shape[0], generator=self.order) for W, _ in lin[:-1]]
        ins = [xperm] + hperm                                 # input order of linear k
        t = list(self.P.t[:2])
        for k, (W, b) in enumerate(lin):
            rows = hperm[k] if k < len(hperm) else torch.arange(W.shape[0])
            t += [W[rows][:, ins[k]], b[rows]]
        Pp = MLPParams(t, self.P.names)

        def masks_p(ms):
            return [m[:, hperm[k]] for k, m in enumerate(ms)]

        def grads_back(g):
            out = list(g[:2])
            for k in range(len(lin)):
                dW, db = g[2 + 2 * k], g[3 + 2 * k]
                rows = torch.argsort(hperm[k]) if k < len(hperm) else torch.arange(dW.shape[0])
                out += [dW[rows][:, torch.argsort(ins[k])], db[rows]]
            return out
        return Pp, masks_p, grads_back, xperm

    def step(self, pos_u, pos_i, masks_pos, masks_neg, return_all=False):
        u = torch.as_tensor(pos_u).long()
        i = torch.as_tensor(pos_i).long()
        u, i, masks_pos = self._permuted(u, i, masks_pos)
        P, mperm, gback, xperm = self._unit_orders()
        masks_pos = mperm(masks_pos)
        p_pos, c_pos = forward(P, u, i, masks_pos, xperm)
        idx, nu, ni = self.draw(self.n * self.batch_size)
        nu, ni, masks_neg = self._permuted(nu, ni, masks_neg)
        masks_neg = mperm(masks_neg)
        p_neg, c_neg = forward(P, nu, ni, masks_neg, xperm)
        kind = self.loss_kind
        loss, dpp, dpn = omf.loss_and_dp(kind, p_pos.reshape(-1), p_neg.reshape(-1), self.n, self.batch_size)
        g1 = backward(P, u, i, masks_pos, c_pos, dpp.reshape(-1, 1), xperm)
        g2 = backward(P, nu, ni, masks_neg, c_neg, dpn.reshape(-1, 1), xperm)
        grads = gback([a + b for a, b in zip(g1, g2)])
        self.opt.step(self.P.t, grads)
        if return_all:
            return dict(loss=float(loss), p_pos=p_pos, p_neg=p_neg, neg_idx=idx, neg_u=nu, neg_i=ni, grads=grads)
        return float(loss)


class NeuMFParams(MLPParams):
    """neuMF.py named_parameters() order: embedding_user_mlp, embedding_item_mlp,
    embedding_user_mf, embedding_item_mf, layers.{3k}.weight/bias, affine_output."""

    def emb(self):
        return self.t[0], self.t[1]

    def emb_mf(self):
        return self.t[2], self.t[3]

    def linears(self):
        return [(self.t[k], self.t[k + 1]) for k in range(4, len(self.t), 2)]


def neumf_forward(P, u, i, masks):
    """neuMF.py:34-55: tower over cat(U_mlp[u], I_mlp[i]), GMF = U_mf[u] * I_mf[i],
    sigmoid(affine_output(cat(tower, GMF)))."""
    Ue, Ie = P.emb()
    Um, Im = P.emb_mf()
    x = torch.cat([Ue[u], Ie[i]], dim=-1)
    lin = P.linears()
    cache = {"z": [], "a": [x]}
    a = x
    for k, (W, b) in enumerate(lin[:-1]):
        z = a.mm(W.t()) + b
        r = torch.where(z > 0, z, z * LRELU)
        a = r * (masks[k].to(z.dtype) * DROP_SCALE)
        cache["z"].append(z)
        cache["a"].append(a)
    gmf = Um[u] * Im[i]
    v = torch.cat([a, gmf], dim=-1)
    W, b = lin[-1]
    p = torch.sigmoid(v.mm(W.t()) + b)
    cache.update(p=p, v=v, gmf_u=Um[u], gmf_i=Im[i])
    return p, cache


def neumf_backward(P, u, i, masks, cache, dp):
    """Dense grads in parameter order (the reference's autograd, restated)."""
    p = cache["p"]
    dz = dp * (1 - p) * p
    lin = P.linears()
    W, b = lin[-1]
    T = lin[-2][0].shape[0] if len(lin) > 1 else 8          # tower width (8)
    dWo, dbo = dz.t().mm(cache["v"]), dz.sum(0)
    dv = dz.mm(W)
    dgmf = dv[:, T:]
    dUm_rows, dIm_rows = dgmf * cache["gmf_i"], dgmf * cache["gmf_u"]
    da = dv[:, :T]
    grads_lin = [(dWo, dbo)]
    for k in range(len(lin) - 2, -1, -1):
        Wk, bk = lin[k]
        z = cache["z"][k]
        da = da * (masks[k].to(z.dtype) * DROP_SCALE)
        dzk = torch.where(z > 0, da, da * LRELU)
        grads_lin.append((dzk.t().mm(cache["a"][k]), dzk.sum(0)))
        da = dzk.mm(Wk)
    grads_lin.reverse()
    Ue, Ie = P.emb()
    Um, Im = P.emb_mf()
    E = Ue.shape[1]
    out = [torch.zeros_like(Ue).index_add_(0, u, da[:, :E]), torch.zeros_like(Ie).index_add_(0, i, da[:, E:]),
           torch.zeros_like(Um).index_add_(0, u, dUm_rows), torch.zeros_like(Im).index_add_(0, i, dIm_rows)]
    for dW, db in grads_lin:
        out += [dW, db]
    return out


class NeuMFOracle(NCFOracle):
    """One run_train_iteration (implicit.py:347-364) of NeuMF per ``step``."""

    def __init__(self, tensors, names, *a, **k):
        super().__init__(tensors, names, *a, **k)
        self.P = NeuMFParams(tensors, names)
        self.opt = omf.Optim("adam", self.P.t, self.opt_lr, self.opt_wd, betas=self.opt_betas)

    def step(self, pos_u, pos_i, masks_pos, masks_neg, return_all=False):
        u = torch.as_tensor(pos_u).long()
        i = torch.as_tensor(pos_i).long()
        u, i, masks_pos = self._permuted(u, i, masks_pos)
        p_pos, c_pos = neumf_forward(self.P, u, i, masks_pos)
        idx, nu, ni = self.draw(self.n * self.batch_size)
        nu, ni, masks_neg = self._permuted(nu, ni, masks_neg)
        p_neg, c_neg = neumf_forward(self.P, nu, ni, masks_neg)
        loss, dpp, dpn = omf.loss_and_dp(self.loss_kind, p_pos.reshape(-1), p_neg.reshape(-1), self.n,
                                         self.batch_size)
        g1 = neumf_backward(self.P, u, i, masks_pos, c_pos, dpp.reshape(-1, 1))
        g2 = neumf_backward(self.P, nu, ni, masks_neg, c_neg, dpn.reshape(-1, 1))
        grads = [a + b for a, b in zip(g1, g2)]
        self.opt.step(self.P.t, grads)
        if return_all:
            return dict(loss=float(loss), p_pos=p_pos, p_neg=p_neg, neg_idx=idx, neg_u=nu, neg_i=ni, grads=grads)
        return float(loss)
