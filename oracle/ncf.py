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

Samples of the fp32 rounding noise (tests/parity_report.py's elementwise band): ``order_seed``
runs a step with the examples, the input features and every hidden layer's units in seeded
orders (every batch sum and every product's inner sum re-ordered, forward and backward);
``kink_flip`` decides every LeakyReLU (mlp.py:36, neuMF.py:48) whose pre-activation lies within
fp32 rounding of the kink the other way from its exact value -- the activation decision a
different fp32 order of the forward dot product can take (see ``kink_band``).
"""
import math

import torch

from . import mf as omf
from . import rng as orng

U32 = 2.0 ** -24          # fp32 unit roundoff


def kink_band(a, W, b, c):
    """The exact (float64) pre-activations z of a @ W.T + b and the rounding band c * u *
    sqrt(K + 1) * S around them (S = |a| @ |W|.T + |b|, K inputs): the typical size of an fp32
    dot product's rounding error in some summation order is u * sqrt(K) * S, so a z inside the
    band is a decision on which fp32 orders of the same sum disagree."""
    a64, W64, b64 = a.double(), W.double(), b.double()
    z64 = a64.mm(W64.t()) + b64
    S = a64.abs().mm(W64.abs().t()) + b64.abs()
    return z64, c * U32 * math.sqrt(W.shape[1] + 1) * S


def _decide(z, a, W, b, flip):
    """The LeakyReLU branch (True: z > 0 side) and the number of flipped decisions."""
    if flip is None:
        return z > 0, None
    z64, band = kink_band(a, W, b, flip)
    amb = z64.abs() <= band
    return torch.where(amb, z64 <= 0, z > 0), amb


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


def _tower(lin, x, masks, cache, flip):
    """Hidden layers: Linear -> LeakyReLU(0.1) -> Dropout(0.5) (mlp.py:30-41, neuMF.py:43-49)."""
    a = x
    for k, (W, b) in enumerate(lin):
        z = a.mm(W.t()) + b
        pos, amb = _decide(z, a, W, b, flip)
        r = torch.where(pos, z, z * LRELU)
        keep = masks[k].to(z.dtype)
        a = r * (keep * DROP_SCALE)
        cache["z"].append(z)
        cache["pos"].append(pos)
        cache["a"].append(a)
        if amb is not None:   # flipped decisions that reach the loss (dropout keeps the unit)
            cache["flips"] += int((amb & (keep > 0)).sum())
    return a


def forward(P, u, i, masks, xperm=None, flip=None):
    """Returns p (N,1) and the cache for backward.  ``masks``: per hidden layer (N, out) 0/1.
    ``xperm``: the input features in that order (P's first layer permuted to match).
    ``flip``: kink_flip's c (None: every branch by the sign of the fp32 pre-activation)."""
    Ue, Ie = P.emb()
    x = torch.cat([Ue[u], Ie[i]], dim=-1)
    if xperm is not None:
        x = x[:, xperm]
    lin = P.linears()
    cache = {"x": x, "z": [], "pos": [], "a": [x], "flips": 0}
    a = _tower(lin[:-1], x, masks, cache, flip)
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
            cache.setdefault("gr", {})[k - 1] = da
            dz = torch.where(cache["pos"][k - 1], da, da * LRELU)
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


def kink_envelope(P, u, i, masks, cache, c, env, n_emb):
    """Adds to ``env`` (per parameter, float64, the oracle's parameter order) the absolute change
    of this batch's gradient that flipping each LeakyReLU decision within kink_band(c) of the
    kink would make -- the reachable set of any fp32 order's decisions at rounding level, by the
    triangle inequality over the flips.  A flip of unit k of hidden layer L for example e changes
    its slope s -> s' (1 <-> 0.1): dz_L[e, k] moves by (s' - s) * gr (gr: the gradient at the
    unit's LeakyReLU output, dropout applied), which moves dW_L[k, :], db_L[k] and, through the
    example's own backward, every lower layer and the example's user / item embedding rows.  The
    forward value moves by (s' - s) |z| <= the band itself, a second-order change neglected here.
    Returns the number of kept decisions inside the band.  (Call after the backward, float64.)"""
    lin = P.linears()
    hid = lin[:-1]
    E = P.emb()[0].shape[1]
    count = 0
    for L, (W, b) in enumerate(hid):
        a_in = cache["a"][L]
        z64, band = kink_band(a_in, W, b, c)
        keep = masks[L] > 0
        amb = (z64.abs() <= band) & keep
        for e, k in amb.nonzero().tolist():
            count += 1
            pos = bool(cache["pos"][L][e, k])
            d = float(cache["gr"][L][e, k]) * ((LRELU - 1.0) if pos else (1.0 - LRELU))
            ddz = torch.zeros(W.shape[0], dtype=torch.float64)
            ddz[k] = d
            for j in range(L, -1, -1):              # the example's backward from layer L down
                Wj = hid[j][0].double()
                env[n_emb + 2 * j] += ddz.abs()[:, None] * cache["a"][j][e].double().abs()[None, :]
                env[n_emb + 2 * j + 1] += ddz.abs()
                dda = ddz @ Wj
                if j > 0:
                    keepj = masks[j - 1][e].double() * DROP_SCALE
                    slope = torch.where(cache["pos"][j - 1][e], 1.0, LRELU).double()
                    ddz = dda * keepj * slope
            env[0][u[e]] += dda[:E].abs()
            env[1][i[e]] += dda[E:].abs()
    return count


class NCFOracle:
    """One run_train_iteration (implicit.py:347-364) of the NCF MLP per ``step``."""

    N_EMB = 2                     # embedding tables before the Linears in parameter order

    def __init__(self, tensors, names, pool_u, pool_i, mt_state, loss="pointwise", lr=1e-2, weight_decay=1e-5,
                 n_neg=5, batch_size=256, betas=(0.5, 0.999), order_seed=None, kink_flip=None, kink_env=None):
        self.P = MLPParams(tensors, names)
        # order_seed (pointwise, test infrastructure): run the step over the examples, the input
        # features and every hidden layer's units in seeded orders -- the same arithmetic summed
        # in other fp32 orders (batch sums and every product's inner sum), a further sample of
        # the rounding noise for tests/parity_report.py's elementwise band
        assert order_seed is None or loss == "pointwise"
        self.order = None if order_seed is None else torch.Generator().manual_seed(order_seed)
        # kink_flip (test infrastructure): c of kink_band -- every LeakyReLU decision within
        # rounding of the kink goes the other way from the exact sign of this run's own state; the
        # count of such decisions that reach the loss, per step, in self.flips
        self.kink_flip = kink_flip
        self.flips = []
        # kink_env (float64, test infrastructure): c of kink_band -- each step also bounds, per
        # element, how far flipping any subset of the kept LeakyReLU decisions within the band
        # moves the parameters after the optimizer (kink_envelope through Optim.sensitivity):
        # self.kink_noise, with the count of such decisions in self.kink_count
        assert kink_env is None or order_seed is None
        self.kink_env = kink_env
        self.kink_noise, self.kink_count = None, []
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
        (P', masks -> masks', grads' -> grads, xperm); identity without order_seed.  The output
        Linear's inputs past the tower's last hidden layer (NeuMF's GMF products) keep their
        order."""
        if self.order is None:
            return self.P, (lambda m: m), (lambda g: g), None
        ne = self.N_EMB
        lin = self.P.linears()
        E2 = lin[0][0].shape[1]
        xperm = torch.randperm(E2, generator=self.order)
        hperm = [torch.randperm(W.shape[0], generator=self.order) for W, _ in lin[:-1]]
        ins = [xperm] + hperm                                 # input order of linear k
        Wo = lin[-1][0]
        if Wo.shape[1] > len(ins[-1]):
            ins[-1] = torch.cat([ins[-1], torch.arange(len(ins[-1]), Wo.shape[1])])
        t = list(self.P.t[:ne])
        for k, (W, b) in enumerate(lin):
            rows = hperm[k] if k < len(hperm) else torch.arange(W.shape[0])
            t += [W[rows][:, ins[k]], b[rows]]
        Pp = type(self.P)(t, self.P.names)

        def masks_p(ms):
            return [m[:, hperm[k]] for k, m in enumerate(ms)]

        def grads_back(g):
            out = list(g[:ne])
            for k in range(len(lin)):
                dW, db = g[ne + 2 * k], g[ne + 1 + 2 * k]
                rows = torch.argsort(hperm[k]) if k < len(hperm) else torch.arange(dW.shape[0])
                out += [dW[rows][:, torch.argsort(ins[k])], db[rows]]
            return out
        return Pp, masks_p, grads_back, xperm

    _fwd = staticmethod(forward)
    _bwd = staticmethod(backward)

    def _envelope(self, P, pos, neg, grads):
        if self.kink_env is None:
            return
        env = [torch.zeros(t.shape, dtype=torch.float64) for t in self.P.t]
        n = sum(kink_envelope(P, uu, ii, mm, cc, self.kink_env, env, self.N_EMB) for uu, ii, mm, cc in (pos, neg))
        self.kink_count.append(n)
        dstate = [(torch.zeros_like(e), torch.zeros_like(e)) for e in env]
        self.kink_noise = self.opt.sensitivity(self.P.t, grads, env, dstate)

    def step(self, pos_u, pos_i, masks_pos, masks_neg, return_all=False):
        u = torch.as_tensor(pos_u).long()
        i = torch.as_tensor(pos_i).long()
        u, i, masks_pos = self._permuted(u, i, masks_pos)
        P, mperm, gback, xperm = self._unit_orders()
        masks_pos = mperm(masks_pos)
        p_pos, c_pos = self._fwd(P, u, i, masks_pos, xperm, self.kink_flip)
        idx, nu, ni = self.draw(self.n * self.batch_size)
        nu, ni, masks_neg = self._permuted(nu, ni, masks_neg)
        masks_neg = mperm(masks_neg)
        p_neg, c_neg = self._fwd(P, nu, ni, masks_neg, xperm, self.kink_flip)
        self.flips.append(c_pos["flips"] + c_neg["flips"])
        kind = self.loss_kind
        loss, dpp, dpn = omf.loss_and_dp(kind, p_pos.reshape(-1), p_neg.reshape(-1), self.n, self.batch_size)
        g1 = self._bwd(P, u, i, masks_pos, c_pos, dpp.reshape(-1, 1), xperm)
        g2 = self._bwd(P, nu, ni, masks_neg, c_neg, dpn.reshape(-1, 1), xperm)
        grads = gback([a + b for a, b in zip(g1, g2)])
        self._envelope(P, (u, i, masks_pos, c_pos), (nu, ni, masks_neg, c_neg), grads)
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


def neumf_forward(P, u, i, masks, xperm=None, flip=None):
    """neuMF.py:34-55: tower over cat(U_mlp[u], I_mlp[i]), GMF = U_mf[u] * I_mf[i],
    sigmoid(affine_output(cat(tower, GMF))).  ``xperm`` / ``flip`` as forward's."""
    Ue, Ie = P.emb()
    Um, Im = P.emb_mf()
    x = torch.cat([Ue[u], Ie[i]], dim=-1)
    if xperm is not None:
        x = x[:, xperm]
    lin = P.linears()
    cache = {"z": [], "pos": [], "a": [x], "flips": 0}
    a = _tower(lin[:-1], x, masks, cache, flip)
    gmf = Um[u] * Im[i]
    v = torch.cat([a, gmf], dim=-1)
    W, b = lin[-1]
    p = torch.sigmoid(v.mm(W.t()) + b)
    cache.update(p=p, v=v, gmf_u=Um[u], gmf_i=Im[i])
    return p, cache


def neumf_backward(P, u, i, masks, cache, dp, xperm=None):
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
        cache.setdefault("gr", {})[k] = da
        dzk = torch.where(cache["pos"][k], da, da * LRELU)
        grads_lin.append((dzk.t().mm(cache["a"][k]), dzk.sum(0)))
        da = dzk.mm(Wk)
    grads_lin.reverse()
    Ue, Ie = P.emb()
    Um, Im = P.emb_mf()
    E = Ue.shape[1]
    if xperm is not None:
        da = da[:, torch.argsort(xperm)]
    out = [torch.zeros_like(Ue).index_add_(0, u, da[:, :E]), torch.zeros_like(Ie).index_add_(0, i, da[:, E:]),
           torch.zeros_like(Um).index_add_(0, u, dUm_rows), torch.zeros_like(Im).index_add_(0, i, dIm_rows)]
    for dW, db in grads_lin:
        out += [dW, db]
    return out


class NeuMFOracle(NCFOracle):
    """One run_train_iteration (implicit.py:347-364) of NeuMF per ``step``."""

    N_EMB = 4
    _fwd = staticmethod(neumf_forward)
    _bwd = staticmethod(neumf_backward)

    def __init__(self, tensors, names, *a, **k):
        super().__init__(tensors, names, *a, **k)
        self.P = NeuMFParams(tensors, names)
        self.opt = omf.Optim("adam", self.P.t, self.opt_lr, self.opt_wd, betas=self.opt_betas)
