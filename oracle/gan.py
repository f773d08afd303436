"""CPU restatement of the reference's cGAN step (TEST INFRASTRUCTURE ONLY: imported by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product).

Follows, in float64 numpy with the dropout masks and noise given:

* ``generator.forward`` (spotlight/dnn_models/cGAN_models.py:41-68): sum of the
  history's item embeddings (padding row N is zero, ``padding_idx``) -> cat([z, e])
  -> LeakyReLU(0.2) -> per hidden layer [Linear, BatchNorm1d (batch stats in train
  mode, running stats in eval), Dropout(0.1), LeakyReLU(0.2)] -> S heads
  Linear(H -> N) + tanh; ``inference=True`` -> argmax per head (first maximum).
* ``discriminator.forward`` (:102-109): cat([sum of history embeddings, slate])
  -> per hidden layer [Linear, Dropout(0.3), LeakyReLU(0.2)] -> Linear(-> 1).  The
  LeakyReLU result at :105 is discarded by the reference and so is not computed.
* ``CGAN.train_discriminator_iteration`` (CGANs.py:410-457): clamp every D
  parameter to +-0.01, D(one-hot real), G(z) (train: BatchNorm running stats move),
  D(fake.detach()), d_loss = mean(D fake) - mean(D real), D optimizer step.
* ``CGAN.train_generator_iteration`` (CGANs.py:370-408): G(z) -> D (train mode,
  its parameters frozen) -> g_loss = -mean, G optimizer step, then eval-mode
  inference on the same z.  The reference's training precision/recall
  (``precision_recall_slates_atk``, spotlight/evaluation.py:394-412) intersects
  sets of 0-d torch tensors, which hash by identity, so it is 0 for every row.
* optimizers: torch.optim RMSprop (alpha 0.99, eps 1e-8), Adam (betas (0.5, 0.999)
  from spotlight/optimizers.py:10-16), SGD; weight decay 0 (CGANs.py:153-162).

Pinned against tests/golden/gan_*.npz (the reference's own steps, recorded by
tests/golden/make_golden.py ``gan``).
"""
import numpy as np

LRELU = 0.2
BN_EPS = 1e-5
BN_MOMENTUM = 0.1
CLAMP = 0.01


def g_hidden(H):
    return [H // 2, H]                      # slate_generation.py:48


def d_hidden(H):
    return [2 * H, H, H // 2]               # slate_generation.py:53


def lrelu(x):
    return np.where(x > 0, x, LRELU * x)


def lrelu_grad(x):
    return np.where(x > 0, 1.0, LRELU)


def hist_sum(emb, hist):
    """emb(hist).sum(1); hist (B, L) holds float ids, padding = N (a zero row)."""
    return emb[hist.astype(np.int64)].sum(1)


def hist_scatter(grad, hist, pad, dE):
    """embedding backward with padding_idx: rows != pad accumulate the row's grad."""
    idx = hist.astype(np.int64)
    for b in range(idx.shape[0]):
        for l in range(idx.shape[1]):
            if idx[b, l] != pad:
                grad[idx[b, l]] += dE[b]


class Optimizer:
    """torch.optim single-tensor CPU paths, weight_decay = 0."""

    def __init__(self, kind, lr, alpha=0.99, betas=(0.5, 0.999), eps=1e-8):
        self.kind, self.lr, self.alpha, self.betas, self.eps = kind, lr, alpha, betas, eps
        self.state = {}
        self.t = 0

    def step(self, params, grads):
        self.t += 1
        for k, g in grads.items():
            p = params[k]
            st = self.state.setdefault(k, [np.zeros_like(p), np.zeros_like(p)])
            if self.kind == "rms":
                st[1] = self.alpha * st[1] + (1 - self.alpha) * g * g
                params[k] = p - self.lr * g / (np.sqrt(st[1]) + self.eps)
            elif self.kind == "adam":
                b1, b2 = self.betas
                st[0] = st[0] + (1 - b1) * (g - st[0])
                st[1] = b2 * st[1] + (1 - b2) * g * g
                bc1, bc2 = 1 - b1 ** self.t, 1 - b2 ** self.t
                params[k] = p - (self.lr / bc1) * st[0] / (np.sqrt(st[1]) / np.sqrt(bc2) + self.eps)
            else:
                params[k] = p - self.lr * g


class GANOracle:
    """G / D parameters under the reference's state_dict names (float64)."""

    def __init__(self, g_init, d_init, N, S, H, E, Z=100, opt="rms", lr=1e-3, dtype=np.float64):
        self.N, self.S, self.H, self.E, self.Z = N, S, H, E, Z
        # dtype float32: the same restatement in fp32 NumPy arithmetic (another fp32 summation
        # order, the fp32 side of tensor_parity's band where the reference cannot run)
        self.G = {k: np.asarray(v, dtype).copy() for k, v in g_init.items()}
        self.D = {k: np.asarray(v, dtype).copy() for k, v in d_init.items()}
        self.gh, self.dh = g_hidden(H), d_hidden(H)
        self.g_lin = [f"layers.{4 * i}" for i in range(len(self.gh))]
        self.g_bn = [f"layers.{4 * i + 1}" for i in range(len(self.gh))]
        self.d_lin = [f"layers.{3 * i}" for i in range(len(self.dh) + 1)]
        self.g_opt = Optimizer(opt, lr)
        self.d_opt = Optimizer(opt, lr)
        self.g_params = [k for k in self.G if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]

    # ---------------------------------------------------------------- generator
    def g_forward(self, z, hist, masks=None, scale=None, train=True):
        G, cache = self.G, {}
        e = hist_sum(G["embedding_layer.weight"], hist)
        x0 = np.concatenate([z, e], 1)
        a = lrelu(x0)
        cache["x0"], cache["layers"] = x0, []
        for k, (lin, bn) in enumerate(zip(self.g_lin, self.g_bn)):
            y = a @ G[lin + ".weight"].T + G[lin + ".bias"]
            if train:
                mu, var = y.mean(0), y.var(0)
                B = y.shape[0]
                G[bn + ".running_mean"] = (1 - BN_MOMENTUM) * G[bn + ".running_mean"] + BN_MOMENTUM * mu
                G[bn + ".running_var"] = (1 - BN_MOMENTUM) * G[bn + ".running_var"] + \
                    BN_MOMENTUM * var * B / (B - 1)
                G[bn + ".num_batches_tracked"] = G[bn + ".num_batches_tracked"] + 1
            else:
                mu, var = G[bn + ".running_mean"], G[bn + ".running_var"]
            rstd = 1.0 / np.sqrt(var + BN_EPS)
            yhat = (y - mu) * rstd
            o = yhat * G[bn + ".weight"] + G[bn + ".bias"]
            mult = masks[k] * scale if train else np.ones_like(o)
            d = o * mult
            cache["layers"].append(dict(a_in=a, yhat=yhat, rstd=rstd, mult=mult, d=d))
            a = lrelu(d)
        cache["a"] = a
        heads = [np.tanh(a @ G[f"mult_heads.head_{s}.weight"].T + G[f"mult_heads.head_{s}.bias"])
                 for s in range(self.S)]
        cache["t"] = heads
        return heads, cache

    def g_backward(self, hist, cache, dfake):
        G, S, N = self.G, self.S, self.N
        grads = {}
        a = cache["a"]
        da = np.zeros_like(a)
        for s in range(S):
            dl = dfake[:, s * N:(s + 1) * N] * (1 - cache["t"][s] ** 2)
            grads[f"mult_heads.head_{s}.weight"] = dl.T @ a
            grads[f"mult_heads.head_{s}.bias"] = dl.sum(0)
            da += dl @ G[f"mult_heads.head_{s}.weight"]
        for k in reversed(range(len(self.gh))):
            L, lin, bn = cache["layers"][k], self.g_lin[k], self.g_bn[k]
            dd = da * lrelu_grad(L["d"])
            do = dd * L["mult"]
            grads[bn + ".weight"] = (do * L["yhat"]).sum(0)
            grads[bn + ".bias"] = do.sum(0)
            dyhat = do * G[bn + ".weight"]
            dy = L["rstd"] * (dyhat - dyhat.mean(0) - L["yhat"] * (dyhat * L["yhat"]).mean(0))
            grads[lin + ".weight"] = dy.T @ L["a_in"]
            grads[lin + ".bias"] = dy.sum(0)
            da = dy @ G[lin + ".weight"]
        dx0 = da * lrelu_grad(cache["x0"])
        gE = np.zeros_like(G["embedding_layer.weight"])
        hist_scatter(gE, hist, self.N, dx0[:, self.Z:])
        grads["embedding_layer.weight"] = gE
        return grads

    def g_infer(self, z, hist):
        heads, _ = self.g_forward(z, hist, train=False)
        return np.stack([np.argmax(h.astype(np.float32), 1) for h in heads], 1).astype(np.float32)

    # ------------------------------------------------------------ discriminator
    def d_forward(self, slate_dense, hist, masks, scale):
        D, cache = self.D, {"h": []}
        c = hist_sum(D["embedding_layer.weight"], hist)
        x = np.concatenate([c, slate_dense], 1)
        h = x
        for k in range(len(self.dh)):
            lin = self.d_lin[k]
            u = (h @ D[lin + ".weight"].T + D[lin + ".bias"]) * (masks[k] * scale)
            cache["h"].append(dict(h_in=h, u=u, mult=masks[k] * scale))
            h = lrelu(u)
        out = h @ D[self.d_lin[-1] + ".weight"].T + D[self.d_lin[-1] + ".bias"]
        cache["h_last"] = h
        return out, cache

    def d_backward(self, hist, cache, dout, grads=None, need_dx=False):
        D = self.D
        grads = grads if grads is not None else {k: np.zeros_like(v) for k, v in D.items()}
        last = self.d_lin[-1]
        grads[last + ".weight"] += dout.T @ cache["h_last"]
        grads[last + ".bias"] += dout.sum(0)
        dh = dout @ D[last + ".weight"]
        for k in reversed(range(len(self.dh))):
            C, lin = cache["h"][k], self.d_lin[k]
            dlin = dh * lrelu_grad(C["u"]) * C["mult"]
            grads[lin + ".weight"] += dlin.T @ C["h_in"]
            grads[lin + ".bias"] += dlin.sum(0)
            dh = dlin @ D[lin + ".weight"]
        dc = dh[:, :self.E]
        hist_scatter(grads["embedding_layer.weight"], hist, self.N, dc)
        return grads, (dh[:, self.E:] if need_dx else None)

    def one_hot(self, slates):
        B = slates.shape[0]
        x = np.zeros((B, self.S * self.N))
        for b in range(B):
            for s in range(self.S):
                x[b, s * self.N + int(slates[b, s])] = 1.0
        return x

    def pre_bn_biases(self):
        """Linear biases feeding a BatchNorm: their gradient is identically zero (the
        batch mean removes them), so after an RMSprop/Adam step their value is set by
        the rounding noise of that zero sum and is not comparable across implementations."""
        return [lin + ".bias" for lin in self.g_lin]

    # -------------------------------------------------------------------- steps
    def d_step(self, hist, slates, z, masks, scales):
        """masks: D(real) x3, G x2, D(fake) x3 (the reference's call order)."""
        sg, sd = scales
        for k in self.D:
            self.D[k] = np.clip(self.D[k], -CLAMP, CLAMP)
        B = hist.shape[0]
        d_real, c_real = self.d_forward(self.one_hot(slates), hist, masks[0:3], sd)
        heads, _ = self.g_forward(z, hist, masks[3:5], sg, train=True)
        fake = np.concatenate(heads, 1)
        d_fake, c_fake = self.d_forward(fake, hist, masks[5:8], sd)
        loss = d_fake.mean() - d_real.mean()
        grads, _ = self.d_backward(hist, c_real, np.full((B, 1), -1.0 / B))
        grads, _ = self.d_backward(hist, c_fake, np.full((B, 1), 1.0 / B), grads)
        self.last_grads = grads
        self.d_opt.step(self.D, grads)
        return loss, d_real, d_fake, fake

    def g_step(self, hist, z, masks, scales):
        """masks: G x2, D(fake) x3.  Returns (g_loss, D(fake), inference slates)."""
        sg, sd = scales
        B = hist.shape[0]
        heads, gc = self.g_forward(z, hist, masks[0:2], sg, train=True)
        fake = np.concatenate(heads, 1)
        d_fake, dcache = self.d_forward(fake, hist, masks[2:5], sd)
        loss = -d_fake.mean()
        _, dfake = self.d_backward(hist, dcache, np.full((B, 1), -1.0 / B), need_dx=True)
        grads = self.g_backward(hist, gc, dfake)
        self.last_grads = grads
        self.g_opt.step(self.G, {k: grads[k] for k in self.g_params})
        slates = self.g_infer(z, hist)
        return loss, d_fake, slates
