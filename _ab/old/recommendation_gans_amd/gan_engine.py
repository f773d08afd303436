"""cGAN training engine on the HIP path (rg_gan.hip through the C-ABI).

Holds the generator / discriminator of spotlight/dnn_models/cGAN_models.py in the
flat device layouts of ``rg_gan_layout`` with their optimizer states, turns user
histories + target slates into device batches, and runs the reference's two
iterations (CGANs.py:410-457 discriminator, :370-408 generator) as one C-ABI call
each.  State dicts come in and go out under the reference's parameter names and
shapes (cGAN_models.py), so checkpoints stay ``torch.save({'network': ...})``
compatible with CGANs.py:565-569.

There is no CPU fallback: constructing an engine loads librg_hip.so and needs a
GPU device.
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib
from ._lib import check

OPT_KINDS = {"adam": 0, "sgd": 1, "rms": 2}
G_BN_BUFFERS = ("running_mean", "running_var")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class GANBatch:
    """Device form of one minibatch: histories (B, L) padded with N, target slates (B, S),
    the history items grouped per item (embedding backward) and the real slates as
    sorted W1 column hits (the one-hot rows of CGANs.py:181-198, never materialised)."""

    def __init__(self, hist, slates, N, S, device):
        hist = np.asarray(hist)
        B, L = hist.shape
        h = hist.astype(np.int64)
        if h.min() < 0 or h.max() > N:
            raise ValueError("history ids must lie in [0, num_items] (num_items = padding)")
        self.rows, self.L = B, L
        self.hist = torch.from_numpy(h.astype(np.int32)).to(device).contiguous()
        b_idx = np.repeat(np.arange(B, dtype=np.int64), L)
        flat = h.reshape(-1)
        keep = flat != N
        items, rows = flat[keep], b_idx[keep]
        order = np.lexsort((rows, items))
        items, rows = items[order], rows[order]
        uniq, start = np.unique(items, return_index=True)
        off = np.append(start, len(items)).astype(np.int32)
        self.n_items = len(uniq)
        self.hist_items = torch.from_numpy(np.ascontiguousarray(uniq.astype(np.int32))).to(device)
        self.hist_off = torch.from_numpy(off).to(device)
        self.hist_rows = torch.from_numpy(np.ascontiguousarray(rows.astype(np.int32))).to(device)
        if len(uniq) == 0:      # keep valid pointers
            self.hist_items = torch.zeros(1, dtype=torch.int32, device=device)
            self.hist_rows = torch.zeros(1, dtype=torch.int32, device=device)
        self.slates = None
        self.n_hits = 0
        if slates is not None:
            sl = np.asarray(slates).astype(np.int64)
            if sl.shape != (B, S) or sl.min() < 0 or sl.max() >= N:
                raise ValueError(f"slates must be ({B}, {S}) item ids in [0, {N})")
            self.slates = torch.from_numpy(sl.astype(np.int32)).to(device).contiguous()
            col = (np.arange(S, dtype=np.int64)[None, :] * N + sl).reshape(-1)
            row = np.repeat(np.arange(B, dtype=np.int64), S)
            o = np.lexsort((row, col))
            self.hit_col = torch.from_numpy(col[o].astype(np.int32)).to(device)
            self.hit_row = torch.from_numpy(row[o].astype(np.int32)).to(device)
            edges = np.arange(0, (S * N + 127) // 128 + 1, dtype=np.int64) * 128      # GEMM column tiles
            self.hit_tile_off = torch.from_numpy(np.searchsorted(col[o], edges).astype(np.int32)).to(device)
            self.n_hits = B * S

    def c_struct(self):
        b = _lib.GANBatch()
        b.rows, b.hist_len, b.hist = self.rows, self.L, ptr(self.hist)
        b.slates = ptr(self.slates)
        b.hist_items, b.hist_off, b.hist_rows = ptr(self.hist_items), ptr(self.hist_off), ptr(self.hist_rows)
        b.n_hist_items = self.n_items
        b.n_hits = self.n_hits
        if self.n_hits:
            b.hit_col, b.hit_row, b.hit_tile_off = ptr(self.hit_col), ptr(self.hit_row), ptr(self.hit_tile_off)
        return b


class GANEngine:
    """Generator + discriminator parameters, optimizer states and workspace on one GPU."""

    def __init__(self, g_state, d_state, num_items, slate_size, hidden, emb_dim, z_dim=100, batch_max=256,
                 optimizer="rms", lr=1e-3, device="cuda:0", alpha=0.99, betas=(0.5, 0.999), eps=1e-8, seed=0):
        if optimizer not in OPT_KINDS:
            raise ValueError(f"optimizer must be one of {sorted(OPT_KINDS)}")
        self.lib = _lib.load()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("GANEngine runs on the GPU only (no CPU fallback)")
        self.N, self.S, self.H, self.E, self.Z = num_items, slate_size, hidden, emb_dim, z_dim
        self.dims = _lib.GANDims(num_items, slate_size, hidden, emb_dim, z_dim, batch_max)
        go = (ctypes.c_int64 * (len(_lib.GAN_G_BLOCKS) + 1))()
        do = (ctypes.c_int64 * (len(_lib.GAN_D_BLOCKS) + 1))()
        st = (ctypes.c_int64 * 2)()
        check(self.lib.rg_gan_layout(ctypes.byref(self.dims), go, do, st), "rg_gan_layout")
        self.go = {k: go[i] for i, k in enumerate(_lib.GAN_G_BLOCKS + ["END"])}
        self.do = {k: do[i] for i, k in enumerate(_lib.GAN_D_BLOCKS + ["END"])}
        self.kz, self.ks = st[0], st[1]
        dev = self.device
        self.g = torch.zeros(self.go["END"], dtype=torch.float32, device=dev)
        self.d = torch.zeros(self.do["END"], dtype=torch.float32, device=dev)
        self.opt_kind, self.lr, self.alpha, self.betas, self.eps = optimizer, lr, alpha, betas, eps
        need_m, need_v = optimizer == "adam", optimizer in ("adam", "rms")
        ng, nd = self.go["RM1"], self.do["END"]
        self.g_m = torch.zeros(ng, device=dev) if need_m else None
        self.g_v = torch.zeros(ng, device=dev) if need_v else None
        self.d_m = torch.zeros(nd, device=dev) if need_m else None
        self.d_v = torch.zeros(nd, device=dev) if need_v else None
        self.ws = torch.zeros(int(self.lib.rg_gan_workspace_bytes(ctypes.byref(self.dims))), dtype=torch.uint8,
                              device=dev)
        self.batch_max = batch_max
        self.g_steps = 0            # optimizer steps taken (Adam bias corrections)
        self.d_steps = 0
        self.bn_tracked = [0, 0]    # num_batches_tracked of the two BatchNorms
        self.seed = int(seed) * 0x100000001 + 1
        self.out = torch.zeros(4, dtype=torch.float32, device=dev)
        self.load_g_state(g_state)
        self.load_d_state(d_state)

    # ------------------------------------------------------------------ layouts
    def _gv(self, blk, shape):
        o = self.go[blk]
        return self.g[o:o + int(np.prod(shape))].view(shape)

    def _dv(self, blk, shape):
        o = self.do[blk]
        return self.d[o:o + int(np.prod(shape))].view(shape)

    def load_g_state(self, sd):
        N, S, H, E, Z = self.N, self.S, self.H, self.E, self.Z
        H1 = H // 2
        with torch.no_grad():
            self._gv("EMB", (N + 1, E)).copy_(sd["embedding_layer.weight"])
            self._gv("W1", (H1, self.kz))[:, :Z + E].copy_(sd["layers.0.weight"])
            self._gv("B1", (H1,)).copy_(sd["layers.0.bias"])
            self._gv("GAMMA1", (H1,)).copy_(sd["layers.1.weight"])
            self._gv("BETA1", (H1,)).copy_(sd["layers.1.bias"])
            self._gv("W2", (H, H1)).copy_(sd["layers.4.weight"])
            self._gv("B2", (H,)).copy_(sd["layers.4.bias"])
            self._gv("GAMMA2", (H,)).copy_(sd["layers.5.weight"])
            self._gv("BETA2", (H,)).copy_(sd["layers.5.bias"])
            wh, bh = self._gv("WH", (self.ks, H)), self._gv("BH", (self.ks,))
            for s in range(S):
                wh[s * N:(s + 1) * N].copy_(sd[f"mult_heads.head_{s}.weight"])
                bh[s * N:(s + 1) * N].copy_(sd[f"mult_heads.head_{s}.bias"])
            for k, (bn, w) in enumerate((("layers.1", H1), ("layers.5", H))):
                self._gv(f"RM{k + 1}", (w,)).copy_(sd[bn + ".running_mean"])
                self._gv(f"RV{k + 1}", (w,)).copy_(sd[bn + ".running_var"])
                self.bn_tracked[k] = int(sd.get(bn + ".num_batches_tracked", torch.tensor(0)))

    def load_d_state(self, sd):
        N, S, H, E = self.N, self.S, self.H, self.E
        SN = S * N
        with torch.no_grad():
            self._dv("EMB", (N + 1, E)).copy_(sd["embedding_layer.weight"])
            w1 = sd["layers.0.weight"]
            self._dv("W1E", (2 * H, E)).copy_(w1[:, :E])
            self._dv("W1S", (2 * H, self.ks))[:, :SN].copy_(w1[:, E:])
            self._dv("B1", (2 * H,)).copy_(sd["layers.0.bias"])
            self._dv("W2", (H, 2 * H)).copy_(sd["layers.3.weight"])
            self._dv("B2", (H,)).copy_(sd["layers.3.bias"])
            self._dv("W3", (H // 2, H)).copy_(sd["layers.6.weight"])
            self._dv("B3", (H // 2,)).copy_(sd["layers.6.bias"])
            self._dv("W4", (1, H // 2)).copy_(sd["layers.9.weight"])
            self._dv("B4", (1,)).copy_(sd["layers.9.bias"])

    def g_state_dict(self):
        """The generator's state_dict (reference names and shapes, CPU copies)."""
        N, S, H, E, Z = self.N, self.S, self.H, self.E, self.Z
        H1 = H // 2
        c = lambda t: t.detach().clone().cpu()  # noqa: E731
        sd = {"embedding_layer.weight": c(self._gv("EMB", (N + 1, E))),
              "layers.0.weight": c(self._gv("W1", (H1, self.kz))[:, :Z + E]),
              "layers.0.bias": c(self._gv("B1", (H1,))),
              "layers.1.weight": c(self._gv("GAMMA1", (H1,))), "layers.1.bias": c(self._gv("BETA1", (H1,))),
              "layers.1.running_mean": c(self._gv("RM1", (H1,))), "layers.1.running_var": c(self._gv("RV1", (H1,))),
              "layers.1.num_batches_tracked": torch.tensor(self.bn_tracked[0]),
              "layers.4.weight": c(self._gv("W2", (H, H1))), "layers.4.bias": c(self._gv("B2", (H,))),
              "layers.5.weight": c(self._gv("GAMMA2", (H,))), "layers.5.bias": c(self._gv("BETA2", (H,))),
              "layers.5.running_mean": c(self._gv("RM2", (H,))), "layers.5.running_var": c(self._gv("RV2", (H,))),
              "layers.5.num_batches_tracked": torch.tensor(self.bn_tracked[1])}
        wh, bh = self._gv("WH", (self.ks, H)), self._gv("BH", (self.ks,))
        for s in range(S):
            sd[f"mult_heads.head_{s}.weight"] = c(wh[s * N:(s + 1) * N])
            sd[f"mult_heads.head_{s}.bias"] = c(bh[s * N:(s + 1) * N])
        return sd

    def d_state_dict(self):
        N, S, H, E = self.N, self.S, self.H, self.E
        c = lambda t: t.detach().clone().cpu()  # noqa: E731
        w1 = torch.cat([self._dv("W1E", (2 * H, E)), self._dv("W1S", (2 * H, self.ks))[:, :S * N]], 1)
        return {"embedding_layer.weight": c(self._dv("EMB", (N + 1, E))), "layers.0.weight": c(w1),
                "layers.0.bias": c(self._dv("B1", (2 * H,))),
                "layers.3.weight": c(self._dv("W2", (H, 2 * H))), "layers.3.bias": c(self._dv("B2", (H,))),
                "layers.6.weight": c(self._dv("W3", (H // 2, H))), "layers.6.bias": c(self._dv("B3", (H // 2,))),
                "layers.9.weight": c(self._dv("W4", (1, H // 2))), "layers.9.bias": c(self._dv("B4", (1,)))}

    # ------------------------------------------------------------------ steps
    def _opt(self, t):
        o = _lib.Opt()
        o.kind = OPT_KINDS[self.opt_kind]
        o.lr, o.beta1, o.beta2 = self.lr, self.betas[0], self.betas[1]
        o.eps, o.weight_decay, o.alpha = self.eps, 0.0, self.alpha    # CGANs.py:153-162: weight_decay=0
        o.one_minus_beta1, o.one_minus_beta2, o.one_minus_alpha = 1 - self.betas[0], 1 - self.betas[1], 1 - self.alpha
        if self.opt_kind == "adam":
            o.step_size = self.lr / (1 - self.betas[0] ** t)
            o.bias_correction2_sqrt = math.sqrt(1 - self.betas[1] ** t)
        return o

    def _model(self):
        m = _lib.GANModel()
        m.dims = self.dims
        m.g, m.g_m, m.g_v = ptr(self.g), ptr(self.g_m), ptr(self.g_v)
        m.d, m.d_m, m.d_v = ptr(self.d), ptr(self.d_m), ptr(self.d_v)
        return m

    def _noise(self, rows, z, masks):
        if z is None:
            z = torch.rand(rows, self.Z, device=self.device)
        z = z.to(self.device, torch.float32).contiguous()
        n = _lib.GANNoise()
        n.z = ptr(z)
        keep = [z]
        if masks is not None:
            for i, m in enumerate(masks):
                mt = torch.as_tensor(m).to(self.device, torch.uint8).contiguous()
                keep.append(mt)
                n.masks[i] = mt.data_ptr()
        self.seed += 1
        n.seed = self.seed
        return n, keep

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def check_batch(self, batch):
        if batch.rows > self.batch_max:
            raise ValueError(f"batch of {batch.rows} rows exceeds batch_max {self.batch_max}")

    def d_step(self, batch, z=None, masks=None):
        """CGAN.train_discriminator_iteration.  Returns the device tensor
        [d_loss, mean D(real), mean D(fake)] (no host sync)."""
        self.check_batch(batch)
        if batch.slates is None:
            raise ValueError("the discriminator step needs the batch's real slates")
        noise, keep = self._noise(batch.rows, z, masks)
        self.d_steps += 1
        out = torch.empty(3, dtype=torch.float32, device=self.device)
        b = batch.c_struct()
        check(self.lib.rg_gan_d_step(self._stream(), ctypes.byref(self._model()), ptr(self.ws), ctypes.byref(b),
                                     ctypes.byref(noise), ctypes.byref(self._opt(self.d_steps)), ptr(out)),
              "rg_gan_d_step")
        self.bn_tracked = [t + 1 for t in self.bn_tracked]
        self._keep = keep
        return out

    def g_step(self, batch, z=None, masks=None, slates=True):
        """CGAN.train_generator_iteration.  Returns (device [g_loss], slates (rows, S) float
        of the eval-mode generator on the same z after the step, or None)."""
        self.check_batch(batch)
        noise, keep = self._noise(batch.rows, z, masks)
        self.g_steps += 1
        out = torch.empty(1, dtype=torch.float32, device=self.device)
        sl = torch.empty(batch.rows, self.S, dtype=torch.float32, device=self.device) if slates else None
        b = batch.c_struct()
        check(self.lib.rg_gan_g_step(self._stream(), ctypes.byref(self._model()), ptr(self.ws), ctypes.byref(b),
                                     ctypes.byref(noise), ctypes.byref(self._opt(self.g_steps)), ptr(out), ptr(sl)),
              "rg_gan_g_step")
        self.bn_tracked = [t + 1 for t in self.bn_tracked]
        self._keep = keep
        return out, sl

    def generate(self, batch, z=None):
        """generator.forward(z, hist, inference=True): (rows, S) float item ids."""
        self.check_batch(batch)
        if z is None:
            z = torch.rand(batch.rows, self.Z, device=self.device)
        z = z.to(self.device, torch.float32).contiguous()
        sl = torch.empty(batch.rows, self.S, dtype=torch.float32, device=self.device)
        b = batch.c_struct()
        check(self.lib.rg_gan_generate(self._stream(), ctypes.byref(self._model()), ptr(self.ws), ctypes.byref(b),
                                       ptr(z), ptr(sl)), "rg_gan_generate")
        self._keep = [z]
        return sl

    def workspace_view(self, which, shape):
        off = int(self.lib.rg_gan_workspace_offset(ctypes.byref(self.dims), which))
        n = int(np.prod(shape))
        return self.ws[off:off + 4 * n].view(torch.float32).view(shape)

    def last_fake(self, rows):
        """G(z) of the last step, (rows, S*N)."""
        return self.workspace_view(_lib.GAN_WS_FAKE, (rows, self.ks))[:, :self.S * self.N]

    def last_d_out(self, rows):
        return self.workspace_view(_lib.GAN_WS_DOUT, (rows,))
