"""Device-resident NCF MLP training engine: the fused replacement of
run_train_iteration (implicit.py:347-364) for the reference's MLP representation
(spotlight/dnn_models/mlp.py:5-46; layers as ncf_spotlight.py:53-56).

Per step: the native stepper provides the step's CPython-exact negatives
(rg_mt_generate + rg_mf_prepare, shared with the MF path), then
rg_ncf_pairs (fused MLP forward / loss / backward on MFMA) -> rg_ncf_update
(MLP weight-gradient reduce + optimizer) -> rg_ncf_apply (embedding pull +
optimizer over every row).  Adaptive hinge runs scores -> rg_ncf_adapt_dp ->
given-dp.  Dropout: recorded masks (parity with the reference's CPU generator)
or a per-(step, example, unit) hash (the documented device RNG).

NeuMF (spotlight/dnn_models/neuMF.py:7-55): pass the GMF tables (``mf_user_w``,
``mf_item_w``); the same kernels run with mf_dim = M, the MLP parameters end in
affine_output (1 x (8 + M)) and its bias, and rg_neumf_apply updates the GMF tables
before the MLP tables.

Data parallelism (``world_size`` > 1, one process per GPU; replicated and reference-exact):
rank r takes columns [r*B, (r+1)*B) of each global batch of R*B positives and of ONE global
draw of n*R*B negatives over the full pool (implicit.py:262, :290, :351-354; dropout keyed
by the global example), with loss means over the global batch; the embedding, GMF and MLP
data gradients (rg_ncf_grads, rg_ncf_mlp_grad) go into one flat buffer that is all-reduced
(RCCL ``comm``, or ``allreduce`` e.g. torch.distributed), then every rank applies the same
update (rg_ncf_apply_dense, rg_ncf_mlp_apply).  R ranks at batch B equal one process at
batch R*B."""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import LOSS_KINDS, OPT_KINDS, RG_MF_LIST_CAP, RG_MF_MAX_NEG, check, ptr
from .mf_engine import build_plan, build_plans


class NCFEngine:
    def __init__(self, user_w, item_w, mlp_params, pool_u, pool_i, mt_state, *, loss="pointwise", optimizer="adam",
                 lr=1e-3, weight_decay=0.0, betas=(0.5, 0.999), eps=1e-8, alpha=0.99, n_neg=5, batch_size=256,
                 device="cuda", seed=0, mf_user_w=None, mf_item_w=None, rank=0, world_size=1, comm=None):
        _lib.require_gpu()
        self.rank, self.world, self.comm = int(rank), int(world_size), comm
        if loss not in LOSS_KINDS or loss == "pointwise_pos":   # the NCF kernels have no positives-only loss
            raise ValueError(f"unknown loss {loss!r}")
        if optimizer not in OPT_KINDS:
            raise ValueError(f"unknown optimizer {optimizer!r}")
        if not 1 <= n_neg <= RG_MF_MAX_NEG:
            raise ValueError(f"num_negative_samples must be in [1, {RG_MF_MAX_NEG}]")
        self.lib = lib = _lib.load()
        self.device = dev = torch.device(device)
        self.U, self.I = int(user_w.shape[0]), int(item_w.shape[0])
        self.E = E = int(user_w.shape[1])
        self.neumf = mf_user_w is not None
        if self.neumf != (mf_item_w is not None):
            raise ValueError("NeuMF needs both GMF tables")
        self.M = int(mf_user_w.shape[1]) if self.neumf else 0
        self.P = int(lib.rg_neumf_param_len(E, self.M) if self.neumf else lib.rg_ncf_mlp_len(E))
        if self.P < 0:
            raise ValueError("NCF embedding_dim must be 8, 16, 32 or 64 (NeuMF mf_embedding_dim in [1, 128])")
        f32 = dict(dtype=torch.float32, device=dev)
        self.user_w = torch.as_tensor(user_w, dtype=torch.float32).to(dev).contiguous()
        self.item_w = torch.as_tensor(item_w, dtype=torch.float32).to(dev).contiguous()
        self.mf_w = [torch.as_tensor(t, dtype=torch.float32).to(dev).contiguous() for t in (mf_user_w, mf_item_w)] \
            if self.neumf else [None, None]
        if self.neumf and (self.mf_w[0].shape[0] != self.U or self.mf_w[1].shape[0] != self.I
                           or self.mf_w[1].shape[1] != self.M):
            raise ValueError("GMF tables must be [num_users, M] and [num_items, M]")
        flat = torch.cat([torch.as_tensor(p, dtype=torch.float32).reshape(-1) for p in mlp_params])
        if flat.numel() != self.P:
            raise ValueError(f"MLP parameters have {flat.numel()} values, the E={E} layout has {self.P}")
        self.mlp_shapes = [tuple(torch.as_tensor(p).shape) for p in mlp_params]
        self.mlp = flat.to(dev).contiguous()
        self.opt_kind = optimizer
        st = lambda t: torch.zeros_like(t)
        tabs_all = [self.user_w, self.item_w, self.mlp] + (self.mf_w if self.neumf else [])
        self.m = [st(t) for t in tabs_all] if optimizer == "adam" else [None] * len(tabs_all)
        self.v = [st(t) for t in tabs_all] if optimizer != "sgd" else [None] * len(tabs_all)
        self.lr, self.wd, self.betas, self.eps, self.alpha = lr, weight_decay, betas, eps, alpha
        pu = np.asarray(pool_u, dtype=np.int64)
        pi = np.asarray(pool_i, dtype=np.int64)
        if len(pu) == 0 or len(pu) != len(pi) or pu.min() < 0 or pu.max() >= self.U or pi.min() < 0 \
                or pi.max() >= self.I:
            raise ValueError("negative pool empty or outside the tables")
        self.pool = torch.from_numpy(np.stack([pu, pi], 1).astype(np.int32)).to(dev).contiguous()
        self.loss, self.n_neg, self.batch_size = loss, int(n_neg), int(batch_size)
        B, n = self.batch_size, self.n_neg
        self.tile_rows = int(lib.rg_ncf_rows_per_tile(E, self.M))
        self.tc = int(lib.rg_ncf_cols_per_tile(n, E, self.M))
        self.tiles = int(lib.rg_ncf_tiles(B, n, E, self.M))
        self.rows = self.tiles * self.tile_rows
        self.blocks = int(lib.rg_ncf_blocks(B, n, E, self.M))
        self.units = int(lib.rg_ncf_mask_units(E))
        rows = self.U + self.I
        self.row_count = torch.zeros(rows, dtype=torch.int32, device=dev)
        self.row_list = torch.empty(rows * RG_MF_LIST_CAP * 2, dtype=torch.int32, device=dev)
        # overflow accumulators: int64 fixed point (order-independent sums, rg_common.h fix_add)
        self.hot_grad = torch.zeros(rows * E, dtype=torch.int64, device=dev)
        self.hot_bias = torch.zeros(rows, dtype=torch.int64, device=dev)
        self.partials = torch.zeros(2 * max(self.tiles, 1), **f32)
        self.adapt_partials = torch.zeros(2, **f32)
        # adaptive hinge over several ranks: per-rank (score, draw index) slots, the active count,
        # this rank's argmax row (rg_ncf_adapt_local / _global / _winner)
        self.adapt_slots = torch.zeros(4 * max(self.world, 1), **f32)
        self.adapt_count = torch.zeros(1, **f32)
        self.adapt_row = torch.zeros(1, dtype=torch.int32, device=dev)
        self.part_row = torch.zeros(B * E, **f32)
        self.contrib = torch.zeros(self.rows * 2 * E, **f32)
        self.mlp_partials = torch.zeros(self.blocks * self.P, **f32)
        self.scores_buf = torch.zeros(self.rows, **f32)
        self.dp_buf = torch.zeros(self.rows, **f32)
        self.loss_out = torch.zeros(1, **f32)
        self.neg_cols = B * self.world
        M = self.M
        # data parallel: [embedding rows (U+I)(E+1)+1 | GMF rows (U+I)(M+1)+1 | MLP P+1], one all-reduce
        self.dp_flat = None
        if self.world > 1:
            ne, nm = rows * (E + 1) + 1, (rows * (M + 1) + 1) if self.neumf else 0
            self.dp_flat = torch.zeros(ne + nm + self.P + 1, **f32)
            self.dp_emb, self.dp_gmf = self.dp_flat[:ne], self.dp_flat[ne:ne + nm]
            self.dp_mlp = self.dp_flat[ne + nm:]
        self.mf_contrib = torch.zeros(self.rows * 2 * M, **f32) if self.neumf else None
        self.mf_hot_grad = torch.zeros(rows * M, dtype=torch.int64, device=dev) if self.neumf else None
        self.mf_part_row = torch.zeros(B * M, **f32) if self.neumf else None
        self.pairs = [torch.zeros(int(lib.rg_mf_pairs_len(B, n)), dtype=torch.int32, device=dev) for _ in range(2)]
        self.mt_buf = torch.from_numpy(np.ascontiguousarray(np.asarray(mt_state, np.uint32)).view(np.int32)).to(dev)
        self.seed = int(seed)
        self.t = 0
        self.kernel_events = None     # optional (start, end) torch.cuda.Event pair around rg_ncf_pairs
        self._prefetch_side = _lib.ab_build() and os.environ.get("RG_NCF_PREFETCH_SIDE") == "1"
        # single rank: the step's tail in one launch (rg_ncf_tail); False runs the three separate
        # calls it replaces (rg_ncf_update, rg_ncf_apply / rg_neumf_apply, the inline prefetch)
        # -- the same bits, checked by tests/test_ncf_gpu.py
        self.fused_tail = True
        self._broken = None           # set when a refused tail left the stepper's state unusable
        self._model = _lib.NCFModel(ptr(self.user_w), ptr(self.item_w), ptr(self.m[0]), ptr(self.v[0]),
                                    ptr(self.m[1]), ptr(self.v[1]), ptr(self.mlp), ptr(self.m[2]), ptr(self.v[2]),
                                    self.U, self.I, E, self.M)
        if self.neumf:
            md = self._model
            md.mf_user_w, md.mf_item_w = ptr(self.mf_w[0]), ptr(self.mf_w[1])
            md.mf_user_m, md.mf_item_m = ptr(self.m[3]), ptr(self.m[4])
            md.mf_user_v, md.mf_item_v = ptr(self.v[3]), ptr(self.v[4])
        # the sampler / prepare part of the native stepper (its MF tables are unused here)
        tabs = _lib.MFTables(ptr(self.user_w), ptr(self.item_w), None, None, None, None, None, None,
                             None, None, None, None, None, None, None, None, self.U, self.I, E, 0)
        cfg = _lib.MFStepperConfig()
        cfg.tables[0], cfg.tables[1] = tabs, tabs
        cfg.work = _lib.MFWork(ptr(self.row_count), ptr(self.row_list), ptr(self.hot_grad), ptr(self.hot_bias),
                               ptr(self.partials), None, None, None, None, None, None, ptr(self.part_row), None)
        cfg.mt_state = ptr(self.mt_buf)
        cfg.pairs[0], cfg.pairs[1] = ptr(self.pairs[0]), ptr(self.pairs[1])
        cfg.pool, cfg.pool_len = ptr(self.pool), len(pu)
        cfg.n_neg, cfg.loss = n, LOSS_KINDS[loss]
        cfg.cols, cfg.col_offset, cfg.global_cols, cfg.neg_cols = B, self.rank * B, B * self.world, B * self.world
        cfg.opt = self._opt_base()
        cfg.lr_d, cfg.beta1_d, cfg.beta2_d = float(lr), float(betas[0]), float(betas[1])
        # single GPU: the step's tail launch (rg_ncf_tail) walks the MT words two steps ahead in
        # its first workgroup, as the MF split step's dense pass does (gen_mode 2: no
        # generator-stream kernel beside the pair kernel) when the launch hides the walk (the
        # stepper's test: the E = 64 tower's tables do, NeuMF's E = 16 ones do not); the
        # data-parallel step has no such launch: 8-step slots on the generator stream (one walk
        # and one hop per 8 steps)
        if _lib.ab_build() and os.environ.get("RG_NCF_GEN_INLINE") == "1":
            cfg.gen_mode = 0
        else:
            cfg.gen_mode = 2 if self.world == 1 else 1
            if self.world == 1 and self.neumf:
                # NeuMF: the walk rides in the GMF tables' launch when that pass hides it (the
                # stepper's test, rg_stepper.cpp, against the GMF rows instead of the MLP ones, at
                # the ~4.5 TB/s the odd-width 16-lane rows stream at: 42 us for mf 50 on ML-20M
                # with Adam); the pass streams p plus the optimizer's state arrays, read and
                # written: SGD 2, RMSprop 4, Adam 6 arrays
                walk_us = 0.47e-3 * 2 * n * B
                streams = {"sgd": 2.0, "rms": 4.0, "rmsprop": 4.0, "adam": 6.0}.get(self.opt_kind, 6.0)
                gmf_us = streams * (self.U + self.I) * 4.0 * self.M / 4.5e6
                cfg.gen_mode = 3 if walk_us <= gmf_us else 2
        self._stepper = lib.rg_mf_stepper_create(ctypes.byref(cfg))
        if not self._stepper:
            raise RuntimeError("rg_mf_stepper_create: " + lib.rg_last_error().decode())
        self._cfg = cfg

    def __del__(self):
        st = getattr(self, "_stepper", None)
        if st:
            try:
                self.lib.rg_mf_stepper_destroy(st)
            except Exception:
                pass
            self._stepper = None

    def _opt_base(self):
        o = _lib.Opt()
        o.kind = OPT_KINDS[self.opt_kind]
        o.lr, o.beta1, o.beta2 = self.lr, self.betas[0], self.betas[1]
        o.eps, o.weight_decay, o.alpha = self.eps, self.wd, self.alpha
        o.one_minus_beta1, o.one_minus_beta2, o.one_minus_alpha = 1 - self.betas[0], 1 - self.betas[1], 1 - self.alpha
        return o

    def _opt(self, t):
        o = _lib.Opt()
        check(self.lib.rg_mf_stepper_opt(self._stepper, t, ctypes.byref(o)), "rg_mf_stepper_opt")
        return o

    def make_plan(self, pos_i):
        return build_plan(pos_i, self.batch_size, self.tc, self.I)

    def make_plans(self, items, offset=0, stride=None, n_batches=None):
        """Plans of every batch [offset + k*stride, +batch_size) of ``items`` in one launch
        (``n_batches``: how many, counting empty ones -- a data-parallel rank's slice of the last
        global batch may be empty)."""
        return build_plans(items, self.batch_size, self.tc, self.I, offset=offset, stride=stride,
                           n_batches=n_batches)

    def mlp_params(self):
        """The MLP parameters as tensors of their reference shapes (views of the flat buffer)."""
        out, o = [], 0
        for shp in self.mlp_shapes:
            k = int(np.prod(shp))
            out.append(self.mlp[o:o + k].view(shp))
            o += k
        return out

    def _work(self, masks, training):
        nw = _lib.NCFWork(ptr(self.contrib), ptr(self.mlp_partials), ptr(self.scores_buf), ptr(self.dp_buf),
                          None, None, 0, 1 if training else 0, self.tile_rows)
        if masks is not None:
            mp, mn = masks
            nw.mask_pos, nw.mask_neg = ptr(mp), ptr(mn)
        nw.seed = (self.seed * 0x9E3779B97F4A7C15 + self.t) & 0xFFFFFFFFFFFFFFFF
        if self.neumf:
            nw.mf_contrib, nw.mf_hot_grad, nw.mf_part_row = ptr(self.mf_contrib), ptr(self.mf_hot_grad), \
                ptr(self.mf_part_row)
        return nw

    def _loss(self, global_pos, out):
        n = self.n_neg
        if self.loss == "pointwise":
            ia, ib = 1.0 / global_pos, 1.0 / (n * self.neg_cols)
        elif self.loss in ("bpr", "hinge"):
            ia, ib = 1.0 / (n * global_pos), 0.0
        else:
            ia, ib = 1.0 / global_pos, 0.0
        np_ = 1 if self.loss == "adaptive_hinge" else self.tiles
        return _lib.MFLoss(np_, ia, ib, ptr(out))

    def _exchange(self, t, allreduce):
        if self.comm is not None:
            self.comm.allreduce_(t)
        else:
            allreduce(t)

    def _adapt_dp(self, batch, work, nw, stream, allreduce):
        """dp of the adaptive hinge from this step's scores: one rank as a single kernel; over
        several ranks the global maximum of ONE draw through two small SUM exchanges."""
        if self.world == 1:
            check(self.lib.rg_ncf_adapt_dp(stream, ctypes.byref(batch), ctypes.byref(nw), ptr(self.adapt_partials)),
                  "rg_ncf_adapt_dp")
            return
        ref = ctypes.byref
        check(self.lib.rg_ncf_adapt_local(stream, ref(batch), ref(work), ref(nw), ptr(self.adapt_slots), self.rank,
                                          self.world, ptr(self.adapt_row)), "rg_ncf_adapt_local")
        self._exchange(self.adapt_slots, allreduce)
        check(self.lib.rg_ncf_adapt_global(stream, ref(batch), ref(nw), ptr(self.adapt_slots), self.world,
                                           ptr(self.adapt_count), ptr(self.adapt_partials)), "rg_ncf_adapt_global")
        self._exchange(self.adapt_count, allreduce)
        check(self.lib.rg_ncf_adapt_winner(stream, ref(batch), ref(nw), ptr(self.adapt_slots), self.world, self.rank,
                                           ptr(self.adapt_row), ptr(self.adapt_count)), "rg_ncf_adapt_winner")

    def _forward_backward(self, batch, work, nw, stream, allreduce=None):
        if self.loss == "adaptive_hinge":
            check(self.lib.rg_ncf_pairs(stream, ctypes.byref(self._model), ctypes.byref(batch), ctypes.byref(work),
                                        ctypes.byref(nw), 1), "rg_ncf_pairs(scores)")
            self._adapt_dp(batch, work, nw, stream, allreduce)
            check(self.lib.rg_ncf_pairs(stream, ctypes.byref(self._model), ctypes.byref(batch), ctypes.byref(work),
                                        ctypes.byref(nw), 2), "rg_ncf_pairs(given dp)")
        else:
            check(self.lib.rg_ncf_pairs(stream, ctypes.byref(self._model), ctypes.byref(batch), ctypes.byref(work),
                                        ctypes.byref(nw), 0), "rg_ncf_pairs")

    def _step_in_of(self, pos_u, pos_i, global_pos, plan):
        n_pos = int(pos_u.numel())
        x = _lib.MFStepIn(ptr(pos_u) if n_pos else None, ptr(pos_i) if n_pos else None, n_pos,
                          n_pos * self.world if global_pos is None else int(global_pos), None, None, None)
        if plan is not None:
            x.plan_perm, x.plan_pos_slot, x.plan_item_slot_off = ptr(plan.perm), ptr(plan.pos_slot), \
                ptr(plan.item_slot_off)
        return x

    def train_step(self, pos_u, pos_i, global_pos=None, plan=None, masks=None, loss_out=None, next_step=None,
                   allreduce=None):
        """One step; ``masks`` = (mask_pos [B, units] uint8, mask_neg [n*B, units] uint8) device
        tensors recorded from the reference, or None for the device dropout RNG.  The loss
        goes to ``loss_out`` (float32 device tensor) or the engine's own slot.  ``next_step``
        = (pos_u, pos_i, plan) of the following step: its negatives are prepared on the
        side stream while this step's updates run (rg_mf_stepper_prefetch).  Data parallel:
        (pos_u, pos_i) are this rank's columns of the global batch, ``global_pos`` its size
        (default R * n_pos), ``masks`` (if given) the GLOBAL batch's, and the exchange runs on
        ``comm`` or ``allreduce(flat)``."""
        if self._broken:
            raise RuntimeError("NCFEngine unusable: " + self._broken)
        n_pos = int(pos_u.numel())
        global_pos = n_pos * self.world if global_pos is None else int(global_pos)
        if self.world > 1 and self.comm is None and allreduce is None:
            raise RuntimeError("a data-parallel NCF step needs an RcclComm or an allreduce")
        x = self._step_in_of(pos_u, pos_i, global_pos, plan)
        stream = _lib.stream_handle()
        batch, work = _lib.MFBatch(), _lib.MFWork()
        check(self.lib.rg_mf_stepper_acquire(self._stepper, stream, ctypes.byref(x), ctypes.byref(batch),
                                             ctypes.byref(work)), "rg_mf_stepper_acquire")
        self.t += 1
        nw = self._work(masks, True)
        if self.kernel_events is not None:
            self.kernel_events[0].record()
        self._forward_backward(batch, work, nw, stream, allreduce)
        if self.kernel_events is not None:
            self.kernel_events[1].record()
        check(self.lib.rg_mf_stepper_release(self._stepper, stream), "rg_mf_stepper_release")
        if next_step is not None:
            nu, ni, nplan = next_step
            self._next_in = self._step_in_of(nu, ni, None, nplan)
            if self._prefetch_side:
                check(self.lib.rg_mf_stepper_prefetch(self._stepper, stream, ctypes.byref(self._next_in)),
                      "rg_mf_stepper_prefetch")
        o = self._opt(self.t)
        parts = self.adapt_partials if self.loss == "adaptive_hinge" else self.partials
        out = self.loss_out if loss_out is None else loss_out
        if self.world > 1:
            return self._dp_update(work, nw, o, parts, global_pos, out, stream, allreduce, next_step)
        if self.fused_tail:
            # one launch: the next step's prepare, the MLP update (with the loss) and the
            # embedding update (rg_ncf_tail; the same sums as the three separate calls)
            nb, nwk, need, gen = _lib.MFBatch(), _lib.MFWork(), 0, _lib.MTGen()
            lossd = self._loss(global_pos, out)
            # the tail's own checks first: the two stepper calls below commit the next unit and
            # the MT ring slot, which only a launched tail may consume
            check(self.lib.rg_ncf_tail_validate(ctypes.byref(self._model), ctypes.byref(work), ctypes.byref(nw),
                                                self.blocks, ctypes.byref(o), ptr(parts), ctypes.byref(lossd)),
                  "rg_ncf_tail")
            if next_step is not None and not self._prefetch_side:
                need = self.lib.rg_mf_stepper_prefetch_args(self._stepper, stream, ctypes.byref(self._next_in),
                                                            ctypes.byref(nb), ctypes.byref(nwk))
                if need < 0:
                    check(need, "rg_mf_stepper_prefetch_args")
            walk = self.lib.rg_mf_stepper_tail_gen(self._stepper, stream, ctypes.byref(gen))
            if walk < 0:
                check(walk, "rg_mf_stepper_tail_gen")
            rc = self.lib.rg_ncf_tail(stream, ctypes.byref(self._model), ctypes.byref(work), ctypes.byref(nw),
                                      self.blocks, ctypes.byref(o), ptr(parts), ctypes.byref(lossd),
                                      ctypes.byref(nb) if need else None, ctypes.byref(nwk) if need else None,
                                      ctypes.byref(gen) if walk else None)
            if rc != 0 and (need or walk):
                # refused after the stepper committed a prepare / walk that never launched: later
                # steps would read stale words and pairs, so this engine cannot continue
                self._broken = "rg_ncf_tail refused after the stepper committed the next unit"
            check(rc, "rg_ncf_tail")
        else:
            check(self.lib.rg_ncf_update(stream, ctypes.byref(self._model), ctypes.byref(nw), self.blocks,
                                         ctypes.byref(o), ptr(parts), ctypes.byref(self._loss(global_pos, out))),
                  "rg_ncf_update")
            if self.neumf:
                check(self.lib.rg_neumf_apply(stream, ctypes.byref(self._model), ctypes.byref(work),
                                              ctypes.byref(nw), ctypes.byref(o), 0, -1), "rg_neumf_apply")
            else:
                check(self.lib.rg_ncf_apply(stream, ctypes.byref(self._model), ctypes.byref(work), nw.contrib,
                                            ctypes.byref(o), 0, -1), "rg_ncf_apply")
            self._prefetch_tail(next_step, stream)
        check(self.lib.rg_mf_stepper_advance(self._stepper, 0, 1), "rg_mf_stepper_advance")
        return out

    def _prefetch_tail(self, next_step, stream):
        """The next step's negatives prepared at the end of this step, on the same stream (no
        cross-stream events; RG_NCF_PREFETCH_SIDE=1: on the side stream beside the updates)."""
        if next_step is not None and not self._prefetch_side:
            check(self.lib.rg_mf_stepper_prefetch_inline(self._stepper, stream, ctypes.byref(self._next_in)),
                  "rg_mf_stepper_prefetch_inline")

    def _dp_update(self, work, nw, o, parts, global_pos, out, stream, allreduce, next_step=None):
        """Data-parallel second half: data gradients -> one all-reduce -> the same update on
        every rank."""
        M, ref = self._model, ctypes.byref
        check(self.lib.rg_ncf_mlp_grad(stream, ref(M), ref(nw), self.blocks, ptr(parts),
                                       ref(self._loss(global_pos, out)), ptr(self.dp_mlp)), "rg_ncf_mlp_grad")
        if self.neumf:
            check(self.lib.rg_ncf_grads(stream, ref(M), ref(work), ref(nw), ptr(self.dp_gmf), 0, -1, 1),
                  "rg_ncf_grads(gmf)")
        check(self.lib.rg_ncf_grads(stream, ref(M), ref(work), ref(nw), ptr(self.dp_emb), 0, -1, 0), "rg_ncf_grads")
        if self.comm is not None:
            self.comm.allreduce_(self.dp_flat)
        else:
            allreduce(self.dp_flat)
        check(self.lib.rg_ncf_mlp_apply(stream, ref(M), ptr(self.dp_mlp), ref(o), ptr(out)), "rg_ncf_mlp_apply")
        check(self.lib.rg_ncf_apply_dense(stream, ref(M), ptr(self.dp_emb), ref(o), 0, -1, 0), "rg_ncf_apply_dense")
        if self.neumf:
            check(self.lib.rg_ncf_apply_dense(stream, ref(M), ptr(self.dp_gmf), ref(o), 0, -1, 1),
                  "rg_ncf_apply_dense(gmf)")
        self._prefetch_tail(next_step, stream)
        check(self.lib.rg_mf_stepper_advance(self._stepper, 0, 1), "rg_mf_stepper_advance")
        return out

    def _step_in(self, pos_u, pos_i, global_pos):
        n_pos = int(pos_u.numel())
        return _lib.MFStepIn(ptr(pos_u) if n_pos else None, ptr(pos_i) if n_pos else None, n_pos,
                             n_pos if global_pos is None else int(global_pos), None, None, None)

    def val_loss(self, pos_u, pos_i, global_pos=None, allreduce=None):
        """run_val_iteration (implicit.py:366-379): eval-mode forward (no dropout) and the
        loss on the same negative stream; no update.  Data parallel: this rank's columns,
        loss shares summed by ``comm`` / ``allreduce``."""
        if global_pos is None:
            global_pos = int(pos_u.numel()) * self.world
        x = self._step_in(pos_u, pos_i, global_pos)
        stream = _lib.stream_handle()
        batch, work = _lib.MFBatch(), _lib.MFWork()
        check(self.lib.rg_mf_stepper_acquire(self._stepper, stream, ctypes.byref(x), ctypes.byref(batch),
                                             ctypes.byref(work)), "rg_mf_stepper_acquire")
        nw = self._work(None, False)
        out = torch.empty(1, dtype=torch.float32, device=self.device)
        l = self._loss(x.global_pos, out)
        if self.loss == "adaptive_hinge":
            check(self.lib.rg_ncf_pairs(stream, ctypes.byref(self._model), ctypes.byref(batch), ctypes.byref(work),
                                        ctypes.byref(nw), 1), "rg_ncf_pairs(scores)")
            self._adapt_dp(batch, work, nw, stream, allreduce)
            parts = self.adapt_partials
        else:
            check(self.lib.rg_ncf_pairs(stream, ctypes.byref(self._model), ctypes.byref(batch), ctypes.byref(work),
                                        ctypes.byref(nw), 3), "rg_ncf_pairs(loss)")
            parts = self.partials
        check(self.lib.rg_mf_stepper_release(self._stepper, stream), "rg_mf_stepper_release")
        check(self.lib.rg_loss_finalize(stream, ptr(parts), l.n_partials, l.inv_a, l.inv_b, ptr(out)),
              "rg_loss_finalize")
        if self.world > 1:
            if self.comm is not None:
                self.comm.allreduce_(out)
            else:
                allreduce(out)
        return out

    def params(self):
        """named_parameters() order as device tensors of the reference's shapes: [user table,
        item table, (NeuMF: GMF user table, GMF item table), MLP parameters...]."""
        return [self.user_w, self.item_w] + (self.mf_w if self.neumf else []) + self.mlp_params()

    def set_params(self, tensors):
        for dst, src in zip(self.params(), tensors):
            dst.copy_(torch.as_tensor(src, dtype=torch.float32).reshape(dst.shape))

    def scores(self, users, items):
        """Eval-mode scores (no dropout) for (user, item) pairs, on the device."""
        users = torch.as_tensor(users).to(self.device, torch.int64).reshape(-1)
        items = torch.as_tensor(items).to(self.device, torch.int64).reshape(-1)
        x = torch.cat([self.user_w[users], self.item_w[items]], 1)
        ps = self.mlp_params()
        for k in range(0, len(ps) - 2, 2):
            z = x @ ps[k].T + ps[k + 1]
            x = torch.where(z > 0, z, z * 0.1)
        if self.neumf:
            x = torch.cat([x, self.mf_w[0][users] * self.mf_w[1][items]], 1)
        return torch.sigmoid(x @ ps[-2].T + ps[-1]).reshape(-1)

    def mt_state(self):
        host = np.zeros(625, dtype=np.uint32)
        check(self.lib.rg_mf_stepper_sync_mt(self._stepper, host.ctypes.data_as(ctypes.c_void_p), 0),
              "rg_mf_stepper_sync_mt")
        return host

    def set_mt_state(self, st):
        host = np.ascontiguousarray(np.asarray(st, dtype=np.uint32))
        check(self.lib.rg_mf_stepper_sync_mt(self._stepper, host.ctypes.data_as(ctypes.c_void_p), 1),
              "rg_mf_stepper_sync_mt")
