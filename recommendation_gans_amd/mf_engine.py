"""Device-resident MF training engine: the fused replacement of
``ImplicitFactorizationModel.run_train_iteration`` (implicit.py:347-364).

Everything of the step lives in HBM and is only touched by librg_hip.so:

    tables   user_w (U,d) item_w (I,d) user_b (U,) item_b (I,)   x2 (ping-pong)
    optim    m, v of the same shapes (Adam), v only (RMSprop), none (SGD)
    pool     negative pool as int32 (user, item) pairs, 8 B per entry
    sampler  CPython MT19937 state (624 words + position) and two word buffers
    scratch  per-row contribution counters/lists, overflow accumulators, loss partials

Per step: rg_mf_pairs (forward, loss, dL/dz, contribution lists) then
rg_mf_apply_prepare (pull gradients + optimizer over every row, and the next
step's draws -> pool pairs in the same launch).  The native stepper
(rg_stepper.cpp) generates the MT19937 words in 8-step slots ahead of use on a
stream of its own, so the sequential sampler is off the critical path.
"""
import ctypes
import os
from collections import namedtuple

import numpy as np
import torch

from . import _lib
from ._lib import LOSS_KINDS, OPT_KINDS, RG_MF_LIST_CAP, RG_MF_MAX_NEG, RG_MT_PAD, check, ptr


def _as_u32_tensor(words, device):
    a = np.ascontiguousarray(np.asarray(words, dtype=np.uint32))
    return torch.from_numpy(a.view(np.int32)).to(device)


class DeviceSampler:
    """CPython ``random`` stream on the GPU, bit-exact with ``random.choices``.

    ``acquire(nwords)`` returns an int32 tensor holding the next ``nwords``
    raw MT state words (bit pattern of uint32; tempered by the consumer) whose producer the current stream
    has waited for; ``release()`` must follow the launch of the consumer and
    starts generating the following ``nwords`` words on the side stream.
    """

    def __init__(self, mt_state, device, prefetch=True):
        self.device = torch.device(device)
        self.state = _as_u32_tensor(mt_state, self.device)
        self.state_before = torch.empty(625, dtype=torch.int32, device=self.device)
        self.prefetch = prefetch
        self.side = torch.cuda.Stream(device=self.device)
        self.bufs = [None, None]
        self.ready = [torch.cuda.Event(), torch.cuda.Event()]
        self.consumed = [None, None]
        self.pending = None      # (buffer index, nwords)
        self.cur = None

    def _gen(self, b, nwords):
        if self.bufs[b] is None or self.bufs[b].numel() < nwords:
            with torch.cuda.stream(self.side):
                self.bufs[b] = torch.empty(nwords + RG_MT_PAD, dtype=torch.int32, device=self.device)
        with torch.cuda.stream(self.side):
            if self.consumed[b] is not None:
                self.side.wait_event(self.consumed[b])
            check(_lib.load().rg_mt_generate(_lib.stream_handle(self.side), ptr(self.state), ptr(self.bufs[b]),
                                             nwords, ptr(self.state_before)), "rg_mt_generate")
            self.ready[b].record(self.side)

    def _discard_pending(self):
        if self.pending is None:
            return
        with torch.cuda.stream(self.side):
            self.state.copy_(self.state_before)   # ordered after the prefetch on the side stream
        self.pending = None

    def acquire(self, nwords):
        cur = torch.cuda.current_stream(self.device)
        if self.pending is not None and self.pending[1] == nwords:
            b = self.pending[0]
            self.pending = None
        else:
            self._discard_pending()
            b = 0 if self.cur is None else 1 - self.cur
            self._gen(b, nwords)
        cur.wait_event(self.ready[b])
        self.cur = b
        self._nwords = nwords
        return self.bufs[b]

    def release(self):
        b = self.cur
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.consumed[b] = ev
        if self.prefetch:
            nb = 1 - b
            self._gen(nb, self._nwords)
            self.pending = (nb, self._nwords)

    def export_state(self):
        """625-word state after the last CONSUMED word (prefetched words are not drawn)."""
        self.side.synchronize()
        torch.cuda.current_stream(self.device).synchronize()
        src = self.state_before if self.pending is not None else self.state
        return src.cpu().numpy().view(np.uint32).copy()

    def import_state(self, mt_state):
        self.side.synchronize()
        self.pending = None
        self.state.copy_(_as_u32_tensor(mt_state, self.device))


MFPlan = namedtuple("MFPlan", "perm pos_slot item_slot_off n_planned", defaults=(None,))


def build_plans(items, batch_size, units_per_block, num_items, *, offset=0, stride=None, n_batches=None,
                users=None, world=1, rank=0, cols=None):
    """Per-batch plans (include/rg_hip.h rg_mf_work_t): positives processed in
    item-sorted column order, one partial slot per (item, pair-kernel block), built on
    the device for every batch in ONE launch (rg_mf_plans_build, rg_plan.hip).

    Batch k covers positives [offset + k*stride, offset + k*stride + batch_size) of
    ``items`` (device int64).  ``world`` > 1: only the positives whose user (``users``)
    this ``rank`` owns (u % world == rank) are planned -- the owner-sharded data-parallel
    step.  The reference shuffles the training set once per fit (implicit.py:262), so
    every epoch revisits the same batches: plans are built once per fit.  Returns a list
    of MFPlan (views into three shared tensors; ``n_planned`` = planned positives)."""
    lib = _lib.load()
    dev = items.device
    stride = stride or batch_size
    n = items.numel()
    if n_batches is None:
        n_batches = max(0, -(-(n - offset) // stride))
    cols = cols or batch_size
    if n_batches == 0:
        return []
    perm = torch.empty(n_batches * cols, dtype=torch.int32, device=dev)
    pos_slot = torch.empty(n_batches * cols, dtype=torch.int32, device=dev)
    off = torch.empty(n_batches * (num_items + 1), dtype=torch.int32, device=dev)
    counts = torch.empty(2 * n_batches, dtype=torch.int32, device=dev)
    for t in (items, users):
        if t is not None and (t.dtype != torch.int64 or not t.is_contiguous() or t.device != dev):
            raise ValueError("plan inputs must be contiguous int64 tensors on one device")

    def run(with_scratch):
        sl = int(lib.rg_mf_plans_scratch_len(cols, n_batches)) if with_scratch else 0
        scratch = torch.empty(max(sl, 1), dtype=torch.int64, device=dev) if sl > 0 else None
        check(lib.rg_mf_plans_build(_lib.stream_handle(), ptr(users) if world > 1 else None, ptr(items), n, offset,
                                    stride, batch_size, n_batches, cols, units_per_block, num_items, world, rank,
                                    ptr(perm), ptr(pos_slot), ptr(off), ptr(counts), ptr(scratch)),
              "rg_mf_plans_build")
        return counts.cpu().numpy()[0::2]
    # the owner filter plans ~cols / world positives of a batch: the LDS path, no scratch
    # (~12 B per training positive otherwise); a batch over the LDS capacity reports -1
    planned = run(with_scratch=world <= 1)
    if (planned < 0).any():
        planned = run(with_scratch=True)
    return [MFPlan(perm[k * cols:(k + 1) * cols], pos_slot[k * cols:(k + 1) * cols],
                   off[k * (num_items + 1):(k + 1) * (num_items + 1)], int(planned[k])) for k in range(n_batches)]


def build_plan(pos_i, cols, units_per_block, num_items):
    """The plan of one batch (see build_plans); ``pos_i``: its positives' items."""
    return build_plans(pos_i.contiguous(), max(1, pos_i.numel()), units_per_block, num_items, n_batches=1,
                       cols=cols)[0]


def build_epoch_plans(items, batch_size, units_per_block, num_items, offset=0, stride=None):
    """Plans of every batch of an epoch: batch k covers positives
    [offset + k*stride, offset + k*stride + batch_size) of ``items`` (device int64)."""
    return build_plans(items, batch_size, units_per_block, num_items, offset=offset, stride=stride)


class MFEngine:
    """Owns the device state of one BilinearNet training run on one GPU (one rank) and
    the native step runtime (rg_mf_stepper_*) that enqueues each step."""

    def __init__(self, user_w, item_w, user_b, item_b, pool_u, pool_i, mt_state, *, loss="pointwise",
                 optimizer="adam", lr=1e-3, weight_decay=0.0, betas=(0.5, 0.999), eps=1e-8, alpha=0.99,
                 n_neg=5, batch_size=256, device="cuda", rank=0, world_size=1, prefetch=True,
                 dp=None, comm=None):
        """``dp``: data-parallel layout when world_size > 1 --
        "global_stream" (default, reference-exact): every rank holds every row
            and consumes columns [r*B, (r+1)*B) of ONE global draw of n*B*R indices from
            the full pool, with loss means over the global batch; the rank-major data
            gradient is reduce-scattered, each rank updates its row shard, the tables are
            all-gathered (``comm``: an RcclComm, native in rg_mf_stepper_train; without
            one, ``train_step_exchange`` takes the two collectives as callables).  R ranks
            at batch B compute the reference's step at batch R*B;
        "user_shard" (opt-in, faster, NOT the reference's sampling at R > 1): the tables
            passed are this rank's user shard plus every item (sharding.py); own MT stream,
            own sub-pool and positives, the item gradient is the only exchange (``comm``,
            else ``train_step_sharded``);
        "owner" (default when world_size > 1, reference-exact like "global_stream"): the
            FULL tables are passed and this rank keeps the users u % R == rank (local rows
            u // R) and every item; every rank walks the one global draw over the full pool
            and keeps the pairs whose user it owns; the step exchanges the pairs' scores and
            the item gradient only (rg_mf_owner_*, ``comm`` or ``train_step_owner_exchange``).
            ``batch_size`` is per rank; a step's input is the GLOBAL batch of R*B positives
            with this rank's plan (``make_plans(items, users=...)``)."""
        _lib.require_gpu()
        if loss not in LOSS_KINDS:
            raise ValueError(f"unknown loss {loss!r}")
        if optimizer not in OPT_KINDS:
            raise ValueError(f"unknown optimizer {optimizer!r}")
        if not 1 <= n_neg <= RG_MF_MAX_NEG:
            raise ValueError(f"num_negative_samples must be in [1, {RG_MF_MAX_NEG}] for the fused kernel")
        dp = dp or ("owner" if world_size > 1 or comm is not None else None)
        if dp not in (None, "user_shard", "global_stream", "owner"):
            raise ValueError(f"unknown data-parallel layout {dp!r}")
        if loss == "adaptive_hinge" and dp in ("global_stream", "user_shard"):
            raise NotImplementedError("adaptive_hinge over several ranks runs on the owner-sharded layout (dp='owner')")
        self.U_global = int(user_w.shape[0])
        if dp == "owner":
            user_w = user_w[rank::world_size]
            user_b = torch.as_tensor(user_b).reshape(-1)[rank::world_size]
        self.lib = _lib.load()
        self.device = torch.device(device)
        dev = self.device
        self.U, self.I = int(user_w.shape[0]), int(item_w.shape[0])
        self.dim = int(user_w.shape[1])
        if not 1 <= self.dim <= 256:
            raise ValueError("embedding_dim must be in [1, 256]")
        if self.U + self.I >= 2 ** 31:
            raise ValueError("num_users + num_items must be < 2^31")
        f32 = dict(dtype=torch.float32, device=dev)

        def put(t, shape):
            return torch.as_tensor(t, dtype=torch.float32).reshape(shape).to(dev).contiguous()

        self.rank, self.world = int(rank), int(world_size)
        if dp == "global_stream":
            # row shards of the rank-major exchange; tables allocated with world * shard rows
            self.shard_users = -(-self.U // self.world)
            self.shard_items = -(-self.I // self.world)
            rows = (self.shard_users * self.world, self.shard_items * self.world)
        elif dp == "owner" and comm is not None and self.world > 1 and _lib.ab_build() and \
                os.environ.get("RG_OWNER_ITEM_SHARD", "0") == "1":
            # the owner step's sharded item update (reduce-scatter -> this rank's 1/R of the items'
            # optimizer update -> all-gather): item tables allocated with world * shard rows.  A/B
            # build only: with local-copy exchanges rank 0 of 8 measured 81.0 us against 74.6 for
            # the all-reduce and the full item update
            self.shard_users, self.shard_items = 0, -(-self.I // self.world)
            rows = (self.U, self.shard_items * self.world)
        else:
            self.shard_users = self.shard_items = 0
            rows = (self.U, self.I)

        def padded():
            bufs = [torch.zeros(rows[0], self.dim, **f32), torch.zeros(rows[1], self.dim, **f32),
                    torch.zeros(rows[0], **f32), torch.zeros(rows[1], **f32)]
            return bufs, [bufs[0][:self.U], bufs[1][:self.I], bufs[2][:self.U], bufs[3][:self.I]]

        self._pad, self.tabs = [], []
        for _ in range(2):
            b, v = padded()
            self._pad.append(b)
            self.tabs.append(v)
        for dst, src, shape in zip(self.tabs[0], (user_w, item_w, user_b, item_b),
                                   ((self.U, self.dim), (self.I, self.dim), (self.U,), (self.I,))):
            dst.copy_(put(src, shape))
        self.opt_kind = optimizer
        self.m = padded()[1] if optimizer == "adam" else [None] * 4
        self.v = padded()[1] if optimizer != "sgd" else [None] * 4
        self.lr, self.wd, self.betas, self.eps, self.alpha = lr, weight_decay, betas, eps, alpha
        pu = np.asarray(pool_u, dtype=np.int64)
        pi = np.asarray(pool_i, dtype=np.int64)
        if len(pu) == 0 or len(pu) != len(pi):
            raise ValueError("negative pool must be non-empty with matching user/item arrays")
        if pu.min() < 0 or pu.max() >= (self.U_global if dp == "owner" else self.U) or pi.min() < 0 or \
                pi.max() >= self.I:
            raise ValueError("negative pool contains ids outside the model's tables")
        self.pool = torch.from_numpy(np.stack([pu, pi], 1).astype(np.int32)).to(dev).contiguous()
        self.pool_len = len(pu)
        self.loss = loss
        self.n_neg = int(n_neg)
        self.batch_size = int(batch_size)
        self.dp = dp
        self.comm = comm
        if dp == "global_stream":
            self.col_offset, self.global_cols = self.rank * self.batch_size, self.batch_size * self.world
        elif dp == "owner":
            self.col_offset, self.global_cols = 0, self.batch_size * self.world
        else:
            self.col_offset, self.global_cols = 0, self.batch_size
        self.cols = self.global_cols if dp == "owner" else self.batch_size
        self.neg_cols = self.batch_size * self.world
        self.words_per_step = 2 * self.n_neg * self.global_cols
        self.prefetch = prefetch
        rows = self.U + self.I
        self.row_count = torch.zeros(rows, dtype=torch.int32, device=dev)
        self.row_list = torch.empty(rows * RG_MF_LIST_CAP * 2, dtype=torch.int32, device=dev)
        # overflow accumulators: int64 fixed point (order-independent sums, rg_common.h fix_add)
        self.hot_grad = torch.zeros(rows * self.dim, dtype=torch.int64, device=dev)
        self.hot_bias = torch.zeros(rows, dtype=torch.int64, device=dev)
        if dp == "owner":
            self.n_partials = self.lib.rg_mf_owner_partials_len(self.global_cols, self.n_neg, self.dim,
                                                                self.world) // 2
        else:
            self.n_partials = self.lib.rg_mf_partials_len(self.batch_size, self.dim) // 2
        self.partials = torch.zeros(2 * self.n_partials, **f32)
        self.scores_buf = torch.empty(self.batch_size, **f32) if loss == "adaptive_hinge" else None
        self.max_key = torch.zeros(1, dtype=torch.int64, device=dev) if loss == "adaptive_hinge" else None
        self.active_count = torch.zeros(1, dtype=torch.int32, device=dev) if loss == "adaptive_hinge" else None
        self.loss_out = torch.zeros(1, **f32)
        self.part_row = torch.zeros(self.cols * self.dim, **f32)
        self.part_bias = torch.zeros(self.cols, **f32)
        self.units_per_block = int(self.lib.rg_mf_plan_units_per_block(self.dim))
        self.grad_buf = None
        self.item_grad = None
        if dp in ("user_shard", "owner"):
            n = self.I * (self.dim + 1) + 1
            if self.shard_items and dp == "owner":
                n = self.world * int(self.lib.rg_mf_item_grad_chunk(self.shard_items, self.dim))
            self.item_grad = torch.zeros(n, **f32)
        if dp == "owner":
            rl = int(self.lib.rg_mf_owner_rec_len(self.global_cols, self.n_neg))
            ns = int(self.lib.rg_mf_owner_segments(self.global_cols, self.n_neg))
            self.owner_rec = [torch.zeros(4 * rl, dtype=torch.int32, device=dev) for _ in range(2)]
            self.owner_seg = [torch.zeros(ns, dtype=torch.int32, device=dev) for _ in range(2)]
            # adaptive hinge: 4 extra slots after the exchanged scores (rg_mf_owner_adapt)
            extra = 4 if loss == "adaptive_hinge" else 0
            self.owner_scores = [torch.zeros((1 + self.n_neg) * self.global_cols + extra, **f32) for _ in range(2)]
        self.chunk = 0
        if dp == "global_stream":
            self.chunk = int(self.lib.rg_mf_grad_chunk(self.shard_users, self.shard_items, self.dim))
            self.dp_grad = torch.zeros(self.world * self.chunk, **f32)
        self.mt_buf = _as_u32_tensor(mt_state, dev)
        self.pairs = [torch.zeros(int(self.lib.rg_mf_pairs_len(self.batch_size, self.n_neg)), dtype=torch.int32,
                                  device=dev) for _ in range(2)]
        self._work = _lib.MFWork(ptr(self.row_count), ptr(self.row_list), ptr(self.hot_grad), ptr(self.hot_bias),
                                 ptr(self.partials), ptr(self.scores_buf), ptr(self.max_key),
                                 ptr(self.active_count), None, None, None, ptr(self.part_row),
                                 ptr(self.part_bias))
        self._tables = [self._make_tables(0), self._make_tables(1)]
        cfg = _lib.MFStepperConfig()
        cfg.tables[0], cfg.tables[1] = self._tables[0], self._tables[1]
        cfg.work = self._work
        cfg.mt_state = ptr(self.mt_buf)
        cfg.pairs[0], cfg.pairs[1] = ptr(self.pairs[0]), ptr(self.pairs[1])
        cfg.pool, cfg.pool_len = ptr(self.pool), self.pool_len
        cfg.n_neg, cfg.loss = self.n_neg, LOSS_KINDS[loss]
        cfg.cols, cfg.col_offset, cfg.global_cols = self.cols, self.col_offset, self.global_cols
        cfg.neg_cols = self.neg_cols
        cfg.item_grad = ptr(self.item_grad)
        cfg.comm = comm.handle if comm is not None else None
        cfg.opt = self._opt_base()
        cfg.lr_d, cfg.beta1_d, cfg.beta2_d = float(lr), float(betas[0]), float(betas[1])
        cfg.step, cfg.n_partials, cfg.current_set = 0, self.n_partials, 0
        if dp == "global_stream":
            cfg.dp_mode, cfg.rank, cfg.world = 1, self.rank, self.world
            cfg.shard_users, cfg.shard_items = self.shard_users, self.shard_items
            cfg.grad_buf = ptr(self.dp_grad)
        elif dp == "owner":
            cfg.dp_mode, cfg.rank, cfg.world = 2, self.rank, self.world
            cfg.shard_items = self.shard_items
            for k in range(2):
                cfg.owner_rec[k] = ptr(self.owner_rec[k])
                cfg.owner_seg[k] = ptr(self.owner_seg[k])
                cfg.owner_scores[k] = ptr(self.owner_scores[k])
        self._stepper = self.lib.rg_mf_stepper_create(ctypes.byref(cfg))
        if not self._stepper:
            raise RuntimeError("rg_mf_stepper_create: " + self.lib.rg_last_error().decode())
        self._cfg = cfg   # keep alive

    def __del__(self):
        st = getattr(self, "_stepper", None)
        if st:
            try:
                self.lib.rg_mf_stepper_destroy(st)
            except Exception:
                pass
            self._stepper = None

    # ------------------------------------------------------------------ plumbing
    def _make_tables(self, cur):
        a, b = self.tabs[cur], self.tabs[1 - cur]
        m, v = self.m, self.v
        return _lib.MFTables(ptr(a[0]), ptr(a[1]), ptr(a[2]), ptr(a[3]),
                             ptr(b[0]), ptr(b[1]), ptr(b[2]), ptr(b[3]),
                             ptr(m[0]), ptr(v[0]), ptr(m[1]), ptr(v[1]),
                             ptr(m[2]), ptr(v[2]), ptr(m[3]), ptr(v[3]),
                             self.U, self.I, self.dim, 0)

    def _opt_base(self):
        o = _lib.Opt()
        o.kind = OPT_KINDS[self.opt_kind]
        o.lr, o.beta1, o.beta2 = self.lr, self.betas[0], self.betas[1]
        o.eps, o.weight_decay, o.alpha = self.eps, self.wd, self.alpha
        o.one_minus_beta1 = 1 - self.betas[0]
        o.one_minus_beta2 = 1 - self.betas[1]
        o.one_minus_alpha = 1 - self.alpha
        return o

    def _state(self):
        cs = ctypes.c_int32()
        st = ctypes.c_int64()
        check(self.lib.rg_mf_stepper_state(self._stepper, ctypes.byref(cs), ctypes.byref(st)), "stepper_state")
        return cs.value, st.value

    @property
    def cur(self):
        return self._state()[0]

    @property
    def t(self):
        return self._state()[1]

    def flush(self):
        """Lazy split step: bring every deferred user row up to the current step
        (rg_mf_stepper_flush, on the current stream; a no-op when no row lags)."""
        check(self.lib.rg_mf_stepper_flush(self._stepper, _lib.stream_handle()), "rg_mf_stepper_flush")

    def lazy_rows(self, enable=False):
        """Diagnostics of the lazy pass: user rows processed since the last call (synchronises);
        ``enable`` switches the (contended) device counter on for the following steps.
        Returns None when the stepper runs the eager pass."""
        n = ctypes.c_uint64()
        lazy = self.lib.rg_mf_stepper_lazy_count(self._stepper, int(bool(enable)), ctypes.byref(n))
        return int(n.value) if lazy == 1 else None

    def params(self):
        """Current (user_w, item_w, user_b, item_b) device tensors (deferred rows flushed)."""
        self.flush()
        return self.tabs[self.cur]

    def loss_scales(self, global_pos):
        n, gc = self.n_neg, self.neg_cols
        if self.loss == "pointwise":
            return 1.0 / global_pos, 1.0 / (n * gc)
        if self.loss in ("bpr", "hinge"):
            return 1.0 / (n * global_pos), 0.0
        return 1.0 / global_pos, 0.0

    def make_plan(self, pos_i):
        return build_plan(pos_i, self.batch_size, self.units_per_block, self.I)

    def make_plans(self, items, offset=0, stride=None, users=None):
        """Plans of every batch [offset + k*stride, +batch_size) of ``items`` in one launch;
        owner layout: of every GLOBAL batch [k*R*B, (k+1)*R*B), this rank's positives
        (``users`` required)."""
        if self.dp == "owner":
            if users is None:
                raise ValueError("the owner-sharded layout plans this rank's positives: pass users=")
            return build_plans(items, self.global_cols, self.units_per_block, self.I, offset=offset,
                               stride=stride or self.global_cols, users=users, world=self.world, rank=self.rank,
                               cols=self.global_cols)
        return build_plans(items, self.batch_size, self.units_per_block, self.I, offset=offset, stride=stride)

    def _loss(self, global_pos, out):
        ia, ib = self.loss_scales(global_pos)
        return _lib.MFLoss(self.n_partials, ia, ib, ptr(out))

    def _check_ids(self, pos_u, pos_i):
        for t in (pos_u, pos_i):
            if t.dtype != torch.int64 or t.device != self.device or not t.is_contiguous():
                raise ValueError("positive ids must be contiguous int64 tensors on the engine's device")
        if pos_u.numel() != pos_i.numel() or pos_u.numel() > self.cols:
            raise ValueError("positive id batch larger than batch_size (owner layout: world * batch_size) "
                             "or mismatched")

    def step_input(self, pos_u, pos_i, global_pos=None, plan=None):
        self._check_ids(pos_u, pos_i)
        n_pos = int(pos_u.numel())
        if self.dp == "owner":
            if plan is None or plan.n_planned is None:
                raise ValueError("the owner-sharded step needs this rank's plan of the global batch (make_plans)")
            global_pos = n_pos
        global_pos = n_pos * self.world if global_pos is None else int(global_pos)
        x = _lib.MFStepIn(ptr(pos_u) if n_pos else None, ptr(pos_i) if n_pos else None, n_pos, global_pos,
                          None, None, None, 0)
        if plan is not None:
            x.plan_perm, x.plan_pos_slot, x.plan_item_slot_off = ptr(plan.perm), ptr(plan.pos_slot), \
                ptr(plan.item_slot_off)
            x.n_planned = plan.n_planned or 0
        x._keep = (pos_u, pos_i, plan)
        return x

    # ------------------------------------------------------------------ step
    def train_step(self, pos_u, pos_i, global_pos=None, plan=None, apply_events=None, next_input=None):
        """One training step on this rank's positives; returns the device loss tensor (1,).
        ``plan``: optional MFPlan for this batch (see build_plan).  ``next_input``: the
        following step's ``step_input(...)`` -- its words and pairs are then produced
        ahead on the side stream.  ``apply_events``: optional (start, end) torch.cuda.Event
        pair recorded around the rg_mf_apply launch (kernel timing for the roofline)."""
        cur = self.step_input(pos_u, pos_i, global_pos, plan)
        return self.train_step_in(cur, next_input if self.prefetch else None, apply_events)

    def train_step_in(self, cur, next_input=None, apply_events=None, loss_out=None, next2=None):
        """One native step for a prebuilt ``step_input``; the loss goes to ``loss_out``
        (a float32 device tensor of >= 1 element) or to the engine's own slot.  ``next_input`` /
        ``next2``: the following steps' inputs (the pipelined single-GPU step runs the next
        step's pair pass and the one after's prepare inside this step's launch)."""
        if self.dp == "user_shard" and self.world > 1 and self.comm is None:
            raise RuntimeError("user-sharded step over several ranks needs an RcclComm (or train_step_sharded)")
        if self.dp == "global_stream" and self.comm is None:
            if self.world > 1:
                raise RuntimeError("dp='global_stream' over several ranks needs an RcclComm (or train_step_exchange)")
            return self.train_step_exchange(cur, next_input, lambda buf, chunk: None, lambda bufs, counts: None,
                                            loss_out=loss_out)
        if self.dp == "owner" and self.comm is None:
            if self.world > 1:
                raise RuntimeError("dp='owner' over several ranks needs an RcclComm (or train_step_owner_exchange)")
            return self.train_step_owner_exchange(cur, next_input, lambda buf: None, loss_out=loss_out,
                                                  apply_events=apply_events)
        ev0 = ev1 = None
        if apply_events is not None:
            ev0, ev1 = (ctypes.c_void_p(e.cuda_event) for e in apply_events)
        out = self.loss_out if loss_out is None else loss_out
        if out.dtype != torch.float32 or out.device != self.device:
            raise ValueError("loss_out must be a float32 tensor on the engine's device")
        if next2 is not None and next_input is not None:
            check(self.lib.rg_mf_stepper_train_ahead(self._stepper, _lib.stream_handle(), ctypes.byref(cur),
                                                     ctypes.byref(next_input), ctypes.byref(next2), ptr(out), ev0,
                                                     ev1), "rg_mf_stepper_train_ahead")
            return out
        check(self.lib.rg_mf_stepper_train(self._stepper, _lib.stream_handle(), ctypes.byref(cur),
                                           ctypes.byref(next_input) if next_input is not None else None,
                                           ptr(out), ev0, ev1), "rg_mf_stepper_train")
        return out

    @property
    def pipelined(self):
        """True if the native step is the single-launch pipelined one (rg_mf_pipe_step, A/B build)."""
        return self.lib.rg_mf_stepper_pipelined(self._stepper) == 1

    @property
    def mt_mode(self):
        """0: one MT walk of every word; 1: jump-ahead segments of the global draw; 2: this rank's
        slice of each step's draw, all-gathered (the owner step over a communicator)."""
        return int(self.lib.rg_mf_stepper_mt_mode(self._stepper))

    @property
    def pipeline_kind(self):
        """0: the split step; 1: the single-launch pipelined step (A/B build); 2: the two-launch
        pipelined step (rg_mf_pipe2_hot / rg_mf_pipe2_cold, opt-in: RG_PIPE2=1)."""
        return int(self.lib.rg_mf_stepper_pipelined(self._stepper))

    def pipe_error(self):
        """True if a pipelined launch's pair workgroups ran out of their bounded wait (then its
        results are wrong; synchronises)."""
        e = ctypes.c_int32(0)
        check(self.lib.rg_mf_stepper_pipe_error(self._stepper, ctypes.byref(e)), "rg_mf_stepper_pipe_error")
        return bool(e.value)

    def _acquire(self, cur):
        batch, work = _lib.MFBatch(), _lib.MFWork()
        check(self.lib.rg_mf_stepper_acquire(self._stepper, _lib.stream_handle(), ctypes.byref(cur),
                                             ctypes.byref(batch), ctypes.byref(work)), "rg_mf_stepper_acquire")
        return batch, work

    def _release(self):
        check(self.lib.rg_mf_stepper_release(self._stepper, _lib.stream_handle()), "rg_mf_stepper_release")

    def _flat_grad(self, nrows):
        n = nrows * (self.dim + 1) + 1
        if self.grad_buf is None or self.grad_buf.numel() < n:
            self.grad_buf = torch.zeros(n, dtype=torch.float32, device=self.device)
        return self.grad_buf[:n]

    def pairs_and_lists(self, pos_u, pos_i, global_pos=None, plan=None):
        """rg_mf_pairs with backward on this step's draw; the lists are then consumed by
        ``grads`` / ``apply_rows``."""
        cur = self.step_input(pos_u, pos_i, global_pos, plan)
        batch, work = self._acquire(cur)
        check(self.lib.rg_mf_pairs(_lib.stream_handle(), self._tables[self.cur], ctypes.byref(batch),
                                   ctypes.byref(work), 1), "rg_mf_pairs")
        self._release()
        self._work_step = work
        self._global_pos = cur.global_pos
        return cur

    def grads(self, pos_u, pos_i, global_pos=None, plan=None, row_begin=0, row_end=-1):
        """pairs + gradient pull of rows [row_begin, row_end) into the flat buffer
        [n*d | n | loss]; no update.  Returns the (device) flat buffer."""
        self.pairs_and_lists(pos_u, pos_i, global_pos, plan)
        return self.pull_grads(row_begin, row_end)

    def pull_grads(self, row_begin=0, row_end=-1):
        re = self.U + self.I if row_end < 0 else row_end
        g = self._flat_grad(re - row_begin)
        check(self.lib.rg_mf_grads(_lib.stream_handle(), self._tables[self.cur], ctypes.byref(self._work_step),
                                   ptr(g), row_begin, re, self._loss(self._global_pos, self.loss_out)),
              "rg_mf_grads")
        return g

    def _opt_step(self, t):
        o = _lib.Opt()
        check(self.lib.rg_mf_stepper_opt(self._stepper, t, ctypes.byref(o)), "rg_mf_stepper_opt")
        return o

    def apply_rows(self, row_begin, row_end, loss=True):
        """Pull + optimizer update of rows [row_begin, row_end) from the current lists
        (does not flip the table sets; see ``finish_step``)."""
        o = self._opt_step(self.t + 1)
        check(self.lib.rg_mf_apply(_lib.stream_handle(), self._tables[self.cur], ctypes.byref(self._work_step),
                                   ctypes.byref(o), row_begin, row_end,
                                   self._loss(self._global_pos, self.loss_out) if loss else None), "rg_mf_apply")

    def apply_dense_rows(self, grad, row_begin, row_end):
        o = self._opt_step(self.t + 1)
        check(self.lib.rg_mf_apply_dense(_lib.stream_handle(), self._tables[self.cur], ptr(grad), ctypes.byref(o),
                                         row_begin, row_end, ptr(self.loss_out)), "rg_mf_apply_dense")

    def finish_step(self):
        """After a split step updated every row: flip the ping-pong sets, count the step."""
        check(self.lib.rg_mf_stepper_advance(self._stepper, 1, 1), "rg_mf_stepper_advance")

    def apply_dense(self, grad):
        """Optimizer update of every row from a (summed) flat gradient buffer."""
        self.apply_dense_rows(grad, 0, self.U + self.I)
        self.finish_step()
        return self.loss_out

    # ------------------------------------------------------------------ replicated DP (global_stream)
    def dp_begin(self, cur, next_input=None, loss_out=None):
        """First half of the replicated step (rg_mf_stepper_dp_begin): this rank's column
        slice of the global draw -> pairs -> the rank-major gradient in ``dp_grad``."""
        out = self.loss_out if loss_out is None else loss_out
        check(self.lib.rg_mf_stepper_dp_begin(self._stepper, _lib.stream_handle(), ctypes.byref(cur),
                                              ctypes.byref(next_input) if next_input is not None else None,
                                              ptr(out)), "rg_mf_stepper_dp_begin")
        return out

    def dp_end(self, loss_out=None):
        """Second half: this rank's rows from its (reduce-scattered) chunk, then the sets
        flip; the caller all-gathers ``dp_gather_buffers()``."""
        out = self.loss_out if loss_out is None else loss_out
        check(self.lib.rg_mf_stepper_dp_end(self._stepper, _lib.stream_handle(), ptr(out)), "rg_mf_stepper_dp_end")
        return out

    def dp_gather_buffers(self):
        """The current set's four padded tables and this layout's all-gather counts (each
        rank's shard = rows [rank * count, (rank + 1) * count) of the flat buffer)."""
        d = self.dim
        return self._pad[self.cur], [self.shard_users * d, self.shard_items * d, self.shard_users, self.shard_items]

    def train_step_exchange(self, cur, next_input, reduce_scatter, all_gather, loss_out=None):
        """The replicated step with caller-run collectives: ``reduce_scatter(buf, chunk)``
        must leave in buf[rank*chunk:(rank+1)*chunk] the sum over ranks of that chunk;
        ``all_gather(bufs, counts)`` must fill every rank's shard of each buffer."""
        out = self.dp_begin(cur, next_input, loss_out)
        reduce_scatter(self.dp_grad, self.chunk)
        self.dp_end(out)
        all_gather(*self.dp_gather_buffers())
        return out

    # ------------------------------------------------------------------ owner-sharded DP
    def train_step_owner_exchange(self, cur, next_input, allreduce, loss_out=None, apply_events=None):
        """The owner-sharded step with caller-run exchanges: ``allreduce(buf)`` must sum
        ``buf`` over the ranks in place (the score vector, then the item gradient) -- what
        rg_mf_stepper_train does natively over RCCL."""
        out = self.loss_out if loss_out is None else loss_out
        st = _lib.stream_handle()
        check(self.lib.rg_mf_stepper_owner_begin(self._stepper, st, ctypes.byref(cur)), "rg_mf_stepper_owner_begin")
        if self.loss != "pointwise":
            allreduce(self.current_scores())
        check(self.lib.rg_mf_stepper_owner_mid(self._stepper, st, ptr(out)), "rg_mf_stepper_owner_mid")
        allreduce(self.item_grad)
        ev0 = ev1 = None
        if apply_events is not None:
            ev0, ev1 = (ctypes.c_void_p(e.cuda_event) for e in apply_events)
        check(self.lib.rg_mf_stepper_owner_end(self._stepper, st, ctypes.byref(next_input)
                                               if next_input is not None else None, ptr(out), ev0, ev1),
              "rg_mf_stepper_owner_end")
        return out

    def current_scores(self):
        """The score vector of the owner step in flight ((1 + n) * R * B floats)."""
        p = ctypes.c_void_p()
        n = ctypes.c_int64()
        check(self.lib.rg_mf_stepper_owner_scores(self._stepper, ctypes.byref(p), ctypes.byref(n)),
              "rg_mf_stepper_owner_scores")
        for t in self.owner_scores:
            if t.data_ptr() == p.value:
                return t[:n.value]
        raise RuntimeError("owner score buffer not found")

    def train_step_sharded(self, pos_u, pos_i, global_pos, allreduce, plan=None):
        """The user-sharded step with the item-gradient exchange done by ``allreduce``
        (in-place sum, e.g. torch.distributed over gloo in tests): what
        rg_mf_stepper_train does natively with an RCCL communicator."""
        if self.dp != "user_shard":
            raise RuntimeError("train_step_sharded needs dp='user_shard'")
        self.pairs_and_lists(pos_u, pos_i, global_pos, plan)
        g = self.pull_grads(self.U, self.U + self.I)
        allreduce(g)
        self.apply_rows(0, self.U, loss=False)
        self.apply_dense_rows(g, self.U, self.U + self.I)
        self.finish_step()
        return self.loss_out

    def val_loss(self, pos_u, pos_i, global_pos=None, plan=None, allreduce=None):
        """run_val_iteration (implicit.py:366): forward + loss on the same draw stream, no update.
        Owner layout: (pos_u, pos_i) is the GLOBAL validation batch and ``plan`` this rank's
        plan of it; the scores are exchanged by the communicator or ``allreduce``."""
        if self.dp == "owner":
            cur = self.step_input(pos_u, pos_i, None, plan)
            out = torch.empty(1, dtype=torch.float32, device=self.device)
            st = _lib.stream_handle()
            if self.comm is not None:
                check(self.lib.rg_mf_stepper_owner_val(self._stepper, st, ctypes.byref(cur), ptr(out)),
                      "rg_mf_stepper_owner_val")
            else:
                if allreduce is None and self.world > 1:
                    raise RuntimeError("owner-layout validation over several ranks needs a communicator or allreduce")
                check(self.lib.rg_mf_stepper_owner_begin(self._stepper, st, ctypes.byref(cur)),
                      "rg_mf_stepper_owner_begin")
                if allreduce is not None:
                    allreduce(self.current_scores())
                check(self.lib.rg_mf_stepper_owner_val_end(self._stepper, st, ptr(out)), "rg_mf_stepper_owner_val_end")
            return out
        cur = self.step_input(pos_u, pos_i, global_pos, None)
        batch, work = self._acquire(cur)
        stream = _lib.stream_handle()
        check(self.lib.rg_mf_pairs(stream, self._tables[self.cur], ctypes.byref(batch), ctypes.byref(work), 0),
              "rg_mf_pairs")
        self._release()
        ia, ib = self.loss_scales(cur.global_pos)
        out = torch.empty(1, dtype=torch.float32, device=self.device)
        check(self.lib.rg_loss_finalize(stream, ptr(self.partials), self.n_partials, ia, ib, ptr(out)),
              "rg_loss_finalize")
        return out

    def scores(self, users, items):
        """BilinearNet.forward (representations.py:62-91) for eval/predict."""
        users = users.to(self.device, torch.int64).contiguous()
        items = items.to(self.device, torch.int64).contiguous()
        out = torch.empty(users.numel(), dtype=torch.float32, device=self.device)
        U, I, ub, ib = self.params()      # flushes deferred rows
        check(self.lib.rg_mf_scores(_lib.stream_handle(), ptr(U), ptr(I), ptr(ub), ptr(ib), self.dim,
                                    ptr(users), ptr(items), users.numel(), ptr(out)), "rg_mf_scores")
        return out

    def set_params(self, user_w, item_w, user_b, item_b):
        """Overwrite the current tables (teacher forcing in tests, checkpoint load)."""
        for dst, src in zip(self.params(), (user_w, item_w, user_b, item_b)):
            dst.copy_(torch.as_tensor(src, dtype=torch.float32).reshape(dst.shape))

    def mt_state(self):
        """CPython random state (624 words + position) after the last consumed draw."""
        host = np.zeros(625, dtype=np.uint32)
        check(self.lib.rg_mf_stepper_sync_mt(self._stepper, host.ctypes.data_as(ctypes.c_void_p), 0),
              "rg_mf_stepper_sync_mt")
        return host

    def set_mt_state(self, st):
        host = np.ascontiguousarray(np.asarray(st, dtype=np.uint32))
        check(self.lib.rg_mf_stepper_sync_mt(self._stepper, host.ctypes.data_as(ctypes.c_void_p), 1),
              "rg_mf_stepper_sync_mt")

    def optimizer_state(self):
        if self.dp == "owner" and self.shard_items:
            # each rank updates (and holds current moments for) only its shard of the item rows;
            # the other rows' m / v are stale, so a checkpoint from them would be wrong
            raise NotImplementedError("optimizer_state: the sharded item update (RG_OWNER_ITEM_SHARD, A/B build) "
                                      "keeps each rank's item moments only for its own shard")
        self.flush()
        return {"step": self.t, "m": self.m, "v": self.v}
