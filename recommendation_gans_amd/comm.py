"""RCCL communicator of the librg_hip.so data-parallel step (include/rg_hip.h,
rg_comm_*).  torch.distributed sets up the process group (one process per GPU,
RANK / WORLD_SIZE / MASTER_ADDR from torchrun) and carries the 128-byte unique
id.  The per-step collectives then run inside rg_mf_stepper_train: the reduce-scatter
of the rank-major gradient and the all-gather of the tables (replicated, reference-exact
step), or the item-gradient all-reduce on the communicator's own stream overlapped with
the user-shard update (user-sharded opt-in)."""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import RG_COMM_ID_BYTES, check, ptr


class RcclComm:
    def __init__(self, device, group=None):
        import torch.distributed as dist
        self.lib = _lib.load()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        uid = np.zeros(RG_COMM_ID_BYTES, dtype=np.uint8)
        if self.rank == 0:
            check(self.lib.rg_comm_unique_id(uid.ctypes.data_as(ctypes.c_void_p), RG_COMM_ID_BYTES),
                  "rg_comm_unique_id")
        box = [uid.tobytes()]
        dist.broadcast_object_list(box, src=0, group=group)
        uid = np.frombuffer(box[0], dtype=np.uint8).copy()
        index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.handle = self.lib.rg_comm_create(uid.ctypes.data_as(ctypes.c_void_p), self.world, self.rank, index)
        if not self.handle:
            raise RuntimeError("rg_comm_create: " + self.lib.rg_last_error().decode())

    def allreduce_(self, t):
        """In-place fp32 sum over ranks, ordered on the current stream."""
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
            raise ValueError("allreduce_ takes a contiguous fp32 tensor on the communicator's device")
        check(self.lib.rg_comm_allreduce_sum_f32(self.handle, _lib.stream_handle(), ptr(t), t.numel()),
              "rg_comm_allreduce_sum_f32")
        return t

    def reduce_scatter_(self, t, chunk):
        """In-place sum: rank r's chunk t[r*chunk:(r+1)*chunk] becomes the sum over ranks."""
        check(self.lib.rg_comm_reduce_scatter_f32(self.handle, _lib.stream_handle(), ptr(t), int(chunk)),
              "rg_comm_reduce_scatter_f32")
        return t

    def all_gather_(self, bufs, counts):
        """In-place all-gather of each buffer's rank shards (one RCCL group)."""
        arr = (ctypes.c_void_p * len(bufs))(*[ptr(b) for b in bufs])
        cnt = (ctypes.c_int64 * len(counts))(*[int(c) for c in counts])
        check(self.lib.rg_comm_allgather_f32(self.handle, _lib.stream_handle(), len(bufs), arr, cnt),
              "rg_comm_allgather_f32")

    def info(self):
        """(count, user_rank, is_rccl) as the native communicator reports them: ncclCommCount /
        ncclCommUserRank for RCCL, the configured world / rank for a stand-in."""
        n, r, k = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(self.lib.rg_comm_info(self.handle, ctypes.byref(n), ctypes.byref(r), ctypes.byref(k)), "rg_comm_info")
        return int(n.value), int(r.value), bool(k.value)

    def close(self):
        if getattr(self, "handle", None):
            self.lib.rg_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LocalComm(RcclComm):
    """One-GPU stand-in for rank ``rank`` of ``world`` (bench.py --emulate-rank): the native
    step's collectives become same-size local copies on the communicator stream
    (rg_comm_create_local), so one rank's step at the multi-rank geometry can be timed and
    profiled on a single GPU.  The data is left unchanged (an identity exchange)."""

    def __init__(self, device, world, rank):
        self.lib = _lib.load()
        self.rank, self.world = int(rank), int(world)
        self.device = torch.device(device)
        index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.handle = self.lib.rg_comm_create_local(self.world, self.rank, index)
        if not self.handle:
            raise RuntimeError("rg_comm_create_local: " + self.lib.rg_last_error().decode())


class HostComm(RcclComm):
    """Test stand-in for rank ``rank`` of a torch.distributed (gloo) group whose ranks share one
    GPU (RCCL refuses that): the native step's all-reduces run on the communicator stream as
    D2H -> a stream-ordered host callback summing over the group with torch.distributed -> H2D
    (rg_comm_create_host), so the step's own placement -- the score exchange fenced on the main
    stream, the item gradient's exchange on the side stream beside the user update -- runs as in
    production.  A reduce-scatter is staged as an all-reduce of every chunk (each rank then reads
    its own), an all-gather as an all-reduce with every other rank's chunk zeroed first; the owner
    step's MT word all-gather goes through a gather callback on a gloo group of its own.

    The callback takes the GIL on the runtime's callback thread: while the step's work is in
    flight, wait with ``sync()`` (a ctypes call, which releases the GIL), not with a torch call
    that may hold it."""

    def __init__(self, device, group=None, max_floats=1 << 26):
        import torch.distributed as dist
        self.lib = _lib.load()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        self.group = group

        def _allreduce(ctx, buf, n):
            try:
                arr = np.ctypeslib.as_array((ctypes.c_float * n).from_address(buf))
                dist.all_reduce(torch.from_numpy(arr), group=self.group)
                return 0
            except Exception:      # reported by the next collective call (rg_comm host_error)
                return 1
        self._cb = _lib.HOST_ALLREDUCE_FN(_allreduce)
        index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.handle = self.lib.rg_comm_create_host(self.world, self.rank, index, int(max_floats),
                                                   ctypes.cast(self._cb, ctypes.c_void_p), None)
        if not self.handle:
            raise RuntimeError("rg_comm_create_host: " + self.lib.rg_last_error().decode())
        # the owner step's MT word all-gather (rank slices of the global draw's words, bit for bit):
        # a gloo group of its own, called synchronously from the stepper's host thread, so it
        # never interleaves with the step's all-reduces on the callback thread
        ranks = list(range(self.world))
        self.words_group = dist.new_group(ranks, backend="gloo")

        def _gather(ctx, send, n, recv):
            try:
                src = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_int32 * n).from_address(send)))
                dst = np.ctypeslib.as_array((ctypes.c_int32 * (n * self.world)).from_address(recv))
                outs = [torch.from_numpy(dst[r * n:(r + 1) * n]) for r in range(self.world)]
                dist.all_gather(outs, src, group=self.words_group)
                return 0
            except Exception:
                return 1
        self._gcb = _lib.HOST_GATHER_FN(_gather)
        check(self.lib.rg_comm_set_host_gather(self.handle, ctypes.cast(self._gcb, ctypes.c_void_p), None),
              "rg_comm_set_host_gather")
        self._hip = ctypes.CDLL("libamdhip64.so.7")

    def sync(self):
        """hipDeviceSynchronize through ctypes (the GIL is released while it waits)."""
        rc = self._hip.hipDeviceSynchronize()
        if rc != 0:
            raise RuntimeError(f"hipDeviceSynchronize failed: {rc}")

