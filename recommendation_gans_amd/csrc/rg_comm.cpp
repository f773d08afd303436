// RCCL communicator for the data-parallel MF steps (host code): the item-gradient
// all-reduce of the user-sharded step, the reduce-scatter / all-gather of the replicated one.
//
// One process per GPU.  The unique id is created by rank 0 (rg_comm_unique_id)
// and broadcast by the caller (torch.distributed), then every rank builds its
// communicator (rg_comm_create).  The collective runs on the communicator's own
// stream, fenced by events against the caller's compute stream, so compute
// enqueued between rg_comm_allreduce_begin and rg_comm_allreduce_end overlaps it.
//
// rg_comm_create_local: a one-GPU stand-in for rank `rank` of a `world`-rank
// communicator (bench.py --emulate-rank): every collective becomes same-size local
// copies on the communicator stream (an all-reduce: buf -> scratch -> buf, so the data
// is left as it was), with the same events and stream placement as the RCCL path.  It
// measures one rank's compute at the multi-rank geometry on a box with one GPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "rg_common.h"

namespace rg {

struct Comm {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    int world = 0, rank = 0;
    bool local = false;           // rg_comm_create_local: collectives are local copies
    float *scratch = nullptr;     // local: copy target
    size_t scratch_floats = 0;
    // rg_comm_create_host: the all-reduce staged through pinned host memory and done by a
    // host callback in stream order on the communicator stream (tests: gloo across two
    // processes sharing one GPU, where RCCL refuses a second rank on the device)
    rg_host_allreduce_fn host_fn = nullptr;
    void *host_ctx = nullptr;
    float *pinned = nullptr;
    int64_t pinned_floats = 0;
    struct HostCall {
        Comm *c;
        int64_t n;
    };
    std::atomic<int> host_error{0};
    // the owner step's MT word all-gather (comm_words_allgather): its own RCCL communicator (split
    // from `comm`), or the host gather callback; the local stand-in's hash seed counter
    ncclComm_t comm_words = nullptr;
    rg_host_gather_fn gather_fn = nullptr;
    void *gather_ctx = nullptr;
    std::vector<uint32_t> gsend, grecv;
    uint32_t words_calls = 0;
    // RCCL deadline (bounded failure of a multi-process run): a watchdog thread checks the
    // communicator's asynchronous error and the completion of the last tracked collective; past
    // the deadline it aborts the communicator (which releases the GPU's waiting kernels) and
    // exits the process non-zero with a message naming the rank
    std::thread watchdog;
    std::atomic<bool> stop{false};
    std::mutex mu;
    // completion tracking of every collective (RCCL ones on either communicator): a FIFO of
    // (event recorded after the collective, enqueue time, collective number) in a ring of kTrack
    // events.  Completed entries are popped from the head (by the watchdog and at every enqueue);
    // the deadline applies to the head's age -- the oldest collective not yet complete -- so a
    // stalled collective reaches it even when the host then blocks on a sync and enqueues
    // nothing more, and a healthy run whose host stays ahead of the GPU never does (each entry
    // completes in turn).  A full ring folds newer collectives into its newest entry (re-recorded,
    // keeping its older time): the host is then kTrack collectives ahead, so the head is old.
    static constexpr int kTrack = 64;
    hipEvent_t ev_ring[kTrack] = {};
    std::chrono::steady_clock::time_point t0_ring[kTrack];
    int64_t id_ring[kTrack] = {};
    int track_head = 0, track_size = 0;
    int64_t ncoll = 0;
    double timeout_s = 600.0;
};

// each in-flight host exchange owns its call record (freed by the callback): any number of
// exchanges may be enqueued before the callbacks drain
static void host_trampoline(void *p) {
    Comm::HostCall *hc = static_cast<Comm::HostCall *>(p);
    if (hc->c->host_fn(hc->c->host_ctx, hc->c->pinned, hc->n) != 0) hc->c->host_error = 1;
    delete hc;
}

static double env_seconds(const char *name, double dflt) {
    const char *e = getenv(name);
    const double v = e ? atof(e) : 0.0;
    return v > 0.0 ? v : dflt;
}

[[noreturn]] static void comm_die(Comm *c, const std::string &why) {
    fprintf(stderr, "[librg_hip] rank %d of %d: %s; aborting the RCCL communicator and exiting\n", c->rank, c->world,
            why.c_str());
    fflush(stderr);
    if (c->comm_words) ncclCommAbort(c->comm_words);
    if (c->comm) ncclCommAbort(c->comm);
    std::_Exit(3);
}

// pop the completed collectives off the head of the tracking FIFO (c->mu held)
static void track_pop_done(Comm *c) {
    while (c->track_size > 0 && hipEventQuery(c->ev_ring[c->track_head]) == hipSuccess) {
        c->track_head = (c->track_head + 1) % Comm::kTrack;
        --c->track_size;
    }
}

static void watchdog_loop(Comm *c) {
    while (!c->stop.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(500));
        if (c->stop.load()) break;
        ncclResult_t ae = ncclSuccess;
        if (c->comm && ncclCommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
            comm_die(c, std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae));
        if (c->comm_words && ncclCommGetAsyncError(c->comm_words, &ae) == ncclSuccess && ae != ncclSuccess &&
            ae != ncclInProgress)
            comm_die(c, std::string("RCCL asynchronous error (word all-gather): ") + ncclGetErrorString(ae));
        std::lock_guard<std::mutex> g(c->mu);
        track_pop_done(c);
        if (c->track_size == 0) continue;
        const double waited =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - c->t0_ring[c->track_head]).count();
        if (waited > c->timeout_s)
            comm_die(c, "collective #" + std::to_string(c->id_ring[c->track_head]) + " (of " +
                            std::to_string(c->ncoll) + " enqueued) not complete after " + std::to_string((int)waited) +
                            " s (RG_COMM_TIMEOUT_S; a peer rank failed or diverged)");
    }
}

// arm the watchdog on the completion of the collective just enqueued on `stream`
static void track(Comm *c, hipStream_t stream) {
    std::lock_guard<std::mutex> g(c->mu);
    ++c->ncoll;
    if (!c->ev_ring[0]) return;            // stand-ins: no watchdog
    track_pop_done(c);
    if (c->track_size == Comm::kTrack) {   // full: fold into the newest entry (keeps its time)
        (void)hipEventRecord(c->ev_ring[(c->track_head + c->track_size - 1) % Comm::kTrack], stream);
        return;
    }
    const int k = (c->track_head + c->track_size) % Comm::kTrack;
    if (hipEventRecord(c->ev_ring[k], stream) != hipSuccess) return;
    c->t0_ring[k] = std::chrono::steady_clock::now();
    c->id_ring[k] = c->ncoll;
    ++c->track_size;
}

// after an RCCL call on `stream`: wait out ncclInProgress (non-blocking communicator) within
// the deadline, and arm the watchdog on the collective's completion (every collective)
static int nccl_after(Comm *c, hipStream_t stream, ncclResult_t r, const char *what) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
        if (ncclCommGetAsyncError(c->comm, &r) != ncclSuccess) break;
        if (r != ncclInProgress) break;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s)
            comm_die(c, std::string(what) + " still in progress after the deadline");
        std::this_thread::yield();
    }
    if (r != ncclSuccess) {
        set_error(std::string(what) + ": " + ncclGetErrorString(r));
        return RG_E_LAUNCH;
    }
    track(c, stream);
    return RG_OK;
}

// host-staged all-reduce: D2H -> host callback -> H2D, all on `stream`
static int host_allreduce(Comm *c, hipStream_t stream, float *buf, int64_t n) {
    if (n > c->pinned_floats) return fail_arg("rg_comm (host): buffer larger than the staging area");
    if (c->host_error) return fail_arg("rg_comm (host): an earlier host all-reduce failed");
    Comm::HostCall *hc = new (std::nothrow) Comm::HostCall{c, n};
    if (!hc) return fail_arg("rg_comm (host): out of memory");
    hipError_t e = hipMemcpyAsync(c->pinned, buf, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipLaunchHostFunc(stream, host_trampoline, hc);
    else delete hc;
    if (e == hipSuccess) e = hipMemcpyAsync(buf, c->pinned, (size_t)n * sizeof(float), hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) {
        set_error(std::string("rg_comm (host): ") + hipGetErrorString(e));
        return RG_E_LAUNCH;
    }
    return RG_OK;
}

// local stand-in: n floats out to the scratch buffer and back, on `stream`
static int local_roundtrip(Comm *c, hipStream_t stream, float *buf, int64_t n) {
    if (n <= 0) return RG_OK;
    if ((size_t)n > c->scratch_floats) {
        hipError_t e = hipStreamSynchronize(stream);
        if (e == hipSuccess && c->scratch) e = hipFree(c->scratch);
        c->scratch = nullptr;
        c->scratch_floats = 0;
        if (e == hipSuccess) e = hipMalloc(&c->scratch, (size_t)n * sizeof(float));
        if (e != hipSuccess) {
            set_error(std::string("rg_comm (local): scratch: ") + hipGetErrorString(e));
            return RG_E_LAUNCH;
        }
        c->scratch_floats = (size_t)n;
    }
    hipError_t e = hipMemcpyAsync(c->scratch, buf, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, stream);
    if (e == hipSuccess) e = hipMemcpyAsync(buf, c->scratch, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) {
        set_error(std::string("rg_comm (local): copy: ") + hipGetErrorString(e));
        return RG_E_LAUNCH;
    }
    return RG_OK;
}

static int nccl_fail(const char *what, ncclResult_t r) {
    set_error(std::string(what) + ": " + ncclGetErrorString(r));
    return RG_E_LAUNCH;
}

static int hip_fail(const char *what, hipError_t e) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return RG_E_LAUNCH;
}

int comm_begin(void *h, hipStream_t stream, float *buf, int64_t n) {
    Comm *c = static_cast<Comm *>(h);
    if (!c || !buf || n < 0) return fail_arg("rg_comm_allreduce_begin: bad argument");
    hipError_t e = hipEventRecord(c->ev_in, stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_in, 0);
    if (e != hipSuccess) return hip_fail("rg_comm_allreduce_begin", e);
    if (c->local) return local_roundtrip(c, c->stream, buf, n);
    if (c->host_fn) return host_allreduce(c, c->stream, buf, n);
    return nccl_after(c, c->stream, ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, c->comm, c->stream),
                      "ncclAllReduce");
}

hipStream_t comm_stream(void *h) { return h ? static_cast<Comm *>(h)->stream : nullptr; }

int comm_allreduce_on(void *h, hipStream_t stream, float *buf, int64_t n) {
    Comm *c = static_cast<Comm *>(h);
    if (!c || !buf || n < 0) return fail_arg("rg_comm allreduce: bad argument");
    // staged through the host on the caller's stream, where RCCL would run it (the stepper's
    // placement: the owner step's exchanges on the compute stream beside the user update)
    if (c->host_fn) return host_allreduce(c, stream, buf, n);
    if (c->local) return local_roundtrip(c, stream, buf, n);
    if (c->world == 1) return RG_OK;       // a one-rank sum is the buffer itself: no RCCL launch
    return nccl_after(c, stream, ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, c->comm, stream),
                      "ncclAllReduce");
}

int comm_end(void *h, hipStream_t stream) {
    Comm *c = static_cast<Comm *>(h);
    if (!c) return fail_arg("rg_comm_allreduce_end: null communicator");
    hipError_t e = hipEventRecord(c->ev_out, c->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, c->ev_out, 0);
    if (e != hipSuccess) return hip_fail("rg_comm_allreduce_end", e);
    return RG_OK;
}

int comm_reduce_scatter(void *h, hipStream_t stream, float *buf, int64_t chunk) {
    Comm *c = static_cast<Comm *>(h);
    if (!c || !buf || chunk < 0) return fail_arg("rg_comm_reduce_scatter_f32: bad argument");
    if (c->local) return local_roundtrip(c, stream, buf, chunk * c->world);   // the exchange's bytes
    // host-staged: an all-reduce of every chunk (this rank then reads its own, summed)
    if (c->host_fn) return host_allreduce(c, stream, buf, chunk * c->world);
    return nccl_after(c, stream, ncclReduceScatter(buf, buf + (int64_t)c->rank * chunk, (size_t)chunk, ncclFloat32,
                                                   ncclSum, c->comm, stream), "ncclReduceScatter");
}

int comm_allgather(void *h, hipStream_t stream, int n, float *const *bufs, const int64_t *counts) {
    Comm *c = static_cast<Comm *>(h);
    if (!c || n < 0 || (n > 0 && (!bufs || !counts))) return fail_arg("rg_comm_allgather_f32: bad argument");
    if (c->host_fn) {
        // host-staged: every other rank's chunk zeroed, then an all-reduce (the sum is the gather)
        for (int k = 0; k < n; ++k) {
            const int64_t cnt = counts[k], r = c->rank;
            hipError_t e = hipSuccess;
            if (r > 0) e = hipMemsetAsync(bufs[k], 0, (size_t)(r * cnt) * sizeof(float), stream);
            if (e == hipSuccess && r + 1 < c->world)
                e = hipMemsetAsync(bufs[k] + (r + 1) * cnt, 0, (size_t)((c->world - r - 1) * cnt) * sizeof(float), stream);
            if (e != hipSuccess) return hip_fail("rg_comm (host): all-gather", e);
            const int rc = host_allreduce(c, stream, bufs[k], cnt * c->world);
            if (rc) return rc;
        }
        return RG_OK;
    }
    if (c->local) {
        for (int k = 0; k < n; ++k) {
            const int rc = local_roundtrip(c, stream, bufs[k], counts[k] * c->world);
            if (rc) return rc;
        }
        return RG_OK;
    }
    ncclResult_t r = ncclGroupStart();
    for (int k = 0; k < n && r == ncclSuccess; ++k)
        r = ncclAllGather(bufs[k] + (int64_t)c->rank * counts[k], bufs[k], (size_t)counts[k], ncclFloat32, c->comm,
                          stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess && r != ncclInProgress) return nccl_fail("ncclAllGather", r);
    return nccl_after(c, stream, r2, "ncclAllGather (group)");
}

int comm_kind(void *h) {
    const Comm *c = static_cast<const Comm *>(h);
    return !c ? -1 : c->local ? 2 : c->host_fn ? 1 : 0;
}

// wait out ncclInProgress of a call on communicator `cm` within the deadline
static ncclResult_t nccl_settle(Comm *c, ncclComm_t cm, ncclResult_t r, const char *what) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
        if (ncclCommGetAsyncError(cm, &r) != ncclSuccess) break;
        if (r != ncclInProgress) break;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s)
            comm_die(c, std::string(what) + " still in progress after the deadline");
        std::this_thread::yield();
    }
    return r;
}

int comm_words_prepare(void *h) {
    Comm *c = static_cast<Comm *>(h);
    if (!c) return fail_arg("comm_words_prepare: null communicator");
    if (c->local || c->host_fn || c->comm_words) return RG_OK;
    // every rank splits at stepper creation (the same point of each rank's call sequence)
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommSplit(c->comm, 0, c->rank, &c->comm_words, &cfg);
    if (r == ncclInProgress && c->comm_words) r = nccl_settle(c, c->comm_words, r, "ncclCommSplit");
    if (r != ncclSuccess) {
        c->comm_words = nullptr;
        return nccl_fail("ncclCommSplit (word all-gather communicator)", r);
    }
    return RG_OK;
}

int comm_words_allgather(void *h, hipStream_t stream, uint32_t *words, int64_t units, int64_t W, int64_t L) {
    Comm *c = static_cast<Comm *>(h);
    if (!c || !words || units < 0 || L <= 0 || W != L * c->world) return fail_arg("comm_words_allgather: bad argument");
    if (c->local) return mt_fill_other_slices(stream, words, units, W, L, c->rank, c->world, 0x5bd1e995u * ++c->words_calls);
    if (c->host_fn) {
        if (!c->gather_fn) return fail_arg("comm_words_allgather: the host communicator has no gather callback");
        c->gsend.resize((size_t)L);
        c->grecv.resize((size_t)W);
        for (int64_t k = 0; k < units; ++k) {
            uint32_t *u = words + k * W;
            hipError_t e = hipMemcpyAsync(c->gsend.data(), u + c->rank * L, (size_t)L * 4, hipMemcpyDeviceToHost, stream);
            if (e == hipSuccess) e = hipStreamSynchronize(stream);
            if (e != hipSuccess) return hip_fail("comm_words_allgather (host)", e);
            if (c->gather_fn(c->gather_ctx, c->gsend.data(), L, c->grecv.data()) != 0)
                return fail_arg("comm_words_allgather: the host gather callback failed");
            e = hipMemcpyAsync(u, c->grecv.data(), (size_t)W * 4, hipMemcpyHostToDevice, stream);
            if (e == hipSuccess) e = hipStreamSynchronize(stream);
            if (e != hipSuccess) return hip_fail("comm_words_allgather (host)", e);
        }
        return RG_OK;
    }
    int rc = comm_words_prepare(h);
    if (rc) return rc;
    ncclResult_t r = ncclGroupStart();
    for (int64_t k = 0; k < units && r == ncclSuccess; ++k)
        r = ncclAllGather(words + k * W + c->rank * L, words + k * W, (size_t)L, ncclUint32, c->comm_words, stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess && r != ncclInProgress) return nccl_fail("ncclAllGather (words)", r);
    r = nccl_settle(c, c->comm_words, r2, "ncclAllGather (words)");
    if (r != ncclSuccess) return nccl_fail("ncclAllGather (words, group)", r);
    track(c, stream);                      // under the same deadline as the step's collectives
    return RG_OK;
}

}  // namespace rg

extern "C" int rg_comm_set_host_gather(void *comm, rg_host_gather_fn fn, void *ctx) {
    rg::Comm *c = static_cast<rg::Comm *>(comm);
    if (!c || !c->host_fn) return rg::fail_arg("rg_comm_set_host_gather: not a host-staged communicator");
    c->gather_fn = fn;
    c->gather_ctx = ctx;
    return RG_OK;
}

extern "C" int rg_comm_reduce_scatter_f32(void *comm, void *stream, float *buf, int64_t chunk) {
    return rg::comm_reduce_scatter(comm, (hipStream_t)stream, buf, chunk);
}

extern "C" int rg_comm_allgather_f32(void *comm, void *stream, int32_t n, float *const *bufs, const int64_t *counts) {
    return rg::comm_allgather(comm, (hipStream_t)stream, n, bufs, counts);
}

extern "C" int rg_comm_unique_id(uint8_t *out, int64_t len) {
    if (!out || len < RG_COMM_ID_BYTES) return rg::fail_arg("rg_comm_unique_id: buffer too small");
    static_assert(sizeof(ncclUniqueId) == RG_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return rg::nccl_fail("ncclGetUniqueId", r);
    std::memcpy(out, &id, sizeof(id));
    return RG_OK;
}

extern "C" void *rg_comm_create(const uint8_t *id, int32_t world, int32_t rank, int32_t device) {
    if (!id || world < 1 || rank < 0 || rank >= world) {
        rg::set_error("rg_comm_create: bad argument");
        return nullptr;
    }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) { rg::hip_fail("rg_comm_create: hipSetDevice", e); return nullptr; }
    rg::Comm *c = new (std::nothrow) rg::Comm();
    if (!c) { rg::set_error("rg_comm_create: out of memory"); return nullptr; }
    c->world = world;
    c->rank = rank;
    int lo = 0, hi = 0;
    e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi);
    const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;   // same-device ordering only
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_in, evf);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_out, evf);
    if (e != hipSuccess) {
        rg::hip_fail("rg_comm_create", e);
        delete c;
        return nullptr;
    }
    for (int k = 0; k < rg::Comm::kTrack && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&c->ev_ring[k], evf);
    if (e != hipSuccess) {
        rg::hip_fail("rg_comm_create", e);
        rg_comm_destroy(c);
        return nullptr;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    // non-blocking initialisation polled against a deadline: a rank that never joins (or a
    // peer that died) ends the run with a message instead of a hang until the job's time limit
    c->timeout_s = rg::env_seconds("RG_COMM_TIMEOUT_S", 600.0);
    const double init_s = rg::env_seconds("RG_COMM_INIT_TIMEOUT_S", 300.0);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&c->comm, world, uid, rank, &cfg);
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        if (ncclCommGetAsyncError(c->comm, &r) != ncclSuccess) break;
        if (r == ncclInProgress &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > init_s)
            rg::comm_die(c, "ncclCommInitRankConfig not complete after " + std::to_string((int)init_s) +
                                " s (RG_COMM_INIT_TIMEOUT_S; a rank did not join)");
    }
    if (r != ncclSuccess) {
        rg::nccl_fail("ncclCommInitRankConfig", r);
        if (c->comm) ncclCommAbort(c->comm);
        c->comm = nullptr;
        rg_comm_destroy(c);
        return nullptr;
    }
    c->watchdog = std::thread(rg::watchdog_loop, c);
    return c;
}

extern "C" void *rg_comm_create_local(int32_t world, int32_t rank, int32_t device) {
    if (world < 1 || rank < 0 || rank >= world) {
        rg::set_error("rg_comm_create_local: bad argument");
        return nullptr;
    }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) { rg::hip_fail("rg_comm_create_local: hipSetDevice", e); return nullptr; }
    rg::Comm *c = new (std::nothrow) rg::Comm();
    if (!c) { rg::set_error("rg_comm_create_local: out of memory"); return nullptr; }
    c->world = world;
    c->rank = rank;
    c->local = true;
    int lo = 0, hi = 0;
    e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi);
    const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_in, evf);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_out, evf);
    if (e != hipSuccess) {
        rg::hip_fail("rg_comm_create_local", e);
        delete c;
        return nullptr;
    }
    return c;
}

extern "C" void *rg_comm_create_host(int32_t world, int32_t rank, int32_t device, int64_t max_floats,
                                     rg_host_allreduce_fn fn, void *ctx) {
    if (world < 1 || rank < 0 || rank >= world || max_floats <= 0 || !fn) {
        rg::set_error("rg_comm_create_host: bad argument");
        return nullptr;
    }
    void *h = rg_comm_create_local(world, rank, device);
    if (!h) return nullptr;
    rg::Comm *c = static_cast<rg::Comm *>(h);
    c->local = false;
    c->host_fn = fn;
    c->host_ctx = ctx;
    hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&c->pinned), (size_t)max_floats * sizeof(float),
                                 hipHostMallocDefault);
    if (e != hipSuccess) {
        rg::hip_fail("rg_comm_create_host: pinned staging", e);
        rg_comm_destroy(h);
        return nullptr;
    }
    c->pinned_floats = max_floats;
    return c;
}

extern "C" int rg_comm_destroy(void *h) {
    rg::Comm *c = static_cast<rg::Comm *>(h);
    if (!c) return RG_OK;
    c->stop = true;
    if (c->watchdog.joinable()) c->watchdog.join();
    if (c->stream) hipStreamSynchronize(c->stream);
    for (int k = 0; k < rg::Comm::kTrack; ++k)
        if (c->ev_ring[k]) hipEventDestroy(c->ev_ring[k]);
    if (c->scratch) hipFree(c->scratch);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->comm_words) ncclCommDestroy(c->comm_words);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->ev_in) hipEventDestroy(c->ev_in);
    if (c->ev_out) hipEventDestroy(c->ev_out);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return RG_OK;
}

// what the native communicator itself reports: ncclCommCount / ncclCommUserRank for an RCCL
// communicator (bench.py prints them in the N > 1 line: the ranks RCCL saw, not WORLD_SIZE),
// the configured world / rank for the local and host-staged stand-ins (is_rccl = 0)
extern "C" int rg_comm_info(void *comm, int32_t *count, int32_t *user_rank, int32_t *is_rccl) {
    rg::Comm *c = static_cast<rg::Comm *>(comm);
    if (!c || !count || !user_rank || !is_rccl) return rg::fail_arg("rg_comm_info: null argument");
    if (!c->comm) {
        *count = c->world;
        *user_rank = c->rank;
        *is_rccl = 0;
        return RG_OK;
    }
    int n = 0, r = 0;
    ncclResult_t e = ncclCommCount(c->comm, &n);
    if (e == ncclSuccess) e = ncclCommUserRank(c->comm, &r);
    if (e != ncclSuccess) return rg::nccl_fail("rg_comm_info", e);
    *count = n;
    *user_rank = r;
    *is_rccl = 1;
    return RG_OK;
}

extern "C" int rg_comm_allreduce_sum_f32(void *comm, void *stream, float *buf, int64_t n) {
    int rc = rg::comm_begin(comm, (hipStream_t)stream, buf, n);
    if (rc) return rc;
    return rg::comm_end(comm, (hipStream_t)stream);
}
