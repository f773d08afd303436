// Native per-step runtime for the MF training loop (host code, no kernels).
//
// Replaces the Python-side loop body of ImplicitFactorizationModel.fit
// (implicit.py:290-298 -> run_train_iteration :347-364) so that one call per step
// enqueues everything, without per-step Python/ctypes overhead:
//
//   gen stream   rg_mt_generate of stream chunk g (+2 ahead)   -> gen_done[g % 3]
//   prep stream  [gen_done] rg_mf_prepare of the NEXT step     -> ready[buf]
//   main stream  [ready] rg_mf_pairs -> consumed -> rg_mf_apply (-> exchange)
//
// The words a step consumes do not depend on the step's input: draw j of any
// consumer (training step or validation batch) is just the next 2 words of
// CPython's stream, and every consumer of this stepper takes the same number of
// words (n_neg * global_cols draws).  So the stream is cut into fixed chunks,
// generated up to two chunks ahead of consumption into a ring of three buffers
// on their own stream (the sequential MT19937 walk is off the critical path),
// while the input-dependent part (rg_mf_prepare: draws -> pool pairs, in the
// plan's column order) runs on a second stream once the next input is known.
// A prefetch for a different input only redoes rg_mf_prepare; the MT stream is
// never rolled back.  The state CPython would hold after the consumed chunks is
// the start state of the oldest unconsumed chunk (kept per ring slot).
//
// Device memory: the caller (PyTorch) owns tables, scratch, pool and pairs; the
// stepper owns its word ring, the per-slot start states and (jump path) the jump
// tables.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>

#include "rg_common.h"

namespace {

constexpr int kSlots = 3;        // word chunks in the ring
constexpr int kAhead = 2;        // chunks generated ahead of consumption

struct Stepper {
    rg_mf_stepper_config_t cfg;
    hipStream_t gen = nullptr, prep = nullptr;
    uint32_t *words[kSlots] = {nullptr, nullptr, nullptr};
    uint32_t *start_state[kSlots] = {nullptr, nullptr, nullptr};   // [625] state before chunk
    hipEvent_t gen_done[kSlots] = {nullptr, nullptr, nullptr};
    hipEvent_t consumed[kSlots] = {nullptr, nullptr, nullptr};     // after the chunk's pairs kernel
    bool consumed_valid[kSlots] = {false, false, false};
    hipEvent_t ready[2] = {nullptr, nullptr};                      // prepared pairs buffers
    int64_t generated = 0, taken = 0;     // chunks generated / consumed
    // prepared pairs of chunk `prep_chunk` for input `prep_in` in pairs buffer prep_chunk % 2
    bool prepared = false;
    int64_t prep_chunk = -1;
    rg_mf_step_in_t prep_in{};
    int set = 0;                          // ping-pong set holding the current tables
    int64_t words_per_step = 0;
    // MT jump-ahead path (opt-in): the device state is in window form after a jump
    // chunk; cp_pos tracks CPython's position-in-block of the same stream point
    rg::MtJumpPlan *jump = nullptr;
    bool window_form = false;
    int32_t cp_pos = 624;
    bool win_at[kSlots] = {false, false, false};   // form / position at each slot's start
    int32_t pos_at[kSlots] = {624, 624, 624};
    bool release_late = false, prep_after_pairs = true;
};

int hip_fail(const char *what, hipError_t e) {
    rg::set_error(std::string(what) + ": " + hipGetErrorString(e));
    return RG_E_LAUNCH;
}

rg_mf_batch_t make_batch(const Stepper &st, const rg_mf_step_in_t &in, int64_t chunk) {
    rg_mf_batch_t x{};
    x.pos_user = in.pos_user;
    x.pos_item = in.pos_item;
    x.n_pos = in.n_pos;
    x.cols = st.cfg.cols;
    x.col_offset = st.cfg.col_offset;
    x.global_cols = st.cfg.global_cols;
    x.global_pos = in.global_pos;
    x.neg_cols = st.cfg.neg_cols;
    x.words = st.words[chunk % kSlots];
    x.pool = st.cfg.pool;
    x.pool_len = st.cfg.pool_len;
    x.n_neg = st.cfg.n_neg;
    x.loss = st.cfg.loss;
    x.pairs = st.cfg.pairs[chunk % 2];
    return x;
}

void set_plan(rg_mf_work_t &w, const rg_mf_step_in_t &in) {
    w.plan_perm = in.plan_perm;
    w.plan_pos_slot = in.plan_pos_slot;
    w.plan_item_slot_off = in.plan_item_slot_off;
}

bool same_input(const rg_mf_step_in_t &a, const rg_mf_step_in_t &b) {
    return std::memcmp(&a, &b, sizeof(a)) == 0;
}

// generate the next chunk of the stream into its ring slot on the gen stream
int generate_one(Stepper &st) {
    const int slot = (int)(st.generated % kSlots);
    hipError_t e;
    if (st.consumed_valid[slot] && (e = hipStreamWaitEvent(st.gen, st.consumed[slot], 0)) != hipSuccess)
        return hip_fail("stepper: wait consumed", e);
    st.win_at[slot] = st.window_form;
    st.pos_at[slot] = st.cp_pos;
    int rc;
    if (st.jump) {
        rc = rg::mt_produce_jump(st.gen, *st.jump, st.cfg.mt_state, st.words[slot], st.start_state[slot]);
        st.window_form = true;
    } else {
        rc = rg_mt_generate(st.gen, st.cfg.mt_state, st.words[slot], st.words_per_step, st.start_state[slot]);
    }
    if (rc) return rc;
    st.cp_pos = (int32_t)((st.cp_pos + st.words_per_step - 1) % 624 + 1);
    if ((e = hipEventRecord(st.gen_done[slot], st.gen)) != hipSuccess) return hip_fail("stepper: record gen", e);
    ++st.generated;
    return RG_OK;
}

int ensure_generated(Stepper &st, int64_t upto) {
    while (st.generated < upto) {
        int rc = generate_one(st);
        if (rc) return rc;
    }
    return RG_OK;
}

// rg_mf_prepare of chunk `chunk` for input `in` on the prep stream.  `after`: an
// event (or null) the preparation must also follow (the current pairs kernel:
// then it runs beside the HBM-bound apply rather than the latency-bound pairs)
int prepare(Stepper &st, int64_t chunk, const rg_mf_step_in_t &in, hipEvent_t after) {
    const int slot = (int)(chunk % kSlots), buf = (int)(chunk % 2);
    hipError_t e = hipStreamWaitEvent(st.prep, st.gen_done[slot], 0);
    if (e != hipSuccess) return hip_fail("stepper: wait gen", e);
    if (chunk >= 2) {   // pairs buffer `buf` was read by chunk - 2's pairs kernel
        const int prev = (int)((chunk - 2) % kSlots);
        if (st.consumed_valid[prev] && (e = hipStreamWaitEvent(st.prep, st.consumed[prev], 0)) != hipSuccess)
            return hip_fail("stepper: wait pairs buffer", e);
    }
    if (after && (e = hipStreamWaitEvent(st.prep, after, 0)) != hipSuccess)
        return hip_fail("stepper: wait pairs", e);
    rg_mf_work_t w = st.cfg.work;
    set_plan(w, in);
    rg_mf_batch_t batch = make_batch(st, in, chunk);
    int rc = rg_mf_prepare(st.prep, &batch, &w);
    if (rc) return rc;
    if ((e = hipEventRecord(st.ready[buf], st.prep)) != hipSuccess) return hip_fail("stepper: record ready", e);
    st.prepared = true;
    st.prep_chunk = chunk;
    st.prep_in = in;
    return RG_OK;
}

// make the next chunk's words + pairs for `in` visible to `stream`; returns the chunk
int acquire(Stepper &st, hipStream_t stream, const rg_mf_step_in_t &in, int64_t *chunk_out) {
    const int64_t chunk = st.taken;
    int rc = ensure_generated(st, chunk + 1);
    if (rc) return rc;
    if (!(st.prepared && st.prep_chunk == chunk && same_input(st.prep_in, in))) {
        if ((rc = prepare(st, chunk, in, nullptr))) return rc;
    }
    hipError_t e = hipStreamWaitEvent(stream, st.ready[chunk % 2], 0);
    if (e != hipSuccess) return hip_fail("stepper: wait ready", e);
    *chunk_out = chunk;
    return RG_OK;
}

// the consumer of chunk `taken` has been enqueued on `stream`
int release(Stepper &st, hipStream_t stream) {
    const int slot = (int)(st.taken % kSlots);
    hipError_t e = hipEventRecord(st.consumed[slot], stream);
    if (e != hipSuccess) return hip_fail("stepper: record consumed", e);
    st.consumed_valid[slot] = true;
    ++st.taken;
    if (st.prepared && st.prep_chunk < st.taken) st.prepared = false;
    return RG_OK;
}

rg_mf_loss_t loss_of(const Stepper &st, int64_t global_pos, float *out) {
    rg_mf_loss_t l{};
    l.n_partials = st.cfg.n_partials;
    l.out = out;
    const double n = (double)st.cfg.n_neg;
    const double gp = (double)global_pos, gc = (double)st.cfg.neg_cols;
    switch (st.cfg.loss) {
        case RG_LOSS_POINTWISE: l.inv_a = 1.0 / gp; l.inv_b = 1.0 / (n * gc); break;
        case RG_LOSS_BPR:
        case RG_LOSS_HINGE: l.inv_a = 1.0 / (n * gp); l.inv_b = 0.0; break;
        default: l.inv_a = 1.0 / gp; l.inv_b = 0.0;
    }
    return l;
}

// Adam step scalars exactly as torch/_single_tensor_adam computes them in Python
// floats: bias_correction = 1 - beta ** step (C pow, as CPython's float_pow),
// step_size = lr / bc1, bc2_sqrt = bc2 ** 0.5
rg_opt_t opt_at(const Stepper &st, int64_t t) {
    rg_opt_t o = st.cfg.opt;
    if (o.kind == RG_OPT_ADAM) {
        const double bc1 = 1.0 - std::pow(st.cfg.beta1_d, (double)t);
        const double bc2 = 1.0 - std::pow(st.cfg.beta2_d, (double)t);
        o.step_size = (float)(st.cfg.lr_d / bc1);
        o.bias_correction2_sqrt = (float)std::pow(bc2, 0.5);
    }
    return o;
}

bool env_flag(const char *name, bool dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) != 0 : dflt;
}

void destroy(Stepper *st) {
    if (st->gen) hipStreamSynchronize(st->gen);
    if (st->prep) hipStreamSynchronize(st->prep);
    for (int i = 0; i < kSlots; ++i) {
        if (st->gen_done[i]) hipEventDestroy(st->gen_done[i]);
        if (st->consumed[i]) hipEventDestroy(st->consumed[i]);
        if (st->words[i]) hipFree(st->words[i]);
        if (st->start_state[i]) hipFree(st->start_state[i]);
    }
    for (int i = 0; i < 2; ++i)
        if (st->ready[i]) hipEventDestroy(st->ready[i]);
    if (st->gen) hipStreamDestroy(st->gen);
    if (st->prep) hipStreamDestroy(st->prep);
    rg::mt_jump_plan_destroy(st->jump);
    delete st;
}

}  // namespace

extern "C" void *rg_mf_stepper_create(const rg_mf_stepper_config_t *cfg) {
    if (!cfg) { rg::set_error("rg_mf_stepper_create: null config"); return nullptr; }
    if (!cfg->mt_state || !cfg->pairs[0] || !cfg->pairs[1]) {
        rg::set_error("rg_mf_stepper_create: null sampler buffers");
        return nullptr;
    }
    Stepper *st = new (std::nothrow) Stepper();
    if (!st) { rg::set_error("rg_mf_stepper_create: out of memory"); return nullptr; }
    st->cfg = *cfg;
    st->set = cfg->current_set;
    st->words_per_step = 2 * (int64_t)cfg->n_neg * cfg->global_cols;
    if (st->cfg.neg_cols <= 0) st->cfg.neg_cols = cfg->global_cols;
    st->release_late = env_flag("RG_RELEASE_LATE", false);
    st->prep_after_pairs = env_flag("RG_PREP_AFTER_PAIRS", true);
    // separate priorities keep the three streams on separate hardware queues: the
    // walk is background work (lowest), the short prepare is on the step's path (highest)
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    const int prio_mode = getenv("RG_STREAM_PRIO") ? atoi(getenv("RG_STREAM_PRIO")) : 1;
    if (e == hipSuccess)
        e = hipStreamCreateWithPriority(&st->gen, hipStreamNonBlocking, prio_mode ? least : 0);
    if (e == hipSuccess)
        e = hipStreamCreateWithPriority(&st->prep, hipStreamNonBlocking, prio_mode ? greatest : 0);
    // the events only order streams of this device: no system-scope fence (which
    // writes back and invalidates caches at every marker, ~7 us of idle per packet)
    const int ev_mode = getenv("RG_EVENT_MODE") ? atoi(getenv("RG_EVENT_MODE")) : 1;
    const unsigned evf = hipEventDisableTiming | (ev_mode == 1 ? hipEventDisableSystemFence
                                                 : ev_mode == 2 ? hipEventReleaseToDevice : 0u);
    for (int i = 0; e == hipSuccess && i < kSlots; ++i) {
        e = hipEventCreateWithFlags(&st->gen_done[i], evf);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&st->consumed[i], evf);
        if (e == hipSuccess) e = hipMalloc(&st->words[i], (size_t)(st->words_per_step + RG_MT_PAD) * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc(&st->start_state[i], 625 * sizeof(uint32_t));
    }
    for (int i = 0; e == hipSuccess && i < 2; ++i) e = hipEventCreateWithFlags(&st->ready[i], evf);
    uint32_t pos = 624;
    if (e == hipSuccess) e = hipMemcpy(&pos, cfg->mt_state + 624, sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        hip_fail("rg_mf_stepper_create", e);
        destroy(st);
        return nullptr;
    }
    st->cp_pos = (int32_t)pos;
    if (env_flag("RG_MT_JUMP", false)) st->jump = rg::mt_jump_plan_create(st->words_per_step);
    return st;
}

extern "C" int rg_mf_stepper_destroy(void *h) {
    Stepper *st = static_cast<Stepper *>(h);
    if (st) destroy(st);
    return RG_OK;
}

extern "C" int rg_mf_stepper_train(void *h, void *stream, const rg_mf_step_in_t *cur, const rg_mf_step_in_t *next,
                                   float *loss_out, void *ev_apply_begin, void *ev_apply_end) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur) return rg::fail_arg("rg_mf_stepper_train: null handle/input");
    hipStream_t s = (hipStream_t)stream;
    int64_t chunk;
    int rc = acquire(*st, s, *cur, &chunk);
    if (rc) return rc;
    rg_mf_work_t w = st->cfg.work;
    set_plan(w, *cur);
    rg_mf_batch_t batch = make_batch(*st, *cur, chunk);
    if ((rc = rg_mf_pairs(s, &st->cfg.tables[st->set], &batch, &w, 1))) return rc;
    if (!st->release_late && (rc = release(*st, s))) return rc;
    if ((rc = ensure_generated(*st, chunk + 1 + kAhead))) return rc;       // keep the walk ahead
    if (next) {
        const hipEvent_t after = (st->prep_after_pairs && !st->release_late) ? st->consumed[chunk % kSlots] : nullptr;
        if ((rc = prepare(*st, chunk + 1, *next, after))) return rc;
    }
    st->cfg.step += 1;
    const rg_opt_t o = opt_at(*st, st->cfg.step);
    const rg_mf_loss_t l = loss_of(*st, cur->global_pos, loss_out);
    hipError_t e;
    const rg_mf_tables_t *tb = &st->cfg.tables[st->set];
    const int64_t U = tb->num_users, R = tb->num_users + tb->num_items;
    if (st->cfg.item_grad) {                     // user-sharded data parallel
        if ((rc = rg_mf_grads(s, tb, &w, st->cfg.item_grad, U, R, &l))) return rc;
        if (st->cfg.comm && (rc = rg::comm_begin(st->cfg.comm, s, st->cfg.item_grad,
                                                 tb->num_items * (int64_t)(tb->dim + 1) + 1)))
            return rc;
    }
    if (ev_apply_begin && (e = hipEventRecord((hipEvent_t)ev_apply_begin, s)) != hipSuccess)
        return hip_fail("stepper: record event", e);
    if (st->cfg.item_grad) {
        if ((rc = rg_mf_apply(s, tb, &w, &o, 0, U, nullptr))) return rc;
    } else {
        if ((rc = rg_mf_apply(s, tb, &w, &o, 0, -1, &l))) return rc;
    }
    if (ev_apply_end && (e = hipEventRecord((hipEvent_t)ev_apply_end, s)) != hipSuccess)
        return hip_fail("stepper: record event", e);
    if (st->cfg.item_grad) {
        if (st->cfg.comm && (rc = rg::comm_end(st->cfg.comm, s))) return rc;
        if ((rc = rg_mf_apply_dense(s, tb, st->cfg.item_grad, &o, U, R, loss_out))) return rc;
    }
    if (st->release_late && (rc = release(*st, s))) return rc;
    st->set = 1 - st->set;
    return RG_OK;
}

extern "C" int rg_mf_stepper_acquire(void *h, void *stream, const rg_mf_step_in_t *cur, rg_mf_batch_t *batch_out,
                                     rg_mf_work_t *work_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur || !batch_out || !work_out) return rg::fail_arg("rg_mf_stepper_acquire: null argument");
    int64_t chunk;
    int rc = acquire(*st, (hipStream_t)stream, *cur, &chunk);
    if (rc) return rc;
    *batch_out = make_batch(*st, *cur, chunk);
    *work_out = st->cfg.work;
    set_plan(*work_out, *cur);
    return RG_OK;
}

extern "C" int rg_mf_stepper_release(void *h, void *stream) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_release: null handle");
    return release(*st, (hipStream_t)stream);
}

extern "C" int rg_mf_stepper_opt(void *h, int64_t step, rg_opt_t *out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !out) return rg::fail_arg("rg_mf_stepper_opt: null argument");
    *out = opt_at(*st, step);
    return RG_OK;
}

extern "C" int rg_mf_stepper_state(void *h, int32_t *current_set, int64_t *step) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_state: null handle");
    if (current_set) *current_set = st->set;
    if (step) *step = st->cfg.step;
    return RG_OK;
}

extern "C" int rg_mf_stepper_advance(void *h, int32_t flip_sets, int64_t steps) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_advance: null handle");
    if (flip_sets) st->set = 1 - st->set;
    st->cfg.step += steps;
    return RG_OK;
}

extern "C" int rg_mf_stepper_sync_mt(void *h, uint32_t *host_state, int32_t direction) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !host_state) return rg::fail_arg("rg_mf_stepper_sync_mt: null argument");
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_fail("stepper: sync", e);
    if (direction == 0) {   // device -> host: the state after the last CONSUMED chunk
        const bool ahead = st->generated > st->taken;
        const int slot = (int)(st->taken % kSlots);
        const uint32_t *src = ahead ? st->start_state[slot] : st->cfg.mt_state;
        const bool window = ahead ? st->win_at[slot] : st->window_form;
        const int32_t pos = ahead ? st->pos_at[slot] : st->cp_pos;
        uint32_t dev[625];
        e = hipMemcpy(dev, src, 625 * sizeof(uint32_t), hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_fail("stepper: copy MT state", e);
        if (!window) {
            std::memcpy(host_state, dev, sizeof(dev));
            return RG_OK;
        }
        return rg_mt_window_to_cpython(dev, pos, host_state);
    }
    // host -> device: chunks generated ahead are dropped
    st->generated = st->taken;
    st->prepared = false;
    st->window_form = false;
    st->cp_pos = (int32_t)host_state[624];
    e = hipMemcpy(st->cfg.mt_state, host_state, 625 * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail("stepper: copy MT state", e);
    return RG_OK;
}
