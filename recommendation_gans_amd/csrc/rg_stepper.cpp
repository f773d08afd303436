// Native per-step runtime for the MF training loop (host code, no kernels).
//
// Replaces the Python-side loop body of ImplicitFactorizationModel.fit
// (implicit.py:290-298 -> run_train_iteration :347-364) so that one call per step
// enqueues everything, without per-step Python/ctypes overhead:
//
//   side stream  [wait consumed(b')] rg_mt_generate -> rg_mf_prepare (NEXT step) -> ready(b')
//   main stream  [wait ready(b)] rg_mf_pairs -> consumed(b) -> rg_mf_apply
//
// The CPython MT19937 stream is sequential (one workgroup), so the next step's
// words are generated while the current step's two HBM-bound kernels run.  All
// device memory belongs to the caller (PyTorch); the stepper owns one stream and
// four events.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>

#include "rg_common.h"

namespace {

struct Stepper {
    rg_mf_stepper_config_t cfg;
    hipStream_t side = nullptr;
    hipEvent_t ready[2] = {nullptr, nullptr};
    hipEvent_t consumed[2] = {nullptr, nullptr};
    bool consumed_valid[2] = {false, false};
    int set = 0;                 // ping-pong set holding the current tables
    int buf = 1;                 // word/pair buffer of the last consumer
    bool pending = false;        // buffer 1-buf holds words (+ pairs) generated ahead
    rg_mf_step_in_t pending_in{};
    int64_t words_per_step = 0;
    // MT jump-ahead (long steps): the device state is then in window form after the
    // first step; cp_pos tracks CPython's position-in-block of the same stream point
    rg::MtJumpPlan *jump = nullptr;
    bool window_form = false, window_prev = false;
    int32_t cp_pos = 624, cp_pos_prev = 624;
};

int hip_fail(const char *what, hipError_t e) {
    rg::set_error(std::string(what) + ": " + hipGetErrorString(e));
    return RG_E_LAUNCH;
}

rg_mf_batch_t make_batch(const Stepper &st, const rg_mf_step_in_t &in, int b) {
    rg_mf_batch_t x{};
    x.pos_user = in.pos_user;
    x.pos_item = in.pos_item;
    x.n_pos = in.n_pos;
    x.cols = st.cfg.cols;
    x.col_offset = st.cfg.col_offset;
    x.global_cols = st.cfg.global_cols;
    x.global_pos = in.global_pos;
    x.neg_cols = st.cfg.neg_cols;
    x.words = st.cfg.words[b];
    x.pool = st.cfg.pool;
    x.pool_len = st.cfg.pool_len;
    x.n_neg = st.cfg.n_neg;
    x.loss = st.cfg.loss;
    x.pairs = st.cfg.pairs[b];
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

// words (+ prepared pairs) for `in` into buffer b on the side stream, after the
// consumer of buffer `after` (b itself, or the buffer the current step's pairs
// kernel reads: then the sampler runs beside the HBM-bound apply, never beside
// the latency-bound pairs kernel whose slowest block sets its duration)
int produce(Stepper &st, const rg_mf_step_in_t &in, int b, int after) {
    hipError_t e;
    if (st.consumed_valid[after] && (e = hipStreamWaitEvent(st.side, st.consumed[after], 0)) != hipSuccess)
        return hip_fail("stepper: wait consumed", e);
    st.cp_pos_prev = st.cp_pos;
    st.window_prev = st.window_form;
    int rc;
    if (st.jump) {
        rc = rg::mt_produce_jump(st.side, *st.jump, st.cfg.mt_state, st.cfg.words[b], st.cfg.mt_state_before);
        st.window_form = true;
    } else {
        rc = rg_mt_generate(st.side, st.cfg.mt_state, st.cfg.words[b], st.words_per_step, st.cfg.mt_state_before);
    }
    if (rc) return rc;
    st.cp_pos = (int32_t)((st.cp_pos + st.words_per_step - 1) % 624 + 1);
    rg_mf_work_t w = st.cfg.work;
    set_plan(w, in);
    rg_mf_batch_t batch = make_batch(st, in, b);
    rc = rg_mf_prepare(st.side, &batch, &w);
    if (rc) return rc;
    if ((e = hipEventRecord(st.ready[b], st.side)) != hipSuccess) return hip_fail("stepper: record ready", e);
    return RG_OK;
}

// drop words generated ahead: the stream position goes back to before them
int discard(Stepper &st) {
    if (!st.pending) return RG_OK;
    hipError_t e = hipMemcpyAsync(st.cfg.mt_state, st.cfg.mt_state_before, 625 * sizeof(uint32_t),
                                  hipMemcpyDeviceToDevice, st.side);
    if (e != hipSuccess) return hip_fail("stepper: restore MT state", e);
    st.cp_pos = st.cp_pos_prev;
    st.window_form = st.window_prev;
    st.pending = false;
    return RG_OK;
}

// make buffer `b` hold the words + pairs of `in`, visible to `stream`
int acquire(Stepper &st, hipStream_t stream, const rg_mf_step_in_t &in, int *b_out) {
    int b;
    if (st.pending && same_input(st.pending_in, in)) {
        b = 1 - st.buf;
        st.pending = false;
    } else {
        int rc = discard(st);
        if (rc) return rc;
        b = 1 - st.buf;
        rc = produce(st, in, b, b);
        if (rc) return rc;
    }
    hipError_t e = hipStreamWaitEvent(stream, st.ready[b], 0);
    if (e != hipSuccess) return hip_fail("stepper: wait ready", e);
    st.buf = b;
    *b_out = b;
    return RG_OK;
}

int release(Stepper &st, hipStream_t stream) {
    hipError_t e = hipEventRecord(st.consumed[st.buf], stream);
    if (e != hipSuccess) return hip_fail("stepper: record consumed", e);
    st.consumed_valid[st.buf] = true;
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

}  // namespace

extern "C" void *rg_mf_stepper_create(const rg_mf_stepper_config_t *cfg) {
    if (!cfg) { rg::set_error("rg_mf_stepper_create: null config"); return nullptr; }
    if (!cfg->mt_state || !cfg->mt_state_before || !cfg->words[0] || !cfg->words[1] || !cfg->pairs[0] ||
        !cfg->pairs[1]) {
        rg::set_error("rg_mf_stepper_create: null sampler buffers");
        return nullptr;
    }
    Stepper *st = new (std::nothrow) Stepper();
    if (!st) { rg::set_error("rg_mf_stepper_create: out of memory"); return nullptr; }
    st->cfg = *cfg;
    st->set = cfg->current_set;
    st->words_per_step = 2 * (int64_t)cfg->n_neg * cfg->global_cols;
    if (st->cfg.neg_cols <= 0) st->cfg.neg_cols = cfg->global_cols;
    hipError_t e = hipStreamCreateWithFlags(&st->side, hipStreamNonBlocking);
    for (int i = 0; e == hipSuccess && i < 2; ++i) {
        e = hipEventCreateWithFlags(&st->ready[i], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&st->consumed[i], hipEventDisableTiming);
    }
    uint32_t pos = 624;
    if (e == hipSuccess) e = hipMemcpy(&pos, cfg->mt_state + 624, sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        hip_fail("rg_mf_stepper_create", e);
        delete st;
        return nullptr;
    }
    st->cp_pos = st->cp_pos_prev = (int32_t)pos;
    const char *env = getenv("RG_MT_JUMP");
    if (!env || atoi(env)) st->jump = rg::mt_jump_plan_create(st->words_per_step);
    return st;
}

extern "C" int rg_mf_stepper_destroy(void *h) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return RG_OK;
    if (st->side) hipStreamSynchronize(st->side);
    for (int i = 0; i < 2; ++i) {
        if (st->ready[i]) hipEventDestroy(st->ready[i]);
        if (st->consumed[i]) hipEventDestroy(st->consumed[i]);
    }
    if (st->side) hipStreamDestroy(st->side);
    rg::mt_jump_plan_destroy(st->jump);
    delete st;
    return RG_OK;
}

extern "C" int rg_mf_stepper_train(void *h, void *stream, const rg_mf_step_in_t *cur, const rg_mf_step_in_t *next,
                                   float *loss_out, void *ev_apply_begin, void *ev_apply_end) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur) return rg::fail_arg("rg_mf_stepper_train: null handle/input");
    hipStream_t s = (hipStream_t)stream;
    int b;
    int rc = acquire(*st, s, *cur, &b);
    if (rc) return rc;
    rg_mf_work_t w = st->cfg.work;
    set_plan(w, *cur);
    rg_mf_batch_t batch = make_batch(*st, *cur, b);
    rc = rg_mf_pairs(s, &st->cfg.tables[st->set], &batch, &w, 1);
    if (rc) return rc;
    static const bool late = [] { const char *e = getenv("RG_RELEASE_LATE"); return e && atoi(e); }();
    if (!late && (rc = release(*st, s))) return rc;
    if (next) {                                  // generate the next step's words ahead
        const int nb = 1 - b;
        static const bool after_pairs = [] { const char *e = getenv("RG_SAMPLER_AFTER_PAIRS"); return !e || atoi(e); }();
        if ((rc = produce(*st, *next, nb, (after_pairs && !late) ? b : nb))) return rc;
        st->pending = true;
        st->pending_in = *next;
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
    // buffer b is free again once this step ends: recorded here rather than between
    // pairs and apply, so the step's event packets sit at one kernel boundary
    if (late && (rc = release(*st, s))) return rc;
    st->set = 1 - st->set;
    return RG_OK;
}

extern "C" int rg_mf_stepper_acquire(void *h, void *stream, const rg_mf_step_in_t *cur, rg_mf_batch_t *batch_out,
                                     rg_mf_work_t *work_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur || !batch_out || !work_out) return rg::fail_arg("rg_mf_stepper_acquire: null argument");
    int b;
    int rc = acquire(*st, (hipStream_t)stream, *cur, &b);
    if (rc) return rc;
    *batch_out = make_batch(*st, *cur, b);
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
    hipError_t e = hipStreamSynchronize(st->side);
    if (e != hipSuccess) return hip_fail("stepper: sync", e);
    e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_fail("stepper: sync", e);
    if (direction == 0) {   // device -> host: the state after the last CONSUMED word
        const uint32_t *src = st->pending ? st->cfg.mt_state_before : st->cfg.mt_state;
        const bool window = st->pending ? st->window_prev : st->window_form;
        const int32_t pos = st->pending ? st->cp_pos_prev : st->cp_pos;
        uint32_t dev[625];
        e = hipMemcpy(dev, src, 625 * sizeof(uint32_t), hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_fail("stepper: copy MT state", e);
        if (!window) {
            std::memcpy(host_state, dev, sizeof(dev));
            return RG_OK;
        }
        return rg_mt_window_to_cpython(dev, pos, host_state);
    }
    // host -> device: drops anything generated ahead
    st->pending = false;
    st->window_form = st->window_prev = false;
    st->cp_pos = st->cp_pos_prev = (int32_t)host_state[624];
    e = hipMemcpy(st->cfg.mt_state, host_state, 625 * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail("stepper: copy MT state", e);
    return RG_OK;
}
