// Native per-step runtime for the MF training loop (host code, no kernels).
//
// Replaces the Python-side loop body of ImplicitFactorizationModel.fit
// (implicit.py:290-298 -> run_train_iteration :347-364) so that one call per step
// enqueues everything, without per-step Python/ctypes overhead.
//
// Word stream (default for a single-GPU split step: the inline walk below).  The words a
// step consumes do not depend on the step's input: draw
// j of any consumer (training step or validation batch) is just the next 2 words
// of CPython's stream, and every consumer of this stepper takes the same number of
// words W = 2 * n_neg * global_cols (one "unit").  The stream is cut into ring
// slots of G units, generated up to two slots ahead of consumption into a ring of
// three slot buffers on a stream of its own (the sequential MT19937 walk, or the
// jump-ahead head + parallel tails, stays off the critical path; one generation
// launch and two events per G steps).  The state CPython would hold after the
// consumed units is the start state of their slot advanced by the units consumed
// inside it (rg_mf_stepper_sync_mt).
//
// Inline walk (split step, one GPU, when the walk hides under the dense pass): slots of
// one unit; the words of unit t+2 are walked by one extra workgroup of step t's dense
// pass (rg_mf_apply_prepare_gen), so the steady state has no generator launch and no
// event: the generator stream only makes up for gaps (the first two units, validation
// consumers that ran ahead).  Events between streams are recorded lazily, when a
// different stream has to be ordered after a production or a consumer.
//
// Overlapped step (RG_FUSED=1; pointwise / bpr / hinge; measured slower):
//   main  rg_mf_step_front(pairs of t | marked prepare of t+1 | cold-row update of t)
//         -> rg_mf_step_hot(touched rows of t, loss)
// Two launches per step on one stream and no per-step event: the prepare of the
// next step rides in the front grid, so the only cross-stream dependency left is
// one wait per ring slot for the generated words.
//
// Split step (the default; adaptive hinge always):
//   main  rg_mf_pairs -> rg_mf_apply_prepare (dense update + the NEXT step's prepare in
//         one launch) (-> exchange): no side stream, no per-step event
// External consumers (validation, NCF, the Python split DP steps) go through
// acquire / release, which prepare on a side stream ordered after the caller's work.
//
// Device memory: the caller (PyTorch) owns tables, scratch, pool and pairs; the
// stepper owns its word ring, the per-slot start states, the row stamps of the
// overlapped step and (jump path) the jump tables.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>

#include "rg_common.h"
#include "rg_owner.h"

#ifndef RG_PIPE_DEFAULT
#define RG_PIPE_DEFAULT 0
#endif

#ifndef RG_OWNER_USER_AFTER_DEFAULT
#define RG_OWNER_USER_AFTER_DEFAULT 0
#endif
#ifndef RG_PIPE2_DEFAULT
#define RG_PIPE2_DEFAULT 0
#endif
namespace {

constexpr int kSlots = 3;        // word slots in the ring
constexpr int kAheadSlots = 2;   // slots generated ahead of the one being consumed

struct Stepper {
    rg_mf_stepper_config_t cfg;
    bool failed = false;          // a step stopped half applied (pipe2's cold launch refused): unusable
    hipStream_t gen = nullptr, prep = nullptr;
    int64_t W = 0;                        // words per unit
    int64_t G = 1;                        // units per ring slot
    uint32_t *words[kSlots] = {nullptr, nullptr, nullptr};
    uint32_t *start_state[kSlots] = {nullptr, nullptr, nullptr};   // [625] state before the slot
    hipEvent_t gen_done[kSlots] = {nullptr, nullptr, nullptr};
    hipEvent_t consumed[kSlots] = {nullptr, nullptr, nullptr};     // after the slot's last consumer
    // Who produced / has seen / last consumed each slot.  Events are recorded lazily,
    // only when a DIFFERENT stream has to be ordered after that work (same-stream
    // order is free): the single-GPU split step then issues no event at all.
    // (a null hipStream_t is the legacy default stream, a real consumer: validity is tracked
    // by flags, never by null handles)
    hipStream_t prod[kSlots] = {nullptr, nullptr, nullptr};        // producing stream
    bool gen_rec[kSlots] = {false, false, false};                  // gen_done recorded after the production
    hipStream_t seen[kSlots] = {nullptr, nullptr, nullptr};        // a stream ordered after the production
    bool seen_ok[kSlots] = {false, false, false};
    hipStream_t cons_on[kSlots] = {nullptr, nullptr, nullptr};     // stream of the last consumer
    bool cons_ok[kSlots] = {false, false, false};                  // the slot was consumed since its production
    bool cons_rec[kSlots] = {false, false, false};                 // consumed recorded after that consumer
    bool inline_gen = false;              // split step: the walk of unit t+2 rides in step t's dense pass
    hipEvent_t ready[2] = {nullptr, nullptr};                      // side-stream prepared pairs buffers
    bool side_pending[2] = {false, false};                         // ready[b] not yet waited by the consumer
    hipEvent_t mark = nullptr;                                     // consumer-stream point a side prepare follows
    int64_t unit_base = 0;                // unit of relative slot 0 (reset when the state is loaded)
    int64_t gen_slots = 0;                // relative slots generated
    int64_t taken = 0;                    // units consumed
    // prepared pairs of unit prep_unit for input prep_in, in pairs buffer prep_unit % 2
    bool prepared = false;
    int64_t prep_unit = -1;
    rg_mf_step_in_t prep_in{};
    int32_t prep_serial = 0;              // nonzero: prepared with row marks (stamp array prep_arr)
    int prep_arr = 0;
    int32_t serial = 0;                   // last mark serial issued
    int32_t *stamp[2] = {nullptr, nullptr};   // [U + I] each, lazily allocated
    int set = 0;                          // ping-pong set holding the current tables
    bool fused = false;
    bool hot_scan = true;
    // MT jump-ahead path: the device state is in window form after a jump slot;
    // cp_pos tracks CPython's position-in-block of the same stream point
    rg::MtJumpPlan *jump = nullptr;
    bool window_form = false;
    int32_t cp_pos = 624;
    bool win_at[kSlots] = {false, false, false};   // form / position at each slot's start
    int32_t pos_at[kSlots] = {624, 624, 624};
    // owner step over a communicator (dp_mode 2, world > 1; opt-in RG_OWNER_MT_SLICE=1 -- the
    // emulated rank 0 of 8 measured 75.0 us per step with it, 74.6 without: the jump launches cost
    // the same either way, and the slot's MT work already hides beside the step): each rank
    // walks only ITS slice of every unit's words (L = W / world words at offset rank * L): a slot's
    // G slices come from one head walk, one jump launch and G parallel segments, the device state
    // ending G * W ahead; the slices are all-gathered on the generator stream
    // (rg::comm_words_allgather), and gstate -- the global stream's state at the start of the next
    // slot to produce, what the CPython state exports read -- is advanced by a jump of G * W per
    // slot.  One rank's MT work per slot: G * L words walked G-wide and two jump launches, instead
    // of the whole global draw's G * W words
    bool slice = false;
    int64_t L = 0;
    rg::MtJumpPlan *slice_plan = nullptr, *gjump = nullptr, *rjump = nullptr;
    uint32_t *gstate = nullptr, *jscratch = nullptr;
    // owner-sharded step (dp_mode 2) between its parts
    rg_mf_step_in_t own_in{};
    int64_t own_unit = -1;
    int own_stage = 0;                    // 0 idle, 1 after begin, 2 after mid
    hipEvent_t own_back = nullptr;        // after the owner backward (the item gradient may start)
    hipEvent_t own_grads = nullptr;       // train_owner: the lists are pulled (the user update may start)
    hipEvent_t own_users = nullptr;       // train_owner: the user update is done (the next step may start)
    // lazy dense pass (single-rank split step): deferred cold user-row updates
    bool lazy = false;
    bool lazy_pending = false;            // some user rows lag the current step
    int64_t lazy_base = 0;                // absolute step of last_rel == 0
    int32_t *last_rel = nullptr;          // [U]
    int32_t *umark = nullptr;             // [U]
    float *consts = nullptr;              // [2 * n_consts] Adam constants per absolute step
    int64_t n_consts = 0;
    uint64_t *rows_done = nullptr;        // diagnostic counter (rg_mf_stepper_lazy_count)
    bool count_rows = false;
    // claimed list slots (single-rank split step, rg_mf_work_t claim_num_users): the prepare of
    // unit u claims in counts[u % 2] (cfg.work.row_count and a second array owned here), so the
    // next unit's claims never meet the dense pass that reads and resets this unit's counts
    bool claim = false;
    int32_t *counts[2] = {nullptr, nullptr};
    int32_t *own_counts = nullptr;
    bool count_dirty[2] = {false, false};  // counts[b] hold claims no dense pass consumed yet
    bool prep_claimed = false;             // the prepared pairs carry claimed slots
    bool prep_in_pairs = false;            // split step: the next prepare rides in the pair pass
    // pipelined step (rg_mf_pipe_step; single rank, claimed slots, pointwise / bpr / hinge):
    // launch t updates step t's rows, runs step t+1's pair pass and step t+2's prepare.  A unit's
    // scratch by its parity -- claims in pcounts[u % 3], lists / overflow accumulators / partials
    // / planned partials in set u % 2 ([0] the caller's cfg.work, [1] owned here) -- and the
    // users its pair pass reads in hot[u % 3] (length pint[u % 3]).
    bool pipe = false;
    int32_t *pcounts[3] = {nullptr, nullptr, nullptr};
    int32_t *p_counts2 = nullptr;          // owned: pcounts[2]
    bool pdirty[3] = {false, false, false};   // pcounts[k] hold claims no dense pass consumed
    int32_t *p_list1 = nullptr;
    int64_t *p_hg1 = nullptr, *p_hbg1 = nullptr;
    float *p_part1 = nullptr, *p_prow1 = nullptr, *p_pbias1 = nullptr;
    int32_t *hot[3] = {nullptr, nullptr, nullptr};
    int32_t *pint = nullptr;               // [0..3) hot-list lengths, [3..5) gates, [5] error flag
    bool pair_dirty[2] = {false, false};   // overflow accumulators of set k hold a pair pass's adds
    int64_t paired = -1;                   // unit whose pair pass has run (its lists ready)
    rg_mf_step_in_t paired_in{};
    int64_t hot_prepped = -1;              // unit prepared with claims and a hot list, pair pending
    rg_mf_step_in_t hot_in{};
    int64_t last_pipe = -1;                // unit of the last pipelined launch (its counter resets)
    // two-launch pipelined step (train_pipe2, the single-GPU default): the same per-unit scratch
    // parities as `pipe`, no gate
    bool pipe2 = false;
};

int hip_fail(const char *what, hipError_t e) {
    rg::set_error(std::string(what) + ": " + hipGetErrorString(e));
    return RG_E_LAUNCH;
}

int64_t rel_slot(const Stepper &st, int64_t unit) { return (unit - st.unit_base) / st.G; }

uint32_t *unit_words(const Stepper &st, int64_t unit) {
    const int64_t rel = unit - st.unit_base;
    return st.words[(rel / st.G) % kSlots] + (rel % st.G) * st.W;
}

rg_mf_batch_t make_batch(const Stepper &st, const rg_mf_step_in_t &in, int64_t unit) {
    rg_mf_batch_t x{};
    x.pos_user = in.pos_user;
    x.pos_item = in.pos_item;
    x.n_pos = in.n_pos;
    x.cols = st.cfg.cols;
    x.col_offset = st.cfg.col_offset;
    x.global_cols = st.cfg.global_cols;
    x.global_pos = in.global_pos;
    x.neg_cols = st.cfg.neg_cols;
    x.words = unit_words(st, unit);
    x.pool = st.cfg.pool;
    x.pool_len = st.cfg.pool_len;
    x.n_neg = st.cfg.n_neg;
    x.loss = st.cfg.loss;
    x.pairs = st.cfg.pairs[unit % 2];
    return x;
}

void set_plan(rg_mf_work_t &w, const rg_mf_step_in_t &in) {
    w.plan_perm = in.plan_perm;
    w.plan_pos_slot = in.plan_pos_slot;
    w.plan_item_slot_off = in.plan_item_slot_off;
}

rg_mf_work_t work_for(const Stepper &st, const rg_mf_step_in_t &in) {
    rg_mf_work_t w = st.cfg.work;
    set_plan(w, in);
    return w;
}

// the scratch of training unit `unit` (claimed slots: its parity's count array)
rg_mf_work_t train_work(const Stepper &st, const rg_mf_step_in_t &in, int64_t unit) {
    rg_mf_work_t w = work_for(st, in);
    if (st.claim) {
        w.row_count = st.counts[unit % 2];
        w.claim_num_users = st.cfg.tables[0].num_users;
    }
    return w;
}

// before a claiming prepare into counts[b]: drop claims a dense pass never consumed (a
// prefetched step that did not run, or ran as validation)
int clean_counts(Stepper &st, hipStream_t s, int b) {
    if (!st.claim || !st.count_dirty[b]) return RG_OK;
    const rg_mf_tables_t &t = st.cfg.tables[0];
    hipError_t e = hipMemsetAsync(st.counts[b], 0, (size_t)(t.num_users + t.num_items) * sizeof(int32_t), s);
    if (e != hipSuccess) return hip_fail("stepper: reset claimed counts", e);
    st.count_dirty[b] = false;
    return RG_OK;
}

bool same_input(const rg_mf_step_in_t &a, const rg_mf_step_in_t &b) {
    return std::memcmp(&a, &b, sizeof(a)) == 0;
}

// `stream` is ordered after the production of `slot` (an event wait only across streams)
int see(Stepper &st, hipStream_t stream, int slot) {
    if ((st.seen_ok[slot] && st.seen[slot] == stream) || st.prod[slot] == stream) {
        st.seen[slot] = stream;
        st.seen_ok[slot] = true;
        return RG_OK;
    }
    hipError_t e = hipSuccess;
    if (!st.gen_rec[slot]) {
        e = hipEventRecord(st.gen_done[slot], st.prod[slot]);
        st.gen_rec[slot] = true;
    }
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, st.gen_done[slot], 0);
    if (e != hipSuccess) return hip_fail("stepper: wait gen", e);
    st.seen[slot] = stream;
    st.seen_ok[slot] = true;
    return RG_OK;
}

// producer stream `p` may overwrite `slot`: ordered after the slot's last consumer
int free_for(Stepper &st, hipStream_t p, int slot) {
    if (!st.cons_ok[slot] || st.cons_on[slot] == p) return RG_OK;
    hipError_t e = hipSuccess;
    if (!st.cons_rec[slot]) {
        e = hipEventRecord(st.consumed[slot], st.cons_on[slot]);
        st.cons_rec[slot] = true;
    }
    if (e == hipSuccess) e = hipStreamWaitEvent(p, st.consumed[slot], 0);
    return e == hipSuccess ? RG_OK : hip_fail("stepper: wait consumed", e);
}

// bookkeeping of a slot production enqueued on `p` (the walk advances the one MT state,
// so productions are ordered: a production on another stream than the previous one waits)
int begin_production(Stepper &st, hipStream_t p, int slot) {
    int rc = free_for(st, p, slot);
    if (rc) return rc;
    if (st.gen_slots > 0 && (rc = see(st, p, (int)((st.gen_slots - 1) % kSlots)))) return rc;
    st.win_at[slot] = st.window_form;
    st.pos_at[slot] = st.cp_pos;
    return RG_OK;
}

void end_production(Stepper &st, hipStream_t p, int slot) {
    st.cp_pos = (int32_t)((st.cp_pos + st.G * st.W - 1) % 624 + 1);
    st.prod[slot] = p;
    st.gen_rec[slot] = false;
    st.seen[slot] = p;
    st.seen_ok[slot] = true;
    st.cons_ok[slot] = false;
    st.cons_rec[slot] = false;
    ++st.gen_slots;
}

// slice mode: this rank's device state at its slice of the unit gstate starts (a jump of rank * L)
int slice_reset(Stepper &st) {
    hipError_t e = hipMemcpyAsync(st.cfg.mt_state, st.gstate, 625 * sizeof(uint32_t), hipMemcpyDeviceToDevice, st.gen);
    if (e != hipSuccess) return hip_fail("stepper: slice state", e);
    if (st.rjump) return rg::mt_produce_jump(st.gen, *st.rjump, st.cfg.mt_state, st.jscratch, nullptr, 0);
    return RG_OK;
}

// generate the next ring slot (G units) on the gen stream
int generate_one(Stepper &st) {
    const int slot = (int)(st.gen_slots % kSlots);
    int rc = begin_production(st, st.gen, slot);
    if (rc) return rc;
    if (st.slice) {
        hipError_t e = hipMemcpyAsync(st.start_state[slot], st.gstate, 625 * sizeof(uint32_t),
                                      hipMemcpyDeviceToDevice, st.gen);
        if (e != hipSuccess) return hip_fail("stepper: slot start state", e);
        // the slot's G slices in one head + jump + parallel-segment production
        rc = rg::mt_produce_jump(st.gen, *st.slice_plan, st.cfg.mt_state, st.words[slot] + (int64_t)st.cfg.rank * st.L,
                                 nullptr, 0);
        if (rc == RG_OK) rc = rg::comm_words_allgather(st.cfg.comm, st.gen, st.words[slot], st.G, st.W, st.L);
        if (rc == RG_OK) rc = rg::mt_produce_jump(st.gen, *st.gjump, st.gstate, st.jscratch, nullptr, 0);
        st.window_form = true;
    } else if (st.jump) {
        rc = rg::mt_produce_jump(st.gen, *st.jump, st.cfg.mt_state, st.words[slot], st.start_state[slot]);
        st.window_form = true;
    } else {
        rc = rg_mt_generate(st.gen, st.cfg.mt_state, st.words[slot], st.G * st.W, st.start_state[slot]);
    }
    if (rc) return rc;
    end_production(st, st.gen, slot);
    hipError_t e = hipEventRecord(st.gen_done[slot], st.gen);
    if (e != hipSuccess) return hip_fail("stepper: record gen", e);
    st.gen_rec[slot] = true;
    return RG_OK;
}

// slots up to the one holding `unit` (+ `ahead` more) are generated or queued
int generate_upto(Stepper &st, int64_t unit, int ahead) {
    const int64_t upto = rel_slot(st, unit) + 1 + ahead;
    while (st.gen_slots < upto) {
        int rc = generate_one(st);
        if (rc) return rc;
    }
    return RG_OK;
}

int keep_ahead(Stepper &st, int64_t unit) { return generate_upto(st, unit, kAheadSlots); }

// make the words of `unit` visible to `stream`
int wait_words(Stepper &st, hipStream_t stream, int64_t unit) {
    return see(st, stream, (int)(rel_slot(st, unit) % kSlots));
}

// an outstanding side-stream write of pairs buffer b must land before `stream` uses it
int wait_side(Stepper &st, hipStream_t stream, int b) {
    if (!st.side_pending[b]) return RG_OK;
    hipError_t e = hipStreamWaitEvent(stream, st.ready[b], 0);
    if (e != hipSuccess) return hip_fail("stepper: wait ready", e);
    st.side_pending[b] = false;
    return RG_OK;
}

// unmarked rg_mf_prepare of `unit` for `in` on the prep stream, ordered after everything
// the consumer stream holds so far (in a training call: the current pairs kernel, so it
// runs beside the HBM-bound apply)
int prepare_side(Stepper &st, hipStream_t consumer, int64_t unit, const rg_mf_step_in_t &in) {
    int rc = keep_ahead(st, unit);
    if (rc) return rc;
    hipError_t e = hipEventRecord(st.mark, consumer);
    if (e == hipSuccess) e = hipStreamWaitEvent(st.prep, st.mark, 0);
    if (e != hipSuccess) return hip_fail("stepper: order prepare", e);
    if ((rc = wait_words(st, st.prep, unit))) return rc;
    const rg_mf_work_t w = work_for(st, in);
    const rg_mf_batch_t batch = make_batch(st, in, unit);
    if ((rc = rg_mf_prepare(st.prep, &batch, &w))) return rc;
    const int b = (int)(unit % 2);
    if ((e = hipEventRecord(st.ready[b], st.prep)) != hipSuccess) return hip_fail("stepper: record ready", e);
    st.side_pending[b] = true;
    st.prepared = true;
    st.prep_unit = unit;
    st.prep_in = in;
    st.prep_serial = 0;
    st.prep_claimed = false;
    return RG_OK;
}

// the same prepare on the consumer stream itself, in stream order (no events: a caller that
// enqueues it after the step's last kernel trades the prepare's few microseconds for the two
// cross-queue hops of prepare_side, each a bubble of ~10 us on the consumer queue)
int prepare_inline(Stepper &st, hipStream_t consumer, int64_t unit, const rg_mf_step_in_t &in) {
    int rc = keep_ahead(st, unit);
    if (rc) return rc;
    const int b = (int)(unit % 2);
    if ((rc = wait_side(st, consumer, b))) return rc;   // an earlier side write of this buffer
    if ((rc = wait_words(st, consumer, unit))) return rc;
    const rg_mf_work_t w = work_for(st, in);
    const rg_mf_batch_t batch = make_batch(st, in, unit);
    if ((rc = rg_mf_prepare(consumer, &batch, &w))) return rc;
    st.side_pending[b] = false;
    st.prepared = true;
    st.prep_unit = unit;
    st.prep_in = in;
    st.prep_serial = 0;
    st.prep_claimed = false;
    return RG_OK;
}

int ensure_stamps(Stepper &st) {
    if (st.stamp[0]) return RG_OK;
    const rg_mf_tables_t &t = st.cfg.tables[0];
    const size_t bytes = (size_t)(t.num_users + t.num_items) * sizeof(int32_t);
    hipError_t e = hipSuccess;
    for (int k = 0; k < 2 && e == hipSuccess; ++k) {
        e = hipMalloc(&st.stamp[k], bytes);
        if (e == hipSuccess) e = hipMemset(st.stamp[k], 0, bytes);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e == hipSuccess ? RG_OK : hip_fail("stepper: stamps", e);
}

rg_mf_mark_t mark_of(const Stepper &st, int arr, int32_t serial) {
    rg_mf_mark_t m{};
    m.stamp = st.stamp[arr];
    m.num_users = st.cfg.tables[0].num_users;
    m.serial = serial;
    return m;
}

int32_t next_serial(Stepper &st) {
    st.serial = st.serial == 0x7fffffff ? 1 : st.serial + 1;
    return st.serial;
}

// the consumer of `taken` has been enqueued on `stream`
int release(Stepper &st, hipStream_t stream) {
    const int64_t rel = st.taken - st.unit_base;
    ++st.taken;
    if (st.prepared && st.prep_unit < st.taken) st.prepared = false;
    if ((rel + 1) % st.G == 0) {                         // the slot's last unit
        const int slot = (int)((rel / st.G) % kSlots);
        st.cons_on[slot] = stream;                       // its event is recorded when a producer needs it
        st.cons_ok[slot] = true;
        st.cons_rec[slot] = false;
    }
    return st.inline_gen ? RG_OK : keep_ahead(st, st.taken);
}

int lazy_flush(Stepper &st, hipStream_t s);

// words + pairs of unit `taken` for `in`, visible to `stream` (split-step consumers)
int pipe_abandon(Stepper &st, hipStream_t s);

int acquire(Stepper &st, hipStream_t stream, const rg_mf_step_in_t &in, int64_t *unit_out) {
    const int64_t unit = st.taken;
    int rc = pipe_abandon(st, stream);    // a pipelined unit ahead is this consumer's now
    if (rc) return rc;
    rc = lazy_flush(st, stream);          // external consumers read every row
    if (rc) return rc;
    // the consumer's tail walks (gen_mode 2): only a missing slot on the generator stream
    // (running ahead there would leave the in-launch walks nothing to do)
    rc = st.inline_gen && st.cfg.gen_mode >= 2 ? generate_upto(st, unit, 0) : keep_ahead(st, unit);
    if (rc) return rc;
    // an external consumer's pair pass claims in cfg.work.row_count (= counts[0]) by itself
    if ((rc = clean_counts(st, stream, 0))) return rc;
    if (!(st.prepared && st.prep_unit == unit && same_input(st.prep_in, in) && !st.prep_claimed)) {
        if ((rc = prepare_side(st, stream, unit, in))) return rc;
    }
    if ((rc = wait_side(st, stream, (int)(unit % 2)))) return rc;
    if ((rc = wait_words(st, stream, unit))) return rc;   // the adaptive-max kernel reads them
    *unit_out = unit;
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

// Adam constants of every absolute step < upto on the device (grown by doubling; the
// copy is synchronous and happens O(log steps) times in a run)
int ensure_consts(Stepper &st, int64_t upto) {
    if (upto < st.n_consts) return RG_OK;
    int64_t cap = st.n_consts > 0 ? st.n_consts : 4096;
    while (cap <= upto) cap *= 2;
    float *host = static_cast<float *>(std::malloc((size_t)cap * 2 * sizeof(float)));
    if (!host) { rg::set_error("stepper: out of host memory"); return RG_E_LAUNCH; }
    for (int64_t s = 0; s < cap; ++s) {
        const rg_opt_t o = opt_at(st, s > 0 ? s : 1);
        host[2 * s] = o.step_size;
        host[2 * s + 1] = o.bias_correction2_sqrt;
    }
    float *dev = nullptr;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMalloc(&dev, (size_t)cap * 2 * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(dev, host, (size_t)cap * 2 * sizeof(float), hipMemcpyHostToDevice);
    std::free(host);
    if (e != hipSuccess) return hip_fail("stepper: step constants", e);
    if (st.consts) (void)hipFree(st.consts);
    st.consts = dev;
    st.n_consts = cap;
    return RG_OK;
}

rg_mf_lazy_t lazy_of(const Stepper &st, int64_t step, bool full) {
    rg_mf_lazy_t l{};
    l.last_rel = st.last_rel;
    l.umark = st.umark;
    l.step_consts = st.consts;
    l.n_consts = st.n_consts;
    l.base = st.lazy_base;
    l.step = step;
    l.full = full ? 1 : 0;
    l.rows_done = st.count_rows ? st.rows_done : nullptr;
    return l;
}

// every user row up to the current step, into the current set (no-op when none lags)
int lazy_flush(Stepper &st, hipStream_t s) {
    if (!st.lazy || !st.lazy_pending) return RG_OK;
    int rc = ensure_consts(st, st.cfg.step + 1);
    if (rc) return rc;
    const rg_opt_t o = opt_at(st, st.cfg.step > 0 ? st.cfg.step : 1);
    const rg_mf_lazy_t l = lazy_of(st, st.cfg.step, true);
    if ((rc = rg_mf_lazy_flush(s, &st.cfg.tables[st.set], &o, &l))) return rc;
    st.lazy_pending = false;
    return RG_OK;
}

bool env_flag(const char *name, bool dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) != 0 : dflt;
}

// a switch of the A/B build only (RG_AB, rg_common.h): the product keeps its default
bool ab_flag(const char *name, bool dflt) {
#if RG_AB
    return env_flag(name, dflt);
#else
    (void)name;
    return dflt;
#endif
}

int ab_int(const char *name, int dflt) {
#if RG_AB
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
#else
    (void)name;
    return dflt;
#endif
}

int record(void *ev, hipStream_t s) {
    if (!ev) return RG_OK;
    hipError_t e = hipEventRecord((hipEvent_t)ev, s);
    return e == hipSuccess ? RG_OK : hip_fail("stepper: record event", e);
}

// Split step: [marked-free prepare if not prefetched] -> rg_mf_pairs -> rg_mf_apply_prepare
// (the dense update plus the NEXT step's prepare in one launch), all on the caller's
// stream: no side stream, no per-step event; the words of a ring slot are waited for
// once per slot.  User-sharded DP: item gradient -> all-reduce (communicator stream)
// beside the user-shard update (+ next prepare) -> item update.
int train_split(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur, const rg_mf_step_in_t *next,
                float *loss_out, void *ev0, void *ev1) {
    const int64_t unit = st.taken;
    // inline: units t, t+1 must exist (the gen stream makes up for any gap, e.g. after a
    // validation pass); unit t+2 is walked inside this step's dense pass
    int rc = st.inline_gen ? generate_upto(st, unit + 1, 0) : keep_ahead(st, unit);
    if (rc) return rc;
    rg_mf_work_t w = train_work(st, cur, unit);
    const rg_mf_batch_t batch = make_batch(st, cur, unit);
    if ((rc = wait_side(st, s, (int)(unit % 2)))) return rc;      // a side prepare (acquire path) of this buffer
    if (!(st.prepared && st.prep_unit == unit && same_input(st.prep_in, cur) && st.prep_claimed == st.claim)) {
        if ((rc = wait_words(st, s, unit))) return rc;
        if ((rc = clean_counts(st, s, (int)(unit % 2)))) return rc;
        if ((rc = rg_mf_prepare(s, &batch, &w))) return rc;
        st.count_dirty[unit % 2] = st.claim;
        st.prepared = true;
        st.prep_unit = unit;
        st.prep_in = cur;
        st.prep_serial = 0;
        st.prep_claimed = st.claim;
    }
    if (st.cfg.loss == RG_LOSS_ADAPTIVE_HINGE && (rc = wait_words(st, s, unit))) return rc;   // adapt-max reads them
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    rg_mf_batch_t nbatch{};
    rg_mf_work_t nw{};
    // RG_PREP_IN_PAIRS: the next step's prepare (pool lookups, claims) in extra workgroups of
    // this pair pass, beside its latency-bound gathers, instead of in the dense pass
    const bool pip = st.prep_in_pairs && next && st.cfg.loss != RG_LOSS_ADAPTIVE_HINGE && !st.cfg.item_grad;
    if (pip) {
        // only the slot of unit + 1 (this unit is not released yet; see train_lazy)
        if (!st.inline_gen && (rc = generate_upto(st, unit + 1, 0))) return rc;
        if ((rc = wait_side(st, s, (int)((unit + 1) % 2)))) return rc;
        if ((rc = wait_words(st, s, unit + 1))) return rc;
        if ((rc = clean_counts(st, s, (int)((unit + 1) % 2)))) return rc;
        nbatch = make_batch(st, *next, unit + 1);
        nw = train_work(st, *next, unit + 1);
        if ((rc = rg_mf_pairs_prepare(s, tb, &batch, &w, &nbatch, &nw, nullptr, 0))) return rc;
    }
    else if ((rc = rg_mf_pairs(s, tb, &batch, &w, 1))) {
        return rc;
    }
    if ((rc = release(st, s))) return rc;
    if (next && !pip) {
        if (!st.inline_gen && (rc = keep_ahead(st, unit + 1))) return rc;
        if ((rc = wait_side(st, s, (int)((unit + 1) % 2)))) return rc;
        if ((rc = wait_words(st, s, unit + 1))) return rc;
        if ((rc = clean_counts(st, s, (int)((unit + 1) % 2)))) return rc;
        nbatch = make_batch(st, *next, unit + 1);
        nw = train_work(st, *next, unit + 1);
    }
    rg_mt_gen_t gen{};
    int gen_slot = -1;
    if (st.inline_gen && !st.cfg.item_grad && st.gen_slots == rel_slot(st, unit + 2)) {
        gen_slot = (int)(st.gen_slots % kSlots);
        if ((rc = begin_production(st, s, gen_slot))) return rc;
        gen.state = st.cfg.mt_state;
        gen.out = st.words[gen_slot];
        gen.state_before = st.start_state[gen_slot];
        gen.nwords = st.G * st.W;
    }
    st.cfg.step += 1;
    const rg_opt_t o = opt_at(st, st.cfg.step);
    const rg_mf_loss_t l = loss_of(st, cur.global_pos, loss_out);
    const int64_t U = tb->num_users, R = tb->num_users + tb->num_items;
    if (st.cfg.item_grad) {                     // user-sharded data parallel
        if ((rc = rg_mf_grads(s, tb, &w, st.cfg.item_grad, U, R, &l))) return rc;
        if (st.cfg.comm && (rc = rg::comm_begin(st.cfg.comm, s, st.cfg.item_grad,
                                                tb->num_items * (int64_t)(tb->dim + 1) + 1)))
            return rc;
    }
    rg::launch_events() = rg::LaunchEvents{(hipEvent_t)ev0, (hipEvent_t)ev1};   // timed by the dispatch itself
    rc = rg_mf_apply_prepare_gen(s, tb, &w, &o, 0, st.cfg.item_grad ? U : R, st.cfg.item_grad ? nullptr : &l,
                                 next && !pip ? &nbatch : nullptr, next && !pip ? &nw : nullptr,
                                 gen_slot >= 0 ? &gen : nullptr);
    rg::launch_events() = rg::LaunchEvents{};
    if (rc) return rc;
    if (gen_slot >= 0) end_production(st, s, gen_slot);
    if (st.cfg.item_grad) {
        if (st.cfg.comm && (rc = rg::comm_end(st.cfg.comm, s))) return rc;
        if ((rc = rg_mf_apply_dense(s, tb, st.cfg.item_grad, &o, U, R, loss_out))) return rc;
    }
    st.count_dirty[unit % 2] = false;           // the dense pass consumed (and reset) this unit's claims
    if (next) {
        st.count_dirty[(unit + 1) % 2] = st.claim;
        st.prepared = true;
        st.prep_unit = unit + 1;
        st.prep_in = *next;
        st.prep_serial = 0;
        st.prep_claimed = st.claim;
    }
    st.set = 1 - st.set;
    return RG_OK;
}

// ---------------------------------------------------------------- pipelined step
rg_mf_work_t pipe_work(const Stepper &st, const rg_mf_step_in_t &in, int64_t unit) {
    rg_mf_work_t w = work_for(st, in);
    w.row_count = st.pcounts[unit % 3];
    w.claim_num_users = st.cfg.tables[0].num_users;
    if (unit % 2) {
        w.row_list = st.p_list1;
        w.hot_grad = st.p_hg1;
        w.hot_bias_grad = st.p_hbg1;
        w.loss_partials = st.p_part1;
        w.part_row = st.p_prow1;
        w.part_bias = st.p_pbias1;
    }
    return w;
}

int pipe_memset(void *p, size_t bytes, hipStream_t s, const char *what) {
    hipError_t e = hipMemsetAsync(p, 0, bytes, s);
    return e == hipSuccess ? RG_OK : hip_fail(what, e);
}

int pipe_clean_counts(Stepper &st, hipStream_t s, int k) {
    if (!st.pdirty[k]) return RG_OK;
    const rg_mf_tables_t &t = st.cfg.tables[0];
    int rc = pipe_memset(st.pcounts[k], (size_t)(t.num_users + t.num_items) * sizeof(int32_t), s,
                         "stepper: reset claims");
    if (rc == RG_OK) st.pdirty[k] = false;
    return rc;
}

// the overflow accumulators of set k after a pair pass whose dense pass never ran
int pipe_clean_accum(Stepper &st, hipStream_t s, int k) {
    if (!st.pair_dirty[k]) return RG_OK;
    const rg_mf_tables_t &t = st.cfg.tables[0];
    const int64_t rows = t.num_users + t.num_items;
    int64_t *hg = k ? st.p_hg1 : reinterpret_cast<int64_t *>(st.cfg.work.hot_grad);
    int64_t *hb = k ? st.p_hbg1 : reinterpret_cast<int64_t *>(st.cfg.work.hot_bias_grad);
    int rc = pipe_memset(hg, (size_t)rows * t.dim * sizeof(int64_t), s, "stepper: reset overflow");
    if (rc == RG_OK) rc = pipe_memset(hb, (size_t)rows * sizeof(int64_t), s, "stepper: reset overflow");
    if (rc == RG_OK) st.pair_dirty[k] = false;
    return rc;
}

// drop every pipelined unit not trained yet (a pair pass and / or a prepare ahead): their
// claims and overflow adds are cleared; their words stay (input independent)
int pipe_abandon(Stepper &st, hipStream_t s) {
    if (!st.pipe && !st.pipe2) return RG_OK;
    int rc = RG_OK;
    for (int k = 0; k < 3 && rc == RG_OK; ++k) rc = pipe_clean_counts(st, s, k);
    for (int k = 0; k < 2 && rc == RG_OK; ++k) rc = pipe_clean_accum(st, s, k);
    st.paired = -1;
    st.hot_prepped = -1;
    st.last_pipe = -1;
    st.prepared = false;
    st.count_dirty[0] = st.count_dirty[1] = false;
    return rc;
}

// Pipelined step of unit t = taken (see rg_mf_pipe_step).  Cold start (no pair pass of t
// pending): prepare t (claims), pair pass t, prepare t+1 with its hot list, each its own launch;
// then, while `next` is known, one launch per step.  Without `next` the step is the plain dense
// pass and the pipeline drains.
int train_pipe(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur, const rg_mf_step_in_t *next,
               const rg_mf_step_in_t *next2, float *loss_out, void *ev0, void *ev1) {
    const int64_t unit = st.taken;
    int rc = generate_upto(st, unit + (next2 ? 2 : next ? 1 : 0), 0);
    if (rc) return rc;
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    const rg_mf_tables_t &t0 = st.cfg.tables[0];
    rg_mf_work_t w = pipe_work(st, cur, unit);
    const rg_mf_batch_t batch = make_batch(st, cur, unit);
    if (!(st.paired == unit && same_input(st.paired_in, cur))) {
        // cold start: whatever ran ahead belongs to another input
        if ((rc = pipe_abandon(st, s))) return rc;
        if ((rc = wait_side(st, s, (int)(unit % 2))) || (rc = wait_words(st, s, unit))) return rc;
        if ((rc = rg_mf_prepare(s, &batch, &w))) return rc;
        st.pdirty[unit % 3] = true;
        if ((rc = rg_mf_pairs(s, tb, &batch, &w, 1))) return rc;
        st.pair_dirty[unit % 2] = true;
        st.paired = unit;
        st.paired_in = cur;
    }
    st.cfg.step += 1;
    const rg_opt_t o = opt_at(st, st.cfg.step);
    const rg_mf_loss_t l = loss_of(st, cur.global_pos, loss_out);
    if (!next) {                       // the last step of a sequence: dense pass only
        if ((rc = release(st, s))) return rc;
        rg::launch_events() = rg::LaunchEvents{(hipEvent_t)ev0, (hipEvent_t)ev1};
        rc = rg_mf_apply_prepare_gen(s, tb, &w, &o, 0, t0.num_users + t0.num_items, &l, nullptr, nullptr, nullptr);
        rg::launch_events() = rg::LaunchEvents{};
        if (rc) return rc;
        st.pdirty[unit % 3] = false;
        st.pair_dirty[unit % 2] = false;
        st.paired = -1;
        st.last_pipe = -1;
        st.set = 1 - st.set;
        return RG_OK;
    }
    // step t+1: prepared with claims and its hot list (done by the previous launch, or now)
    const int64_t u1 = unit + 1, u2 = unit + 2;
    rg_mf_work_t w1 = pipe_work(st, *next, u1);
    const rg_mf_batch_t b1 = make_batch(st, *next, u1);
    int32_t *nhot = st.pint, *gate = st.pint + 3, *err = st.pint + 5;
    if (!(st.hot_prepped == u1 && same_input(st.hot_in, *next))) {
        if ((rc = pipe_clean_counts(st, s, (int)(u1 % 3)))) return rc;
        if ((rc = pipe_clean_accum(st, s, (int)(u1 % 2)))) return rc;
        if ((rc = wait_side(st, s, (int)(u1 % 2))) || (rc = wait_words(st, s, u1))) return rc;
        if ((rc = pipe_memset(nhot + u1 % 3, sizeof(int32_t), s, "stepper: hot list"))) return rc;
        if ((rc = rg_mf_prepare_hot(s, &b1, &w1, st.hot[u1 % 3], nhot + u1 % 3))) return rc;
        st.pdirty[u1 % 3] = true;
        st.hot_prepped = u1;
        st.hot_in = *next;
    }
    if (st.last_pipe != unit - 1) {    // counters a previous launch of the sequence would have reset
        if ((rc = pipe_memset(gate + unit % 2, sizeof(int32_t), s, "stepper: gate")) ||
            (rc = pipe_memset(nhot + u2 % 3, sizeof(int32_t), s, "stepper: hot list")))
            return rc;
    }
    rg_mf_batch_t b2{};
    rg_mf_work_t w2{};
    if (next2) {
        if ((rc = pipe_clean_counts(st, s, (int)(u2 % 3)))) return rc;
        if ((rc = wait_side(st, s, (int)(u2 % 2))) || (rc = wait_words(st, s, u2))) return rc;
        b2 = make_batch(st, *next2, u2);
        w2 = pipe_work(st, *next2, u2);
    }
    if ((rc = pipe_clean_accum(st, s, (int)(u1 % 2)))) return rc;   // set u1 % 2 is the pair pass's
    if ((rc = release(st, s))) return rc;
    rg_mt_gen_t gen{};
    int gen_slot = -1;
    if (st.inline_gen && st.gen_slots == rel_slot(st, unit + 3)) {
        gen_slot = (int)(st.gen_slots % kSlots);
        if ((rc = begin_production(st, s, gen_slot))) return rc;
        gen.state = st.cfg.mt_state;
        gen.out = st.words[gen_slot];
        gen.state_before = st.start_state[gen_slot];
        gen.nwords = st.G * st.W;
    }
    rg_mf_pipe_t pp{};
    pp.hot_users = st.hot[u1 % 3];
    pp.nhot = nhot + u1 % 3;
    pp.counts_next = st.pcounts[u1 % 3];
    pp.gate = gate + unit % 2;
    pp.gate_next = gate + u1 % 2;
    pp.nhot_free = nhot + unit % 3;
    pp.hot_out = next2 ? st.hot[u2 % 3] : nullptr;
    pp.nhot_out = next2 ? nhot + u2 % 3 : nullptr;
    pp.err = err;
    rg::launch_events() = rg::LaunchEvents{(hipEvent_t)ev0, (hipEvent_t)ev1};
    rc = rg_mf_pipe_step(s, tb, &w, &o, &l, &b1, &w1, next2 ? &b2 : nullptr, next2 ? &w2 : nullptr, &pp,
                         gen_slot >= 0 ? &gen : nullptr);
    rg::launch_events() = rg::LaunchEvents{};
    if (rc) return rc;
    if (gen_slot >= 0) end_production(st, s, gen_slot);
    st.pdirty[unit % 3] = false;                 // the dense pass consumed and reset its claims
    st.pair_dirty[unit % 2] = false;             // and its overflow accumulators
    st.pair_dirty[u1 % 2] = true;
    st.paired = u1;
    st.paired_in = *next;
    if (next2) {
        st.pdirty[u2 % 3] = true;
        st.hot_prepped = u2;
        st.hot_in = *next2;
    } else {
        st.hot_prepped = -1;
    }
    st.last_pipe = unit;
    st.set = 1 - st.set;
    return RG_OK;
}

// Two-launch pipelined step of unit t = taken (rg_mf_pipe2_hot / rg_mf_pipe2_cold):
//   hot  (t): step t's dense update of every item row and of the users step t+1's pair pass reads
//   cold (t): step t+1's pair pass | the MT walk | step t+2's prepare | step t's dense update of
//             every other user
// Preconditions carried from the previous call: step t's pair pass ran (its lists), step t+1 was
// prepared with claims and its hot list.  A cold start (nothing pending, or pending for another
// input) runs prepare t, pair pass t and prepare t+1 as launches of their own; without `next` the
// step is the plain dense pass and the pipeline drains; without `next2` the cold launch prepares
// nothing ahead (the next call prepares its t+1 on its own).
int train_pipe2(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur, const rg_mf_step_in_t *next,
                const rg_mf_step_in_t *next2, float *loss_out, void *ev0, void *ev1) {
    const int64_t unit = st.taken;
    int rc = st.inline_gen ? generate_upto(st, unit + (next2 ? 2 : next ? 1 : 0), 0) : keep_ahead(st, unit);
    if (rc) return rc;
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    const rg_mf_tables_t &t0 = st.cfg.tables[0];
    rg_mf_work_t w = pipe_work(st, cur, unit);
    const rg_mf_batch_t batch = make_batch(st, cur, unit);
    if (!(st.paired == unit && same_input(st.paired_in, cur))) {
        // cold start: whatever ran ahead belongs to another input
        if ((rc = pipe_abandon(st, s))) return rc;
        if ((rc = wait_side(st, s, (int)(unit % 2))) || (rc = wait_words(st, s, unit))) return rc;
        if ((rc = rg_mf_prepare(s, &batch, &w))) return rc;
        st.pdirty[unit % 3] = true;
        if ((rc = rg_mf_pairs(s, tb, &batch, &w, 1))) return rc;
        st.pair_dirty[unit % 2] = true;
        st.paired = unit;
        st.paired_in = cur;
    }
    st.cfg.step += 1;
    const rg_opt_t o = opt_at(st, st.cfg.step);
    const rg_mf_loss_t l = loss_of(st, cur.global_pos, loss_out);
    const int64_t U = t0.num_users, R = U + t0.num_items;
    if (!next) {                       // the last step of a sequence: dense pass only
        if ((rc = release(st, s))) return rc;
        rg::launch_events() = rg::LaunchEvents{(hipEvent_t)ev0, (hipEvent_t)ev1};
        rc = rg_mf_apply_prepare_gen(s, tb, &w, &o, 0, R, &l, nullptr, nullptr, nullptr);
        rg::launch_events() = rg::LaunchEvents{};
        if (rc) return rc;
        st.pdirty[unit % 3] = false;
        st.pair_dirty[unit % 2] = false;
        st.paired = -1;
        st.hot_prepped = -1;
        st.set = 1 - st.set;
        return RG_OK;
    }
    const int64_t u1 = unit + 1, u2 = unit + 2;
    rg_mf_work_t w1 = pipe_work(st, *next, u1);
    const rg_mf_batch_t b1 = make_batch(st, *next, u1);
    int32_t *nhot = st.pint;
    if (!(st.hot_prepped == u1 && same_input(st.hot_in, *next))) {
        if ((rc = pipe_clean_counts(st, s, (int)(u1 % 3)))) return rc;
        if ((rc = pipe_clean_accum(st, s, (int)(u1 % 2)))) return rc;
        if ((rc = wait_side(st, s, (int)(u1 % 2))) || (rc = wait_words(st, s, u1))) return rc;
        if ((rc = pipe_memset(nhot + u1 % 3, sizeof(int32_t), s, "stepper: hot list"))) return rc;
        if ((rc = rg_mf_prepare_hot(s, &b1, &w1, st.hot[u1 % 3], nhot + u1 % 3))) return rc;
        st.pdirty[u1 % 3] = true;
        st.hot_prepped = u1;
        st.hot_in = *next;
    }
    rg_mf_batch_t b2{};
    rg_mf_work_t w2{};
    if (next2) {
        if ((rc = pipe_clean_counts(st, s, (int)(u2 % 3)))) return rc;
        if ((rc = wait_side(st, s, (int)(u2 % 2))) || (rc = wait_words(st, s, u2))) return rc;
        b2 = make_batch(st, *next2, u2);
        w2 = pipe_work(st, *next2, u2);
    }
    if ((rc = pipe_clean_accum(st, s, (int)(u1 % 2)))) return rc;   // set u1 % 2 is the pair pass's
    if ((rc = release(st, s))) return rc;
    rg_mt_gen_t gen{};
    int gen_slot = -1;
    if (st.inline_gen && st.gen_slots == rel_slot(st, unit + 3)) {
        gen_slot = (int)(st.gen_slots % kSlots);
        if ((rc = begin_production(st, s, gen_slot))) return rc;
        gen.state = st.cfg.mt_state;
        gen.out = st.words[gen_slot];
        gen.state_before = st.start_state[gen_slot];
        gen.nwords = st.G * st.W;
    }
    const int64_t hot_cap = std::min<int64_t>(U, (int64_t)(1 + st.cfg.n_neg) * st.cfg.cols);
    if ((rc = rg_mf_pipe2_hot(s, tb, &w, &o, &l, st.hot[u1 % 3], nhot + u1 % 3, hot_cap,
                              next2 ? nhot + u2 % 3 : nullptr, nullptr))) {
        st.cfg.step -= 1;                          // nothing of this step ran
        return rc;
    }
    rg::launch_events() = rg::LaunchEvents{(hipEvent_t)ev0, (hipEvent_t)ev1};   // the cold launch
    rc = rg_mf_pipe2_cold(s, tb, &w, &o, &b1, &w1, st.pcounts[u1 % 3], next2 ? &b2 : nullptr,
                          next2 ? &w2 : nullptr, next2 ? st.hot[u2 % 3] : nullptr, next2 ? nhot + u2 % 3 : nullptr,
                          gen_slot >= 0 ? &gen : nullptr);
    rg::launch_events() = rg::LaunchEvents{};
    if (rc) {
        // the hot launch updated part of the rows: the step is half applied and cannot be resumed
        st.failed = true;
        return rc;
    }
    if (gen_slot >= 0) end_production(st, s, gen_slot);
    st.pdirty[unit % 3] = false;                 // the two launches consumed and reset its claims
    st.pair_dirty[unit % 2] = false;             // and its overflow accumulators
    st.pair_dirty[u1 % 2] = true;
    st.paired = u1;
    st.paired_in = *next;
    if (next2) {
        st.pdirty[u2 % 3] = true;
        st.hot_prepped = u2;
        st.hot_in = *next2;
    } else {
        st.hot_prepped = -1;
    }
    st.set = 1 - st.set;
    return RG_OK;
}

// Lazy split step (single rank):
//   main  rg_mf_pairs_prepare (this step's pairs + the NEXT step's prepare, which marks the
//         users that step reads) -> rg_mf_apply_lazy (items, and the users with a gradient
//         or a mark; a full pass when no next step is known; + the inline MT walk)
// Every row a kernel reads is current; rows nobody reads lag until rg_mf_stepper_flush /
// the next full pass / an external consumer (acquire) catches them up.
int train_lazy(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur, const rg_mf_step_in_t *next,
               float *loss_out, void *ev0, void *ev1) {
    const int64_t unit = st.taken;
    int rc = st.inline_gen ? generate_upto(st, unit + 1, 0) : keep_ahead(st, unit);
    if (rc) return rc;
    rg_mf_work_t w = work_for(st, cur);
    const rg_mf_batch_t batch = make_batch(st, cur, unit);
    if ((rc = wait_side(st, s, (int)(unit % 2)))) return rc;
    if (!(st.prepared && st.prep_unit == unit && same_input(st.prep_in, cur))) {
        // the pairs were not prepared (with marks) by the previous lazy step: bring every row
        // up to date first, so whatever this step reads is current
        if ((rc = lazy_flush(st, s))) return rc;
        if ((rc = wait_words(st, s, unit))) return rc;
        if ((rc = rg_mf_prepare(s, &batch, &w))) return rc;
        st.prepared = true;
        st.prep_unit = unit;
        st.prep_in = cur;
        st.prep_serial = 0;
    }
    if (!st.lazy_pending) {                    // every row current at cfg.step: restart the clock
        hipError_t e = hipMemsetAsync(st.last_rel, 0, (size_t)st.cfg.tables[0].num_users * sizeof(int32_t), s);
        if (e != hipSuccess) return hip_fail("stepper: reset last_rel", e);
        st.lazy_base = st.cfg.step;
    }
    if (st.cfg.loss == RG_LOSS_ADAPTIVE_HINGE && (rc = wait_words(st, s, unit))) return rc;
    const int64_t t = st.cfg.step + 1;
    if ((rc = ensure_consts(st, t + 1))) return rc;
    rg_mf_batch_t nbatch{};
    rg_mf_work_t nw{};
    if (next) {
        // only the slot holding unit + 1: this unit is not released yet, and keeping two
        // slots ahead of unit + 1 could overwrite its words under the adaptive-max kernel
        // (release() below keeps the ring ahead once the pair pass is enqueued)
        if (!st.inline_gen && (rc = generate_upto(st, unit + 1, 0))) return rc;
        if ((rc = wait_side(st, s, (int)((unit + 1) % 2)))) return rc;
        if ((rc = wait_words(st, s, unit + 1))) return rc;
        nbatch = make_batch(st, *next, unit + 1);
        nw = work_for(st, *next);
    }
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    if ((rc = rg_mf_pairs_prepare(s, tb, &batch, &w, next ? &nbatch : nullptr, next ? &nw : nullptr, st.umark,
                                  (int32_t)(t + 1))))
        return rc;
    if ((rc = release(st, s))) return rc;
    rg_mt_gen_t gen{};
    int gen_slot = -1;
    if (st.inline_gen && st.gen_slots == rel_slot(st, unit + 2)) {
        gen_slot = (int)(st.gen_slots % kSlots);
        if ((rc = begin_production(st, s, gen_slot))) return rc;
        gen.state = st.cfg.mt_state;
        gen.out = st.words[gen_slot];
        gen.state_before = st.start_state[gen_slot];
        gen.nwords = st.G * st.W;
    }
    st.cfg.step = t;
    const rg_opt_t o = opt_at(st, t);
    const rg_mf_loss_t l = loss_of(st, cur.global_pos, loss_out);
    const rg_mf_lazy_t lz = lazy_of(st, t, next == nullptr);
    rg::launch_events() = rg::LaunchEvents{(hipEvent_t)ev0, (hipEvent_t)ev1};
    rc = rg_mf_apply_lazy(s, tb, &w, &o, &l, &lz, gen_slot >= 0 ? &gen : nullptr);
    rg::launch_events() = rg::LaunchEvents{};
    if (rc) return rc;
    if (gen_slot >= 0) end_production(st, s, gen_slot);
    if (next) {
        st.prepared = true;
        st.prep_unit = unit + 1;
        st.prep_in = *next;
        st.prep_serial = 0;
    }
    st.lazy_pending = next != nullptr;
    st.set = 1 - st.set;
    return RG_OK;
}

// Replicated data-parallel step (dp_mode 1): every rank holds every row and
// consumes its column slice of ONE global draw, so R ranks at batch B compute exactly the
// reference's step at batch R*B (up to fp32 summation order).  First half: pairs of this
// rank's columns -> the next step's prepare -> every row's data gradient, rank-major.
int dp_begin(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur, const rg_mf_step_in_t *next, float *loss_out,
             void *ev0, void *ev1) {
    const int64_t unit = st.taken;
    int rc = keep_ahead(st, unit);
    if (rc) return rc;
    rg_mf_work_t w = work_for(st, cur);
    const rg_mf_batch_t batch = make_batch(st, cur, unit);
    if ((rc = wait_side(st, s, (int)(unit % 2)))) return rc;
    if (!(st.prepared && st.prep_unit == unit && same_input(st.prep_in, cur))) {
        if ((rc = wait_words(st, s, unit))) return rc;
        if ((rc = rg_mf_prepare(s, &batch, &w))) return rc;
    }
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    if ((rc = rg_mf_pairs(s, tb, &batch, &w, 1))) return rc;
    if ((rc = release(st, s))) return rc;
    st.prepared = false;
    if (next) {
        if ((rc = keep_ahead(st, unit + 1))) return rc;
        if ((rc = wait_side(st, s, (int)((unit + 1) % 2)))) return rc;
        if ((rc = wait_words(st, s, unit + 1))) return rc;
        const rg_mf_batch_t nbatch = make_batch(st, *next, unit + 1);
        const rg_mf_work_t nw = work_for(st, *next);
        if ((rc = rg_mf_prepare(s, &nbatch, &nw))) return rc;
        st.prepared = true;
        st.prep_unit = unit + 1;
        st.prep_in = *next;
        st.prep_serial = 0;
    }
    const rg_mf_loss_t l = loss_of(st, cur.global_pos, loss_out);
    if ((rc = record(ev0, s))) return rc;
    if ((rc = rg_mf_grads_sharded(s, tb, &w, st.cfg.grad_buf, st.cfg.shard_users, st.cfg.shard_items, st.cfg.world,
                                  &l)))
        return rc;
    return record(ev1, s);
}

// second half: this rank's rows from its reduce-scattered chunk, then flip the sets
int dp_end(Stepper &st, hipStream_t s, float *loss_out) {
    st.cfg.step += 1;
    const rg_opt_t o = opt_at(st, st.cfg.step);
    int rc = rg_mf_apply_shard(s, &st.cfg.tables[st.set], st.cfg.grad_buf, &o, st.cfg.shard_users,
                               st.cfg.shard_items, st.cfg.world, st.cfg.rank, loss_out);
    if (rc) return rc;
    st.set = 1 - st.set;
    return RG_OK;
}

int64_t dp_chunk(const Stepper &st) {
    return rg_mf_grad_chunk(st.cfg.shard_users, st.cfg.shard_items, st.cfg.tables[0].dim);
}

// the whole replicated step with the communicator: begin -> RCCL reduce-scatter -> end ->
// RCCL all-gather of the four tables the step wrote (now the current set)
int train_dp(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur, const rg_mf_step_in_t *next, float *loss_out,
             void *ev0, void *ev1) {
    int rc = dp_begin(st, s, cur, next, loss_out, ev0, ev1);
    if (rc) return rc;
    if ((rc = rg::comm_reduce_scatter(st.cfg.comm, s, st.cfg.grad_buf, dp_chunk(st)))) return rc;
    if ((rc = dp_end(st, s, loss_out))) return rc;
    const rg_mf_tables_t &t = st.cfg.tables[st.set];
    float *bufs[4] = {const_cast<float *>(t.user_w), const_cast<float *>(t.item_w), const_cast<float *>(t.user_b),
                      const_cast<float *>(t.item_b)};
    const int64_t d = t.dim;
    const int64_t counts[4] = {st.cfg.shard_users * d, st.cfg.shard_items * d, st.cfg.shard_users,
                               st.cfg.shard_items};
    return rg::comm_allgather(st.cfg.comm, s, 4, bufs, counts);
}

// ---------------------------------------------------------------- owner-sharded step (dp_mode 2)
rg_mf_owner_batch_t owner_batch(const Stepper &st, const rg_mf_step_in_t &in, int64_t unit) {
    rg_mf_owner_batch_t b{};
    b.pos_user = in.pos_user;
    b.pos_item = in.pos_item;
    b.n_pos = in.n_pos;
    b.global_cols = st.cfg.global_cols;
    b.plan_perm = in.plan_perm;
    b.plan_pos_slot = in.plan_pos_slot;
    b.n_planned = in.n_planned;
    b.words = unit_words(st, unit);
    b.pool = st.cfg.pool;
    b.pool_len = st.cfg.pool_len;
    b.n_neg = st.cfg.n_neg;
    b.loss = st.cfg.loss;
    b.world = st.cfg.world;
    b.rank = st.cfg.rank;
    b.neg_rec = st.cfg.owner_rec[unit % 2];
    b.seg_count = st.cfg.owner_seg[unit % 2];
    b.scores = st.cfg.owner_scores[unit % 2];
    if (st.claim) {                       // the owner prepare claims the kept draws' list slots
        b.claim_count = st.counts[unit % 2];
        b.claim_num_users = st.cfg.tables[0].num_users;
    }
    return b;
}

// the owner step's scratch for `unit` (claimed slots: that unit's count array)
rg_mf_work_t owner_work(const Stepper &st, const rg_mf_step_in_t &in, int64_t unit) {
    rg_mf_work_t w = work_for(st, in);
    if (st.claim) w.row_count = st.counts[unit % 2];
    return w;
}

int owner_check_in(const Stepper &st, const rg_mf_step_in_t &in) {
    if (!in.plan_perm || !in.plan_pos_slot || !in.plan_item_slot_off)
        return rg::fail_arg("owner-sharded step: every step input needs this rank's plan (rg_mf_plans_build, owner filter)");
    if (in.n_pos > st.cfg.global_cols || in.n_planned < 0 || in.n_planned > in.n_pos || in.global_pos != in.n_pos)
        return rg::fail_arg("owner-sharded step: n_pos / n_planned / global_pos inconsistent with the global batch");
    return RG_OK;
}

// part 1: this unit's owner prepare (unless the previous dense pass prepared it) and the
// scores of this rank's pairs into the zeroed global score vector
int owner_begin(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur) {
    int rc = owner_check_in(st, cur);
    if (rc) return rc;
    const int64_t unit = st.taken;
    if ((rc = keep_ahead(st, unit))) return rc;
    const rg_mf_owner_batch_t b = owner_batch(st, cur, unit);
    if (!(st.prepared && st.prep_unit == unit && same_input(st.prep_in, cur))) {
        if ((rc = wait_words(st, s, unit))) return rc;
        if ((rc = clean_counts(st, s, (int)(unit % 2)))) return rc;
        if ((rc = rg_mf_owner_prepare(s, &b))) return rc;
        st.count_dirty[unit % 2] = st.claim;
    }
    st.prepared = false;
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    if ((rc = rg_mf_owner_scores(s, tb, &b))) return rc;
    if ((rc = release(st, s))) return rc;               // the unit's words were read by its prepare
    st.own_in = cur;
    st.own_unit = unit;
    st.own_stage = 1;
    return RG_OK;
}

// the owner step with a sharded item update (dp_mode 2, shard_items > 0, a communicator of more than
// one rank): the item gradient in rank-major chunks -> reduce-scatter -> this rank's 1/R of the
// items' optimizer update -> all-gather of the updated item rows and biases (the same wire bytes as
// the all-reduce, 1/R of the update work)
bool item_sharded(const Stepper &st) {
    return st.cfg.dp_mode == 2 && st.cfg.shard_items > 0 && st.cfg.comm != nullptr && st.cfg.world > 1;
}

// part 2a (after the score exchange): dL/dz and the contribution lists (after_back: recorded
// after them -- the user rows' lists are complete, their update need not wait for the items')
int owner_backward(Stepper &st, hipStream_t s, hipEvent_t after_back = nullptr) {
    if (st.own_stage != 1) return rg::fail_arg("rg_mf_stepper_owner_mid: owner_begin must come first");
    const rg_mf_owner_batch_t b = owner_batch(st, st.own_in, st.own_unit);
    rg_mf_work_t w = owner_work(st, st.own_in, st.own_unit);
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    int rc = RG_OK;
    if (st.cfg.loss == RG_LOSS_ADAPTIVE_HINGE && (rc = rg_mf_owner_adapt(s, &b))) return rc;   // global max, count
    if ((rc = rg_mf_owner_back(s, tb, &b, &w))) return rc;
    if (after_back) {
        const hipError_t e = hipEventRecord(after_back, s);
        if (e != hipSuccess) return hip_fail("stepper: record the backward", e);
    }
    st.own_stage = 3;
    return RG_OK;
}

// part 2b: the item rows' data gradient (grad_stream: where it runs, ordered after the backward on s)
int owner_item_grad(Stepper &st, hipStream_t s, float *loss_out, hipStream_t grad_stream = nullptr) {
    if (st.own_stage != 3) return rg::fail_arg("rg_mf_stepper_owner_mid: the backward must come first");
    rg_mf_work_t w = owner_work(st, st.own_in, st.own_unit);
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    int rc = RG_OK;
    if (grad_stream && grad_stream != s) {
        hipError_t e = hipSuccess;
        if (!st.own_back) e = hipEventCreateWithFlags(&st.own_back, hipEventDisableTiming | hipEventDisableSystemFence);
        if (e == hipSuccess) e = hipEventRecord(st.own_back, s);
        if (e == hipSuccess) e = hipStreamWaitEvent(grad_stream, st.own_back, 0);
        if (e != hipSuccess) return hip_fail("stepper: order the item gradient", e);
        s = grad_stream;
    }
    rg_mf_loss_t l = loss_of(st, st.own_in.global_pos, loss_out);
    l.n_partials = rg_mf_owner_partials_used(st.cfg.global_cols, st.cfg.n_neg, tb->dim, st.cfg.world,
                                             st.own_in.n_planned) / 2;
    const int64_t U = tb->num_users, R = U + tb->num_items;
    if (item_sharded(st)) rc = rg_mf_grads_item_shard(s, tb, &w, st.cfg.item_grad, st.cfg.shard_items, st.cfg.world, &l);
    else rc = rg_mf_grads(s, tb, &w, st.cfg.item_grad, U, R, &l);
    if (rc) return rc;
    st.own_stage = 2;
    return RG_OK;
}

// part 2 (the caller-run exchange API): 2a then 2b
int owner_mid(Stepper &st, hipStream_t s, float *loss_out, hipStream_t grad_stream = nullptr) {
    const int rc = owner_backward(st, s);
    return rc ? rc : owner_item_grad(st, s, loss_out, grad_stream);
}

// part 3 (after the item-gradient exchange, or beside it on the communicator stream): the
// user rows' update with the next unit's owner prepare in the same launch, the items
int owner_user_update(Stepper &st, hipStream_t s, const rg_mf_step_in_t *next, const rg_opt_t &o) {
    int rc = RG_OK;
    rg_mf_owner_batch_t nb{};
    const int64_t unit = st.own_unit;
    if (next) {
        if ((rc = owner_check_in(st, *next))) return rc;
        if ((rc = keep_ahead(st, unit + 1))) return rc;
        if ((rc = wait_words(st, s, unit + 1))) return rc;
        if ((rc = clean_counts(st, s, (int)((unit + 1) % 2)))) return rc;
        nb = owner_batch(st, *next, unit + 1);
    }
    rg_mf_work_t w = owner_work(st, st.own_in, unit);
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    if ((rc = rg::apply_prepare_owner(s, tb, &w, &o, 0, tb->num_users, nullptr, next ? &nb : nullptr))) return rc;
    st.count_dirty[unit % 2] = false;     // the item gradient and this pass consumed (reset) its claims
    if (next) {
        st.count_dirty[(unit + 1) % 2] = st.claim;
        st.prepared = true;
        st.prep_unit = unit + 1;
        st.prep_in = *next;
        st.prep_serial = 0;
    }
    return RG_OK;
}

int owner_item_update(Stepper &st, hipStream_t s, const rg_opt_t &o, float *loss_out) {
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    const int64_t U = tb->num_users, R = U + tb->num_items;
    int rc;
    if (item_sharded(st)) {
        const int64_t si = st.cfg.shard_items;
        rc = rg_mf_apply_item_shard(s, tb, st.cfg.item_grad, &o, si, st.cfg.world, st.cfg.rank, loss_out);
        if (rc) return rc;
        float *bufs[2] = {tb->item_w_out, tb->item_b_out};
        const int64_t counts[2] = {si * (int64_t)tb->dim, si};
        rc = rg::comm_allgather(st.cfg.comm, s, 2, bufs, counts);
    } else {
        rc = rg_mf_apply_dense(s, tb, st.cfg.item_grad, &o, U, R, loss_out);
    }
    if (rc) return rc;
    st.set = 1 - st.set;
    st.own_stage = 0;
    return RG_OK;
}

// the whole owner-sharded step with the communicator.  The critical path stays on the
// caller's stream s with the collectives enqueued on s itself (no cross-stream hop):
//   s: scores -> score all-reduce (not for pointwise: no pairing) -> backward -> item
//      gradient -> item-gradient all-reduce -> item update -> [wait for the user update]
//   u: (after the item gradient) the user update + the next step's owner prepare
// The user update (communicator stream u) runs beside the item-gradient exchange.
int train_owner(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur, const rg_mf_step_in_t *next, float *loss_out,
                void *ev0, void *ev1) {
    int rc = owner_begin(st, s, cur);
    if (rc) return rc;
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    if (st.cfg.loss != RG_LOSS_POINTWISE) {
        const int64_t len = (int64_t)(1 + st.cfg.n_neg) * st.cfg.global_cols;
        if ((rc = rg::comm_allreduce_on(st.cfg.comm, s, st.cfg.owner_scores[st.own_unit % 2], len))) return rc;
    }
    // one rank: nothing to overlap (the exchanges are no-ops), so no cross-stream hops
    const bool side = st.cfg.world > 1;
    hipStream_t u = side ? rg::comm_stream(st.cfg.comm) : s;
    hipError_t e = hipSuccess;
    if (side) {
        // same-device ordering only: no system-scope fence (a cache write-back at every marker)
        const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
        if (!st.own_grads) e = hipEventCreateWithFlags(&st.own_grads, evf);
        if (e == hipSuccess && !st.own_users) e = hipEventCreateWithFlags(&st.own_users, evf);
        if (e != hipSuccess) return hip_fail("stepper: owner events", e);
    }
    // the user update (it touches user rows; the item pull, the item exchange and the item update
    // touch item rows) runs on the communicator stream from the point RG_OWNER_USER_AFTER names:
    // 0 the end of the backward (its lists are complete there), 1 the end of the item pull (the
    // pull then has the GPU alone), 2 the item exchange's enqueue -- measured, emulated rank 0 of
    // 8: 74.0-74.7 / 85.5-85.7 / 88.6-92.0 us per step (profiles/r5/owner/emul_order_r5x.txt).
    // It is enqueued as soon as that point is: behind the host's later launches it starts late
    static const int after = ab_int("RG_OWNER_USER_AFTER", RG_OWNER_USER_AFTER_DEFAULT);
    const rg_opt_t o = opt_at(st, st.cfg.step + 1);
    auto start_users = [&]() -> int {
        if (!side) return RG_OK;
        hipError_t e2 = hipEventRecord(st.own_grads, s);
        if (e2 == hipSuccess) e2 = hipStreamWaitEvent(u, st.own_grads, 0);
        if (e2 != hipSuccess) return hip_fail("stepper: order the user update", e2);
        int r2 = record(ev0, u);
        if (r2 == RG_OK) r2 = owner_user_update(st, u, next, o);
        if (r2 == RG_OK) r2 = record(ev1, u);
        if (r2 == RG_OK && (e2 = hipEventRecord(st.own_users, u)) != hipSuccess)
            r2 = hip_fail("stepper: record the user update", e2);
        return r2;
    };
    if ((rc = owner_backward(st, s))) return rc;
    if (after == 0 && (rc = start_users())) return rc;
    if ((rc = owner_item_grad(st, s, loss_out))) return rc;
    if (after == 1 && (rc = start_users())) return rc;
    if (item_sharded(st))
        rc = rg::comm_reduce_scatter(st.cfg.comm, s, st.cfg.item_grad, rg_mf_item_grad_chunk(st.cfg.shard_items, tb->dim));
    else
        rc = rg::comm_allreduce_on(st.cfg.comm, s, st.cfg.item_grad, tb->num_items * (int64_t)(tb->dim + 1) + 1);
    if (rc) return rc;
    if (after >= 2 && (rc = start_users())) return rc;
    st.cfg.step += 1;
    if (!side) {
        if ((rc = record(ev0, u))) return rc;
        if ((rc = owner_user_update(st, u, next, o))) return rc;
        if ((rc = record(ev1, u))) return rc;
    }
    if ((rc = owner_item_update(st, s, o, loss_out))) return rc;
    if (side && (e = hipStreamWaitEvent(s, st.own_users, 0)) != hipSuccess)
        return hip_fail("stepper: wait the user update", e);
    return RG_OK;
}

// the touched rows of the hot pass: a stamp scan (RG_HOT_SCAN=1, default) or the owner flags
const rg_mf_mark_t *hot_mark(const Stepper &st, const rg_mf_mark_t &m) { return st.hot_scan ? &m : nullptr; }

int train_fused(Stepper &st, hipStream_t s, const rg_mf_step_in_t &cur, const rg_mf_step_in_t *next,
                float *loss_out, void *ev0, void *ev1) {
    int rc = ensure_stamps(st);
    if (rc) return rc;
    const int64_t unit = st.taken;
    if ((rc = keep_ahead(st, unit))) return rc;
    rg_mf_work_t w = work_for(st, cur);
    const rg_mf_batch_t batch = make_batch(st, cur, unit);
    if (!(st.prepared && st.prep_unit == unit && st.prep_serial != 0 && same_input(st.prep_in, cur))) {
        // first step, or the prefetched pairs were for another input: marked prepare here
        if ((rc = wait_side(st, s, (int)(unit % 2)))) return rc;
        if ((rc = wait_words(st, s, unit))) return rc;
        st.prep_arr = 1 - st.prep_arr;
        st.prep_serial = next_serial(st);
        const rg_mf_mark_t m = mark_of(st, st.prep_arr, st.prep_serial);
        if ((rc = rg_mf_prepare_marked(s, &batch, &w, &m))) return rc;
        st.prepared = true;
        st.prep_unit = unit;
        st.prep_in = cur;
    }
    const rg_mf_mark_t cur_mark = mark_of(st, st.prep_arr, st.prep_serial);
    const rg_mf_tables_t *tb = &st.cfg.tables[st.set];
    const int64_t U = tb->num_users, R = tb->num_users + tb->num_items;
    const int64_t cold_end = st.cfg.item_grad ? U : R;    // DP: items go through the exchange
    st.cfg.step += 1;
    const rg_opt_t o = opt_at(st, st.cfg.step);
    const rg_mf_loss_t l = loss_of(st, cur.global_pos, loss_out);

    rg_mf_batch_t nbatch{};
    rg_mf_work_t nw{};
    rg_mf_mark_t nmark{};
    const int narr = 1 - st.prep_arr;
    if (next) {
        if ((rc = keep_ahead(st, unit + 1))) return rc;
        if ((rc = wait_side(st, s, (int)((unit + 1) % 2)))) return rc;
        if ((rc = wait_words(st, s, unit + 1))) return rc;
        nbatch = make_batch(st, *next, unit + 1);
        nw = work_for(st, *next);
        nmark = mark_of(st, narr, next_serial(st));
    }
    if ((rc = record(ev0, s))) return rc;
    if ((rc = rg_mf_step_front(s, tb, &batch, &w, &cur_mark, &o, 0, cold_end, next ? &nbatch : nullptr,
                               next ? &nw : nullptr, next ? &nmark : nullptr)))
        return rc;
    if ((rc = release(st, s))) return rc;               // clears `prepared` for this unit
    if (next) {
        st.prepared = true;
        st.prep_unit = unit + 1;
        st.prep_in = *next;
        st.prep_serial = nmark.serial;
        st.prep_arr = narr;
    }
    if (st.cfg.item_grad) {
        if ((rc = rg_mf_grads(s, tb, &w, st.cfg.item_grad, U, R, &l))) return rc;
        if (st.cfg.comm && (rc = rg::comm_begin(st.cfg.comm, s, st.cfg.item_grad,
                                                tb->num_items * (int64_t)(tb->dim + 1) + 1)))
            return rc;
        if ((rc = rg_mf_step_hot(s, tb, &batch, &w, hot_mark(st, cur_mark), &o, 0, U, nullptr))) return rc;
        if ((rc = record(ev1, s))) return rc;
        if (st.cfg.comm && (rc = rg::comm_end(st.cfg.comm, s))) return rc;
        if ((rc = rg_mf_apply_dense(s, tb, st.cfg.item_grad, &o, U, R, loss_out))) return rc;
    } else {
        if ((rc = rg_mf_step_hot(s, tb, &batch, &w, hot_mark(st, cur_mark), &o, 0, R, &l))) return rc;
        if ((rc = record(ev1, s))) return rc;
    }
    st.set = 1 - st.set;
    return RG_OK;
}

void destroy(Stepper *st) {
    if (st->gen) hipStreamSynchronize(st->gen);
    if (st->prep) hipStreamSynchronize(st->prep);
    hipDeviceSynchronize();
    for (int i = 0; i < kSlots; ++i) {
        if (st->gen_done[i]) hipEventDestroy(st->gen_done[i]);
        if (st->consumed[i]) hipEventDestroy(st->consumed[i]);
        if (st->words[i]) hipFree(st->words[i]);
        if (st->start_state[i]) hipFree(st->start_state[i]);
    }
    for (int i = 0; i < 2; ++i) {
        if (st->ready[i]) hipEventDestroy(st->ready[i]);
        if (st->stamp[i]) hipFree(st->stamp[i]);
    }
    if (st->mark) hipEventDestroy(st->mark);
    if (st->last_rel) hipFree(st->last_rel);
    if (st->umark) hipFree(st->umark);
    if (st->consts) hipFree(st->consts);
    if (st->rows_done) hipFree(st->rows_done);
    if (st->own_counts) hipFree(st->own_counts);
    for (void *p : {(void *)st->p_counts2, (void *)st->p_list1, (void *)st->p_hg1, (void *)st->p_hbg1,
                    (void *)st->p_part1, (void *)st->p_prow1, (void *)st->p_pbias1, (void *)st->hot[0],
                    (void *)st->hot[1], (void *)st->hot[2], (void *)st->pint})
        if (p) hipFree(p);
    if (st->own_back) hipEventDestroy(st->own_back);
    if (st->own_grads) hipEventDestroy(st->own_grads);
    if (st->own_users) hipEventDestroy(st->own_users);
    if (st->gen) hipStreamDestroy(st->gen);
    if (st->prep) hipStreamDestroy(st->prep);
    rg::mt_jump_plan_destroy(st->jump);
    rg::mt_jump_plan_destroy(st->slice_plan);
    rg::mt_jump_plan_destroy(st->gjump);
    rg::mt_jump_plan_destroy(st->rjump);
    if (st->gstate) hipFree(st->gstate);
    if (st->jscratch) hipFree(st->jscratch);
    delete st;
}

}  // namespace

extern "C" void *rg_mf_stepper_create(const rg_mf_stepper_config_t *cfg) {
    if (!cfg) { rg::set_error("rg_mf_stepper_create: null config"); return nullptr; }
    if (!cfg->mt_state || !cfg->pairs[0] || !cfg->pairs[1]) {
        rg::set_error("rg_mf_stepper_create: null sampler buffers");
        return nullptr;
    }
    if (cfg->dp_mode == 2) {
        const int64_t segs = rg_mf_owner_segments(cfg->global_cols, cfg->n_neg);
        if (cfg->world < 1 || cfg->rank < 0 || cfg->rank >= cfg->world || !cfg->item_grad ||
            cfg->cols != cfg->global_cols || cfg->col_offset != 0 || segs <= 0 || !cfg->owner_rec[0] || !cfg->owner_rec[1] ||
            !cfg->owner_seg[0] || !cfg->owner_seg[1] || !cfg->owner_scores[0] || !cfg->owner_scores[1] ||
            cfg->shard_items < 0 || (cfg->shard_items > 0 && cfg->shard_items * cfg->world < cfg->tables[0].num_items)) {
            rg::set_error("rg_mf_stepper_create: inconsistent owner-sharded data-parallel configuration");
            return nullptr;
        }
    }
    if (cfg->dp_mode == 1) {
        const rg_mf_tables_t &t = cfg->tables[0];
        if (cfg->world < 1 || cfg->rank < 0 || cfg->rank >= cfg->world || !cfg->grad_buf ||
            cfg->shard_users * cfg->world < t.num_users || cfg->shard_items * cfg->world < t.num_items ||
            cfg->global_cols != cfg->cols * cfg->world || cfg->col_offset != cfg->rank * cfg->cols || cfg->item_grad ||
            cfg->loss == RG_LOSS_ADAPTIVE_HINGE) {
            rg::set_error("rg_mf_stepper_create: inconsistent replicated data-parallel configuration");
            return nullptr;
        }
    }
    Stepper *st = new (std::nothrow) Stepper();
    if (!st) { rg::set_error("rg_mf_stepper_create: out of memory"); return nullptr; }
    st->cfg = *cfg;
    st->set = cfg->current_set;
    st->W = 2 * (int64_t)cfg->n_neg * cfg->global_cols;
    if (st->cfg.neg_cols <= 0) st->cfg.neg_cols = cfg->global_cols;
    st->fused = ab_flag("RG_FUSED", false);
    {
        // inline walk (default): one unit per slot, walked inside the dense pass two steps
        // ahead, when the walk (~0.47 ns/word on one workgroup) hides under that pass
        // (~5 TB/s over p, m, v of every row); otherwise 8-unit slots on the gen stream
        const rg_mf_tables_t &t = cfg->tables[0];
        const double walk_us = 0.47e-3 * (double)st->W;
        const double dense_us = 6.0 * (double)(t.num_users + t.num_items) * (4.0 * t.dim + 4.0) / 5.0e6;
        // RG_MT_INLINE: 0 off, 1 (default) when it hides, 2 always (tests at small sizes)
        const char *im = getenv("RG_MT_INLINE");
        const int mode = im ? atoi(im) : 1;
        // gen_mode 2: the consumer's tail launch walks (rg_mf_stepper_tail_gen), under the same test;
        // 3: the same, the caller having made the test against a pass these tables do not show
        // (NeuMF's GMF tables)
        st->inline_gen = mode != 0 && !st->fused && !env_flag("RG_MT_JUMP", false) && !cfg->item_grad &&
                         (cfg->gen_mode == 0 || cfg->gen_mode >= 2 || mode == 2) &&
                         cfg->dp_mode == 0 && (mode == 2 || cfg->gen_mode == 3 || walk_us <= 0.85 * dense_us);
        const char *g = getenv("RG_MT_UNITS");
        st->G = st->inline_gen ? 1 : (g ? atoi(g) : 8);
        if (st->G < 1) st->G = 1;
        if (st->G > 64) st->G = 64;
    }
    st->hot_scan = ab_flag("RG_HOT_SCAN", true);
    // separate priorities keep the streams on separate hardware queues: the walk is
    // background work (lowest), the short side prepare is on the step's path (highest)
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    const int prio_mode = ab_int("RG_STREAM_PRIO", 1);
    if (e == hipSuccess)
        e = hipStreamCreateWithPriority(&st->gen, hipStreamNonBlocking, prio_mode ? least : 0);
    if (e == hipSuccess)
        e = hipStreamCreateWithPriority(&st->prep, hipStreamNonBlocking, prio_mode ? greatest : 0);
    // the events only order streams of this device: no system-scope fence (which
    // writes back and invalidates caches at every marker, ~7 us of idle per packet)
    const int ev_mode = ab_int("RG_EVENT_MODE", 1);
    const unsigned evf = hipEventDisableTiming | (ev_mode == 1 ? hipEventDisableSystemFence
                                                 : ev_mode == 2 ? hipEventReleaseToDevice : 0u);
    const size_t slot_words = (size_t)(st->G * st->W + RG_MT_PAD);
    for (int i = 0; e == hipSuccess && i < kSlots; ++i) {
        e = hipEventCreateWithFlags(&st->gen_done[i], evf);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&st->consumed[i], evf);
        if (e == hipSuccess) e = hipMalloc(&st->words[i], slot_words * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc(&st->start_state[i], 625 * sizeof(uint32_t));
    }
    for (int i = 0; e == hipSuccess && i < 2; ++i) e = hipEventCreateWithFlags(&st->ready[i], evf);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&st->mark, evf);
    uint32_t pos = 624;
    if (e == hipSuccess) e = hipMemcpy(&pos, cfg->mt_state + 624, sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        hip_fail("rg_mf_stepper_create", e);
        destroy(st);
        return nullptr;
    }
    st->cp_pos = (int32_t)pos;
    // lazy dense pass (opt-in, RG_LAZY=1): the single-rank split step.  Bit-exact with the
    // eager pass but measured slower on gfx950 (the catch-up is ALU-bound).
    st->lazy = ab_flag("RG_LAZY", false) && cfg->dp_mode == 0 && !cfg->item_grad && !st->fused;
    if (st->lazy) {
        const size_t ub = (size_t)cfg->tables[0].num_users * sizeof(int32_t);
        e = hipMalloc(&st->last_rel, ub);
        if (e == hipSuccess) e = hipMalloc(&st->umark, ub);
        if (e == hipSuccess) e = hipMemset(st->umark, 0, ub);
        if (e == hipSuccess) e = hipMemset(st->last_rel, 0, ub);
        if (e == hipSuccess) e = hipMalloc(&st->rows_done, sizeof(uint64_t));
        if (e == hipSuccess) e = hipMemset(st->rows_done, 0, sizeof(uint64_t));
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            hip_fail("rg_mf_stepper_create: lazy state", e);
            destroy(st);
            return nullptr;
        }
        st->lazy_base = cfg->step;
    }
    // claimed list slots: the single-rank eager split step (RG_MF_CLAIM=0: the pair pass
    // claims its slots with returning atomics, as before)
    const rg_mf_tables_t &t0 = cfg->tables[0];
    // (the owner-sharded step claims in its owner prepare, records keep the slots beside the ids)
    st->claim = ab_flag("RG_MF_CLAIM", true) && !cfg->item_grad && !st->fused && !st->lazy &&
                cfg->loss != RG_LOSS_ADAPTIVE_HINGE && cfg->work.row_count != nullptr &&
                (cfg->dp_mode == 2 ||
                 (cfg->dp_mode == 0 && t0.num_users < ((int64_t)1 << 27) && t0.num_items < ((int64_t)1 << 27)));
    if (st->claim) {
        const size_t cb = (size_t)(t0.num_users + t0.num_items) * sizeof(int32_t);
        e = hipMalloc(&st->own_counts, cb);
        if (e == hipSuccess) e = hipMemset(st->own_counts, 0, cb);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            hip_fail("rg_mf_stepper_create: claimed counts", e);
            destroy(st);
            return nullptr;
        }
        st->counts[0] = cfg->work.row_count;
        st->counts[1] = st->own_counts;
    }
    st->prep_in_pairs = ab_flag("RG_PREP_IN_PAIRS", false);
    // pipelined step (rg_mf_pipe_step): single rank, claimed slots, pointwise / bpr / hinge, a
    // float4 row layout of >= 8 lanes (dim a multiple of 4, 32..256)
    st->pipe = ab_flag("RG_PIPE", RG_PIPE_DEFAULT) && st->claim && cfg->dp_mode == 0 && !st->prep_in_pairs &&
               (cfg->loss == RG_LOSS_POINTWISE || cfg->loss == RG_LOSS_BPR || cfg->loss == RG_LOSS_HINGE) &&
               t0.dim % 4 == 0 && t0.dim >= 32 && t0.dim <= 256 && cfg->work.part_row && cfg->work.part_bias &&
               cfg->work.loss_partials && cfg->n_partials > 0;
    if (st->pipe) {
        // the pair workgroups wait inside the launch: keep them at most half of what the chip
        // holds (>= 4 workgroups per CU at the launch's register count), so the rows they wait
        // for always have room to run whatever the dispatch order
        const int64_t upb = rg_mf_plan_units_per_block(t0.dim);
        st->pipe = upb > 0 && (cfg->cols + upb - 1) / upb <= 2 * (int64_t)rg::num_cus() &&
                   std::max(t0.num_users, t0.num_items) * (int64_t)t0.dim * 4 < ((int64_t)1 << 31);
    }
    // two-launch pipelined step (rg_mf_pipe2_hot / _cold) for the single-rank losses with claimed
    // slots: RG_PIPE2=1 selects it, RG_PIPE2_DEFAULT the build's default (0: the split step, which
    // measures faster -- DESIGN §4.1)
    st->pipe2 = !st->pipe && ab_flag("RG_PIPE2", RG_PIPE2_DEFAULT != 0) && st->claim && cfg->dp_mode == 0 && !st->prep_in_pairs &&
                (cfg->loss == RG_LOSS_POINTWISE || cfg->loss == RG_LOSS_BPR || cfg->loss == RG_LOSS_HINGE) &&
                cfg->work.part_row && cfg->work.part_bias && cfg->work.loss_partials && cfg->n_partials > 0;
    if (st->pipe || st->pipe2) {
        const int64_t rows = t0.num_users + t0.num_items;
        const int64_t hot_len = std::min<int64_t>(t0.num_users, (int64_t)(1 + cfg->n_neg) * cfg->cols);
        e = hipMalloc(&st->p_counts2, (size_t)rows * sizeof(int32_t));
        if (e == hipSuccess) e = hipMemset(st->p_counts2, 0, (size_t)rows * sizeof(int32_t));
        if (e == hipSuccess) e = hipMalloc(&st->p_list1, (size_t)rows * RG_MF_LIST_CAP * 2 * sizeof(int32_t));
        if (e == hipSuccess) e = hipMalloc(&st->p_hg1, (size_t)rows * t0.dim * sizeof(int64_t));
        if (e == hipSuccess) e = hipMemset(st->p_hg1, 0, (size_t)rows * t0.dim * sizeof(int64_t));
        if (e == hipSuccess) e = hipMalloc(&st->p_hbg1, (size_t)rows * sizeof(int64_t));
        if (e == hipSuccess) e = hipMemset(st->p_hbg1, 0, (size_t)rows * sizeof(int64_t));
        if (e == hipSuccess) e = hipMalloc(&st->p_part1, (size_t)cfg->n_partials * 2 * sizeof(float));
        if (e == hipSuccess) e = hipMalloc(&st->p_prow1, (size_t)cfg->cols * t0.dim * sizeof(float));
        if (e == hipSuccess) e = hipMalloc(&st->p_pbias1, (size_t)cfg->cols * sizeof(float));
        for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipMalloc(&st->hot[k], (size_t)hot_len * sizeof(int32_t));
        if (e == hipSuccess) e = hipMalloc(&st->pint, 8 * sizeof(int32_t));
        if (e == hipSuccess) e = hipMemset(st->pint, 0, 8 * sizeof(int32_t));
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            hip_fail("rg_mf_stepper_create: pipelined step buffers", e);
            destroy(st);
            return nullptr;
        }
        st->pcounts[0] = st->counts[0];
        st->pcounts[1] = st->counts[1];
        st->pcounts[2] = st->p_counts2;
    }
    // the jump-ahead walk (parallel segments) by default when every rank walks the global
    // stream of a multi-rank step: R times the words of one GPU's step
    if (cfg->dp_mode == 2 && cfg->comm && cfg->world > 1 && st->W % cfg->world == 0 && !st->inline_gen &&
        st->G < rg::kMtMaxTail &&
        ab_flag("RG_OWNER_MT_SLICE", false)) {
        // each rank walks its slice of the global draw (see Stepper::slice); falls back to the
        // jump-ahead walk of the whole draw when a slice is shorter than a jump's stream window
        st->L = st->W / cfg->world;
        st->slice_plan = rg::mt_slice_plan_create(st->W, st->L, st->G);
        st->gjump = rg::mt_jump_plan_create(st->G * st->W, 0);
        if (cfg->rank > 0) st->rjump = rg::mt_jump_plan_create((int64_t)cfg->rank * st->L, 0);
        st->slice = st->slice_plan && st->gjump && (cfg->rank == 0 || st->rjump) && st->L >= st->slice_plan->head;
        if (st->slice) {
            const size_t scratch = (size_t)(st->slice_plan->head + 2 * 227 + RG_MT_PAD);
            e = hipMalloc(&st->gstate, 625 * sizeof(uint32_t));
            if (e == hipSuccess) e = hipMalloc(&st->jscratch, scratch * sizeof(uint32_t));
            if (e == hipSuccess) e = hipMemcpy(st->gstate, cfg->mt_state, 625 * sizeof(uint32_t), hipMemcpyDeviceToDevice);
            int rc = e == hipSuccess ? rg::comm_words_prepare(cfg->comm) : RG_E_LAUNCH;
            if (e != hipSuccess) hip_fail("rg_mf_stepper_create: slice state", e);
            if (rc == RG_OK) rc = slice_reset(*st);
            if (rc == RG_OK && (e = hipStreamSynchronize(st->gen)) != hipSuccess) rc = hip_fail("rg_mf_stepper_create", e);
            if (rc != RG_OK) {
                destroy(st);
                return nullptr;
            }
        } else {
            rg::mt_jump_plan_destroy(st->slice_plan);
            rg::mt_jump_plan_destroy(st->gjump);
            rg::mt_jump_plan_destroy(st->rjump);
            st->slice_plan = st->gjump = st->rjump = nullptr;
        }
    }
    if (!st->slice && env_flag("RG_MT_JUMP", cfg->dp_mode != 0 && cfg->world > 1))
        st->jump = rg::mt_jump_plan_create(st->G * st->W);
    return st;
}

extern "C" int32_t rg_mf_stepper_mt_mode(void *h) {
    const Stepper *st = static_cast<const Stepper *>(h);
    if (!st) return -1;
    return st->slice ? 2 : st->jump ? 1 : 0;
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
    if (st->failed) return rg::fail_arg("rg_mf_stepper_train: an earlier step stopped half applied; rebuild the stepper");
    hipStream_t s = (hipStream_t)stream;
    if (st->cfg.dp_mode == 1) {
        if (!st->cfg.comm) return rg::fail_arg("rg_mf_stepper_train: replicated DP step needs a communicator "
                                               "(or rg_mf_stepper_dp_begin / _dp_end around the caller's exchange)");
        return train_dp(*st, s, *cur, next, loss_out, ev_apply_begin, ev_apply_end);
    }
    if (st->cfg.dp_mode == 2) {
        if (!st->cfg.comm) return rg::fail_arg("rg_mf_stepper_train: owner-sharded DP step needs a communicator "
                                               "(or rg_mf_stepper_owner_begin / _mid / _end around the exchanges)");
        return train_owner(*st, s, *cur, next, loss_out, ev_apply_begin, ev_apply_end);
    }
    if (st->pipe) return train_pipe(*st, s, *cur, next, nullptr, loss_out, ev_apply_begin, ev_apply_end);
    if (st->pipe2) return train_pipe2(*st, s, *cur, next, nullptr, loss_out, ev_apply_begin, ev_apply_end);
    if (st->fused && st->cfg.loss != RG_LOSS_ADAPTIVE_HINGE)
        return train_fused(*st, s, *cur, next, loss_out, ev_apply_begin, ev_apply_end);
    if (st->lazy) return train_lazy(*st, s, *cur, next, loss_out, ev_apply_begin, ev_apply_end);
    return train_split(*st, s, *cur, next, loss_out, ev_apply_begin, ev_apply_end);
}

extern "C" int rg_mf_stepper_train_ahead(void *h, void *stream, const rg_mf_step_in_t *cur,
                                         const rg_mf_step_in_t *next, const rg_mf_step_in_t *next2, float *loss_out,
                                         void *ev_apply_begin, void *ev_apply_end) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur) return rg::fail_arg("rg_mf_stepper_train_ahead: null handle/input");
    if (!next && next2) return rg::fail_arg("rg_mf_stepper_train_ahead: next2 without next");
    if (st->pipe) return train_pipe(*st, (hipStream_t)stream, *cur, next, next2, loss_out, ev_apply_begin, ev_apply_end);
    if (st->pipe2 && st->cfg.dp_mode == 0)
        return train_pipe2(*st, (hipStream_t)stream, *cur, next, next2, loss_out, ev_apply_begin, ev_apply_end);
    return rg_mf_stepper_train(h, stream, cur, next, loss_out, ev_apply_begin, ev_apply_end);
}

extern "C" int rg_mf_stepper_pipelined(void *h) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_pipelined: null handle");
    return st->pipe ? 1 : st->pipe2 ? 2 : 0;
}

extern "C" int rg_mf_stepper_pipe_error(void *h, int32_t *err_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !err_out) return rg::fail_arg("rg_mf_stepper_pipe_error: null argument");
    *err_out = 0;
    if (!st->pipe) return RG_OK;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(err_out, st->pint + 5, sizeof(int32_t), hipMemcpyDeviceToHost);
    return e == hipSuccess ? RG_OK : hip_fail("rg_mf_stepper_pipe_error", e);
}

extern "C" int rg_mf_stepper_dp_begin(void *h, void *stream, const rg_mf_step_in_t *cur, const rg_mf_step_in_t *next,
                                      float *loss_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur) return rg::fail_arg("rg_mf_stepper_dp_begin: null handle/input");
    if (st->cfg.dp_mode != 1) return rg::fail_arg("rg_mf_stepper_dp_begin: stepper is not in dp_mode 1");
    return dp_begin(*st, (hipStream_t)stream, *cur, next, loss_out, nullptr, nullptr);
}

extern "C" int rg_mf_stepper_dp_end(void *h, void *stream, float *loss_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_dp_end: null handle");
    if (st->cfg.dp_mode != 1) return rg::fail_arg("rg_mf_stepper_dp_end: stepper is not in dp_mode 1");
    return dp_end(*st, (hipStream_t)stream, loss_out);
}

extern "C" int rg_mf_stepper_owner_begin(void *h, void *stream, const rg_mf_step_in_t *cur) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur) return rg::fail_arg("rg_mf_stepper_owner_begin: null handle/input");
    if (st->cfg.dp_mode != 2) return rg::fail_arg("rg_mf_stepper_owner_begin: stepper is not in dp_mode 2");
    if (st->own_stage != 0) return rg::fail_arg("rg_mf_stepper_owner_begin: the previous step is not finished");
    return owner_begin(*st, (hipStream_t)stream, *cur);
}

extern "C" int rg_mf_stepper_owner_mid(void *h, void *stream, float *loss_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_owner_mid: null handle");
    if (st->cfg.dp_mode != 2) return rg::fail_arg("rg_mf_stepper_owner_mid: stepper is not in dp_mode 2");
    return owner_mid(*st, (hipStream_t)stream, loss_out);
}

extern "C" int rg_mf_stepper_owner_end(void *h, void *stream, const rg_mf_step_in_t *next, float *loss_out,
                                       void *ev0, void *ev1) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_owner_end: null handle");
    if (st->cfg.dp_mode != 2 || st->own_stage != 2)
        return rg::fail_arg("rg_mf_stepper_owner_end: needs dp_mode 2 after owner_mid");
    hipStream_t s = (hipStream_t)stream;
    st->cfg.step += 1;
    const rg_opt_t o = opt_at(*st, st->cfg.step);
    int rc = record(ev0, s);
    if (rc || (rc = owner_user_update(*st, s, next, o)) || (rc = record(ev1, s))) return rc;
    return owner_item_update(*st, s, o, loss_out);
}

extern "C" int rg_mf_stepper_owner_val_end(void *h, void *stream, float *loss_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !loss_out) return rg::fail_arg("rg_mf_stepper_owner_val_end: null argument");
    if (st->cfg.dp_mode != 2 || st->own_stage != 1)
        return rg::fail_arg("rg_mf_stepper_owner_val_end: needs dp_mode 2 after owner_begin");
    const rg_mf_owner_batch_t b = owner_batch(*st, st->own_in, st->own_unit);
    st->own_stage = 0;
    return rg_mf_owner_loss((hipStream_t)stream, &b, loss_out);
}

extern "C" int rg_mf_stepper_owner_val(void *h, void *stream, const rg_mf_step_in_t *cur, float *loss_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur || !loss_out) return rg::fail_arg("rg_mf_stepper_owner_val: null argument");
    if (st->cfg.dp_mode != 2 || !st->cfg.comm || st->own_stage != 0)
        return rg::fail_arg("rg_mf_stepper_owner_val: needs dp_mode 2 with a communicator, between steps");
    hipStream_t s = (hipStream_t)stream;
    int rc = owner_begin(*st, s, *cur);
    if (rc) return rc;
    const int64_t len = (int64_t)(1 + st->cfg.n_neg) * st->cfg.global_cols;
    if ((rc = rg::comm_begin(st->cfg.comm, s, st->cfg.owner_scores[st->own_unit % 2], len)) ||
        (rc = rg::comm_end(st->cfg.comm, s)))
        return rc;
    return rg_mf_stepper_owner_val_end(h, stream, loss_out);
}

extern "C" int rg_mf_stepper_owner_scores(void *h, float **scores_out, int64_t *len_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !scores_out || !len_out) return rg::fail_arg("rg_mf_stepper_owner_scores: null argument");
    if (st->cfg.dp_mode != 2 || st->own_unit < 0) return rg::fail_arg("rg_mf_stepper_owner_scores: no owner step yet");
    *scores_out = st->cfg.owner_scores[st->own_unit % 2];
    *len_out = (int64_t)(1 + st->cfg.n_neg) * st->cfg.global_cols;
    return RG_OK;
}

extern "C" int rg_mf_stepper_acquire(void *h, void *stream, const rg_mf_step_in_t *cur, rg_mf_batch_t *batch_out,
                                     rg_mf_work_t *work_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !cur || !batch_out || !work_out) return rg::fail_arg("rg_mf_stepper_acquire: null argument");
    int64_t unit;
    int rc = acquire(*st, (hipStream_t)stream, *cur, &unit);
    if (rc) return rc;
    *batch_out = make_batch(*st, *cur, unit);
    *work_out = work_for(*st, *cur);
    return RG_OK;
}

extern "C" int rg_mf_stepper_release(void *h, void *stream) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_release: null handle");
    return release(*st, (hipStream_t)stream);
}

// the pairs of the next unit (`taken`, i.e. called after the current step's release) for
// `next`, prepared now on the side stream behind the work `stream` holds so far: a split
// consumer (NCF / NeuMF) then finds them ready at its acquire instead of serialising a
// prepare between its steps.  A different input at that acquire prepares again.
extern "C" int rg_mf_stepper_prefetch(void *h, void *stream, const rg_mf_step_in_t *next) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !next) return rg::fail_arg("rg_mf_stepper_prefetch: null argument");
    if (st->prepared && st->prep_unit == st->taken && same_input(st->prep_in, *next) && !st->prep_claimed)
        return RG_OK;
    return prepare_side(*st, (hipStream_t)stream, st->taken, *next);
}

extern "C" int rg_mf_stepper_prefetch_inline(void *h, void *stream, const rg_mf_step_in_t *next) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !next) return rg::fail_arg("rg_mf_stepper_prefetch_inline: null argument");
    if (st->prepared && st->prep_unit == st->taken && same_input(st->prep_in, *next) && !st->prep_claimed)
        return RG_OK;
    return prepare_inline(*st, (hipStream_t)stream, st->taken, *next);
}

// prefetch_inline's bookkeeping without its launch: the caller launches the prepare of the
// returned batch / work on `stream` itself, inside another kernel (rg_ncf_tail).
// Returns 1 when a prepare is to be launched, 0 when the unit is already prepared.
extern "C" int rg_mf_stepper_prefetch_args(void *h, void *stream, const rg_mf_step_in_t *next,
                                           rg_mf_batch_t *batch_out, rg_mf_work_t *work_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !next || !batch_out || !work_out) return rg::fail_arg("rg_mf_stepper_prefetch_args: null argument");
    if (st->prepared && st->prep_unit == st->taken && same_input(st->prep_in, *next) && !st->prep_claimed) return 0;
    const int64_t unit = st->taken;
    hipStream_t s = (hipStream_t)stream;
    int rc = st->inline_gen ? generate_upto(*st, unit, 0) : keep_ahead(*st, unit);
    if (rc) return rc;
    const int b = (int)(unit % 2);
    if ((rc = wait_side(*st, s, b))) return rc;   // an earlier side write of this buffer
    if ((rc = wait_words(*st, s, unit))) return rc;
    *work_out = work_for(*st, *next);
    *batch_out = make_batch(*st, *next, unit);
    st->side_pending[b] = false;
    st->prepared = true;
    st->prep_unit = unit;
    st->prep_in = *next;
    st->prep_serial = 0;
    st->prep_claimed = false;
    return 1;
}

// gen_mode 2 (single-GPU NCF): the walk of unit taken + 1 -- two after the step just released --
// rides in the caller's tail launch on `stream`, as the MF split step's dense pass carries it
extern "C" int rg_mf_stepper_tail_gen(void *h, void *stream, rg_mt_gen_t *gen_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !gen_out) return rg::fail_arg("rg_mf_stepper_tail_gen: null argument");
    *gen_out = rg_mt_gen_t{};
    if (!st->inline_gen || st->cfg.gen_mode < 2 || st->gen_slots != rel_slot(*st, st->taken + 1)) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int slot = (int)(st->gen_slots % kSlots);
    int rc = begin_production(*st, s, slot);
    if (rc) return rc;
    gen_out->state = st->cfg.mt_state;
    gen_out->out = st->words[slot];
    gen_out->state_before = st->start_state[slot];
    gen_out->nwords = st->G * st->W;
    end_production(*st, s, slot);    // the caller's launch is the next work on `stream`
    return 1;
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
    if ((st->pipe || st->pipe2) && (st->paired >= 0 || st->hot_prepped >= 0))
        return rg::fail_arg("rg_mf_stepper_advance: a pipelined step is pending (acquire first)");
    if (st->lazy_pending) return rg::fail_arg("rg_mf_stepper_advance: lazy rows pending (rg_mf_stepper_flush first)");
    if (flip_sets) st->set = 1 - st->set;
    st->cfg.step += steps;
    return RG_OK;
}

extern "C" int rg_mf_stepper_sync_mt(void *h, uint32_t *host_state, int32_t direction) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st || !host_state) return rg::fail_arg("rg_mf_stepper_sync_mt: null argument");
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_fail("stepper: sync", e);
    if (direction == 0) {   // device -> host: the state after the last CONSUMED unit
        const int64_t rel = st->taken - st->unit_base;
        const int64_t slot_rel = rel / st->G, inside = rel % st->G;
        const bool ahead = st->gen_slots > slot_rel;
        const int slot = (int)(slot_rel % kSlots);
        const uint32_t *src = ahead ? st->start_state[slot] : st->slice ? st->gstate : st->cfg.mt_state;
        const bool window = ahead ? st->win_at[slot] : st->window_form;
        const int32_t pos = ahead ? st->pos_at[slot] : st->cp_pos;
        uint32_t dev[625];
        e = hipMemcpy(dev, src, 625 * sizeof(uint32_t), hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_fail("stepper: copy MT state", e);
        int rc = RG_OK;
        if (!window) std::memcpy(host_state, dev, sizeof(dev));
        else rc = rg_mt_window_to_cpython(dev, pos, host_state);
        if (rc == RG_OK && inside > 0) rc = rg_mt_advance_host(host_state, inside * st->W);
        return rc;
    }
    // host -> device: words generated ahead are dropped; unit numbering restarts here
    {
        const int rc = pipe_abandon(*st, nullptr);
        if (rc) return rc;
        e = hipDeviceSynchronize();
        if (e != hipSuccess) return hip_fail("stepper: sync", e);
    }
    st->unit_base = st->taken;
    st->gen_slots = 0;
    for (int i = 0; i < kSlots; ++i) {
        st->prod[i] = st->seen[i] = st->cons_on[i] = nullptr;
        st->gen_rec[i] = st->cons_rec[i] = st->seen_ok[i] = st->cons_ok[i] = false;
    }
    st->prepared = false;
    st->window_form = false;
    st->cp_pos = (int32_t)host_state[624];
    e = hipMemcpy(st->slice ? st->gstate : st->cfg.mt_state, host_state, 625 * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail("stepper: copy MT state", e);
    if (st->slice) {
        const int rc = slice_reset(*st);
        if (rc) return rc;
        if ((e = hipStreamSynchronize(st->gen)) != hipSuccess) return hip_fail("stepper: slice state", e);
    }
    return RG_OK;
}

extern "C" int rg_mf_stepper_flush(void *h, void *stream) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_flush: null handle");
    return lazy_flush(*st, (hipStream_t)stream);
}

extern "C" int rg_mf_stepper_lazy_count(void *h, int32_t enable, uint64_t *rows_out) {
    Stepper *st = static_cast<Stepper *>(h);
    if (!st) return rg::fail_arg("rg_mf_stepper_lazy_count: null handle");
    if (rows_out) {
        *rows_out = 0;
        if (st->rows_done) {
            hipError_t e = hipDeviceSynchronize();
            if (e == hipSuccess) e = hipMemcpy(rows_out, st->rows_done, sizeof(uint64_t), hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemset(st->rows_done, 0, sizeof(uint64_t));
            if (e != hipSuccess) return hip_fail("rg_mf_stepper_lazy_count", e);
        }
    }
    st->count_rows = enable != 0 && st->rows_done != nullptr;
    return st->lazy ? 1 : 0;
}
