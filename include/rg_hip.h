/*
 * rg_hip.h -- C-ABI of librg_hip.so, the MI355X (gfx950) hot path of the
 * recommendation_Gans embedding-training loop.
 *
 * Conventions
 *   - Every pointer named *_dev / inside the structs is a DEVICE pointer owned by
 *     the caller (PyTorch's caching allocator); the library allocates no device
 *     memory.  Host pointers are marked "host".
 *   - Every call is stream-ordered on `stream` (a hipStream_t passed as void*),
 *     never synchronises the host, and returns RG_OK (0) or a negative status;
 *     rg_last_error() then holds a thread-local message.
 *   - No torch types cross this boundary.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference checkout):
 *   rg_mt_generate      random.choices' MT19937 stream      implicit.py:352, :370
 *   rg_mf_pairs         BilinearNet.forward x2 + loss + autograd
 *                                                          implicit.py:348-361,
 *                                                          spotlight/factorization/representations.py:62-91,
 *                                                          spotlight/losses.py:20-172
 *   rg_mf_apply         optimizer.step() over every row     implicit.py:363,
 *                                                          spotlight/optimizers.py:4-22
 *   rg_mf_grads /       the same step split around an RCCL all-reduce of the
 *   rg_mf_apply_dense   gradient (data parallel; no reference counterpart)
 *   rg_mf_scores        BilinearNet.forward (eval / predict)
 *                                                          implicit.py:368, :412
 *   rg_loss_finalize    loss.item() of run_val_iteration    implicit.py:366-379
 *   rg_mf_stepper_*     the loop body of fit: one call per run_train_iteration
 *                                                          implicit.py:290-298, :347-364
 *   rg_comm_*           RCCL communicator of the user-sharded data-parallel step
 *                       (the reference is single-device)
 */
#ifndef RG_HIP_H
#define RG_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RG_OK 0
#define RG_E_ARG (-1)      /* invalid argument / unsupported shape */
#define RG_E_LAUNCH (-2)   /* HIP launch or runtime error */

/* capacity of the per-row contribution list (rows touched more often spill into
 * the overflow accumulators hot_grad / hot_bias_grad) */
#define RG_MF_LIST_CAP 8
/* maximum negatives per positive handled by the fused pair kernel */
#define RG_MF_MAX_NEG 8

enum rg_loss_kind {
    RG_LOSS_POINTWISE = 0,       /* spotlight/losses.py:20   BCE(pos,1) + BCE(neg,0) */
    RG_LOSS_BPR = 1,             /* spotlight/losses.py:59   mean(1 - sigmoid(pos - neg)), neg.view(n,B) */
    RG_LOSS_HINGE = 2,           /* spotlight/losses.py:99   mean(clamp(neg - pos + 1, 0)), neg.view(n,B) */
    RG_LOSS_ADAPTIVE_HINGE = 3,  /* spotlight/losses.py:133  hinge against max over ALL negatives */
    RG_LOSS_POINTWISE_POS = 4    /* implicit.py:359-360 (neg_examples=None): BCE(pos,1) only; the step's
                                    negatives are drawn but take no part (single-rank MF step only) */
};

enum rg_opt_kind {
    RG_OPT_ADAM = 0,   /* torch.optim.Adam, coupled L2 (optimizers.py:10-16) */
    RG_OPT_SGD = 1,    /* torch.optim.SGD, momentum 0     (optimizers.py:4-8)   */
    RG_OPT_RMSPROP = 2 /* torch.optim.RMSprop, centered=False, momentum 0 (optimizers.py:18-22) */
};

/* The four BilinearNet tables (fp32, row-major, rows contiguous) plus optimizer
 * state.  Updates are written to the *_out tables (ping-pong): the pull-style
 * gradient gather reads the pre-step rows of the OTHER table while rows are
 * being updated, so *_out must not alias the inputs. */
typedef struct rg_mf_tables {
    const float *user_w, *item_w;   /* [num_users, dim], [num_items, dim] */
    const float *user_b, *item_b;   /* [num_users], [num_items] */
    float *user_w_out, *item_w_out, *user_b_out, *item_b_out;
    float *user_w_m, *user_w_v, *item_w_m, *item_w_v;   /* Adam m/v; RMSprop uses *_v */
    float *user_b_m, *user_b_v, *item_b_m, *item_b_v;
    int64_t num_users, num_items;
    int32_t dim;                    /* 1..256 */
    int32_t pad_;
} rg_mf_tables_t;

/* One training step's positives and negatives, for the caller's rank.
 * Negative draw j (0 <= j < n_neg * global_cols) belongs to column j % global_cols
 * and negative slot j / global_cols (the reference's flat draw order viewed as
 * (n, B) -- SURVEY §0.1); this rank owns columns [col_offset, col_offset + cols).
 * rg_mf_prepare fills `pairs` with the (user, item) ids of every pair in
 * processing order (position s = column, or plan_perm[s] with a plan), one record
 * per position (rg_mf_pairs_len): entry 0 the positive, 1 + k negative slot k,
 * n_neg + 1 the positive's plan slot.  rg_mf_pairs reads only `pairs` (plus
 * words/pool for the adaptive hinge's max). */
typedef struct rg_mf_batch {
    const int64_t *pos_user, *pos_item;  /* [n_pos] this rank's positives (column order) */
    int64_t n_pos;          /* <= cols; < cols only on the last partial batch */
    int64_t cols;           /* this rank's columns (batch_size) */
    int64_t col_offset;     /* first global column owned by this rank */
    int64_t global_cols;    /* columns of the draw this slice is cut from (batch_size [* world_size]) */
    int64_t global_pos;     /* positives in the whole (global) batch */
    int64_t neg_cols;       /* negatives per draw row over every rank (mean denominator); 0: global_cols */
    const uint32_t *words;  /* raw MT19937 words of this step (rg_mt_generate): draw j uses [2j], [2j+1] */
    const int32_t *pool;    /* negative pool as int32 (user, item) pairs [pool_len] */
    int64_t pool_len;
    int32_t n_neg;          /* negatives per positive, 1..RG_MF_MAX_NEG */
    int32_t loss;           /* enum rg_loss_kind */
    int32_t *pairs;         /* [rg_mf_pairs_len(cols, n_neg)] int32, see above */
} rg_mf_batch_t;

/* Caller-owned scratch.  row_count, hot_grad and hot_bias_grad must be zero
 * before the first step; the library leaves them zero after every
 * rg_mf_pairs + rg_mf_apply/rg_mf_grads pair.
 *
 * Optional per-batch plan (all plan_* null: no plan).  Positives are processed in
 * item-sorted column order and the item-side gradient of the positives is reduced
 * per pair-kernel block into partial rows (plain stores, fixed order) instead of
 * per-row lists + atomics -- the Zipf-hot items.  With U = rg_mf_plan_units_per_block(dim):
 *   plan_perm[s]          column processed at position s (a permutation of [0, cols)),
 *                         positives (column < n_pos) sorted by item, then the rest
 *   plan_pos_slot[s]      partial slot of position s: consecutive positions with the same
 *                         item inside one block of U positions share a slot; slots are
 *                         numbered in position order
 *   plan_item_slot_off[i] item i's slots are [off[i], off[i+1])  (num_items + 1 entries)
 * part_row / part_bias: [slots * dim] / [slots] partial sums (slots <= cols).
 *
 * claim_num_users > 0 (= the tables' num_users; split step, not the adaptive hinge;
 * num_users, num_items < 2^27):
 * rg_mf_prepare claims every valid pair's list slots in row_count (one atomic per row
 * side) and stores them in bits 27-30 of the prepared ids, so rg_mf_pairs writes its
 * list entries at those slots without returning atomics.  The prepare of step t + 1
 * runs inside step t's dense pass, which resets step t's counts: consecutive steps
 * then need separate row_count arrays (the stepper alternates two). */
typedef struct rg_mf_work {
    int32_t *row_count;      /* [num_users + num_items] */
    int32_t *row_list;       /* [(num_users + num_items) * RG_MF_LIST_CAP * 2] {other row, dz bits} */
    int64_t *hot_grad;       /* [(num_users + num_items) * dim] overflow accumulators, int64 fixed
                                point (value * 2^48): order-independent, bit-reproducible sums */
    int64_t *hot_bias_grad;  /* [num_users + num_items], the same */
    float *loss_partials;    /* [rg_mf_partials_len(cols, dim)] */
    float *scores;           /* [cols]  (adaptive hinge only) */
    uint64_t *max_key;       /* [1] (adaptive hinge only) */
    int32_t *active_count;   /* [1] (adaptive hinge only) */
    const int32_t *plan_perm, *plan_pos_slot, *plan_item_slot_off;
    float *part_row, *part_bias;
    int64_t claim_num_users; /* see above; 0: the pair pass claims list slots itself */
} rg_mf_work_t;

/* Loss reduction requested from rg_mf_apply / rg_mf_grads:
 * *out = sum(partials[:,0]) * inv_a + sum(partials[:,1]) * inv_b. */
typedef struct rg_mf_loss {
    int64_t n_partials;
    double inv_a, inv_b;
    float *out;
} rg_mf_loss_t;

typedef struct rg_opt {
    int32_t kind;            /* enum rg_opt_kind */
    float lr, beta1, beta2, eps, weight_decay, alpha;
    /* 1 - beta1, 1 - beta2, 1 - alpha evaluated in double on the host (as the
     * Python optimizer does) and rounded once; fp32 (1 - 0.999f) would differ by 1.3e-5 */
    float one_minus_beta1, one_minus_beta2, one_minus_alpha;
    float step_size;         /* Adam: lr / (1 - beta1^t)  (host, double -> float) */
    float bias_correction2_sqrt;  /* Adam: sqrt(1 - beta2^t) */
} rg_opt_t;

/* Extra words rg_mt_generate may write past nwords (the output buffer must hold
 * nwords + RG_MT_PAD words). */
#define RG_MT_PAD 1280

/* MT19937 stream: advances `state_dev` (624 words + position, the layout of
 * CPython's random.getstate()[1]) by `nwords` and writes the RAW (untempered)
 * state words; output k, tempered, is the k-th genrand_uint32() CPython would
 * return.  If state_before_dev is non-null, the state on entry is copied there
 * first.  Runs as ONE workgroup (the recurrence is sequential). */
int rg_mt_generate(void *stream, uint32_t *state_dev, uint32_t *out_words_dev,
                   int64_t nwords, uint32_t *state_before_dev);

/* Host reference of the MT19937 jump-ahead (rg_mtjump.cpp): the window-form state
 * (x[D .. D+624), position 624) of the word stream x[] that starts at state_host's
 * next word, computed as an XOR of stream windows with the coefficients of
 * t^(D-1) mod chi(t).  D >= 1.  Host memory only. */
int rg_mt_window_host(const uint32_t *state_host, int64_t D, uint32_t *window_out_host);
/* Window-form state x[P-624 .. P) -> CPython's getstate() layout for the same stream
 * position with position `pos` (1..624) inside its block.  Host memory only. */
int rg_mt_window_to_cpython(const uint32_t *window_host, int32_t pos, uint32_t *state_out_host);
/* Advance a CPython getstate() layout state (625 words, host memory) by k raw words
 * in place, as k calls of getrandbits(32) would. */
int rg_mt_advance_host(uint32_t *state_host, int64_t k);

/* NumPy legacy RandomState.randint(low, high, n_out) (int64) from raw MT19937 words
 * (rg_mt_generate started at the RandomState's (key, pos) state): NumPy's masked rejection
 * (distributions.c random_bounded_uint64_fill) as an ordered compaction.  Replaces the host
 * draw of spotlight/sampling.py:9-35 sample_items (random_state.randint(0, num_items, shape)).
 * Needs 2 <= high - low <= 2^32.  *consumed_dev = words the draw used (advance the state by
 * it), or 0 when n_words held fewer than n_out accepted words (generate more and retry).
 * scratch: rg_uniform_scratch_len(n_words) int32 elements, 8-byte aligned. */
int64_t rg_uniform_scratch_len(int64_t n_words);
/* Measurement only (bench.py's STREAM-copy ceiling): dst[i] = src[i] for n_float4 float4s. */
int rg_stream_copy(void *stream, float *dst_dev, const float *src_dev, int64_t n_float4);
int rg_uniform_int64(void *stream, const uint32_t *words_dev, int64_t n_words, int64_t low, int64_t high,
                     int64_t n_out, int64_t *out_dev, int32_t *scratch_dev, int64_t *consumed_dev);

/* int32 elements of a prepared-pairs buffer: one record of S int2 per column (S = 8
 * for n_neg <= 6, else 16): [q] = (user, item) of pair q (0 = the positive, 1 + k =
 * negative k), [n_neg + 1] = (the positive's plan slot or -1, 0), zero padding. */
int64_t rg_mf_pairs_len(int64_t cols, int32_t n_neg);

/* Number of float loss partials rg_mf_pairs writes for `cols` columns. */
int64_t rg_mf_partials_len(int64_t cols, int32_t dim);

/* Positions per pair-kernel block, the block size a batch plan is built for. */
int64_t rg_mf_plan_units_per_block(int32_t dim);

/* The plans (rg_mf_work_t plan_*) of many batches in ONE launch, one workgroup per batch
 * (rg_plan.hip; replaces building them batch by batch on the host).  The reference
 * shuffles once per fit and revisits the same contiguous batches every epoch
 * (implicit.py:262, :290), so they are built once per fit.
 *   batch k = positives [offset + k*stride, offset + k*stride + batch_len) of items / users
 *             (device int64, n entries in all; clipped at n);
 *   owner_world > 1: only the positives whose user u has u % owner_world == owner_rank are
 *             planned (owner-sharded data parallelism; users required), else all;
 *   per batch k (cols >= batch_len is the output stride):
 *     perm[k*cols + s]      planned positives' columns (relative to the batch start) sorted
 *                           by (item, column); then, single rank, the other columns ascending;
 *                           -1 past the planned positives when owner_world > 1
 *     pos_slot[k*cols + s]  partial slot (a new slot where the item changes or a block of
 *                           units_per_block positions starts), -1 past the planned positives
 *     item_slot_off[k*(num_items+1) + i]   item i's slots [off[i], off[i+1])
 *     counts[2k], counts[2k+1]             planned positives, slots
 * scratch: rg_mf_plans_scratch_len(cols, n_batches) uint64 of device memory (0: null is
 * fine; only batches of more than 16,384 planned positives use it). */
int64_t rg_mf_plans_scratch_len(int64_t cols, int64_t n_batches);
int rg_mf_plans_build(void *stream, const int64_t *users, const int64_t *items, int64_t n, int64_t offset,
                      int64_t stride, int64_t batch_len, int64_t n_batches, int64_t cols, int32_t units_per_block,
                      int64_t num_items, int32_t owner_world, int32_t owner_rank, int32_t *perm, int32_t *pos_slot,
                      int32_t *item_slot_off, int32_t *counts, uint64_t *scratch);

/* Resolve the step's pairs: positives permuted to processing order and every
 * negative draw -> pool index (CPython random.choices arithmetic) -> (user, item).
 * Fully parallel; depends only on the words, the pool, the plan and the ids, so it
 * can run ahead on another stream. */
int rg_mf_prepare(void *stream, const rg_mf_batch_t *batch, const rg_mf_work_t *work);

/* Row marks of one prepared step (the overlapped step below).  stamp: [U + I] int32
 * (caller-owned, zero-initialised), serial: nonzero, unique per marked prepare. */
typedef struct rg_mf_mark {
    int32_t *stamp;
    int64_t num_users;
    int32_t serial, pad_;
} rg_mf_mark_t;

/* rg_mf_prepare that also stamps every row the step's pairs touch with
 * mark->serial; the first pair to stamp a row gets the row's ownership flag (bit 31
 * of its prepared id; rg_mf_pairs and the NCF kernels ignore the flags). */
int rg_mf_prepare_marked(void *stream, const rg_mf_batch_t *batch, const rg_mf_work_t *work,
                         const rg_mf_mark_t *mark);

/* The overlapped training step (implicit.py:347-364 as two launches):
 *   rg_mf_step_front: rg_mf_pairs(backward) of `cur` (prepared with cur_mark), the
 *     marked prepare of `next` (optional; its own stamp array and serial), and the
 *     optimizer update of every row in [cold_begin, cold_end) whose stamp is not
 *     cur_mark->serial (no data gradient: weight decay only), all in ONE grid;
 *   rg_mf_step_hot: the update of every touched row in [row_begin, row_end), pulling
 *     the lists / partials of the pair pass, plus the loss: rows found by a scan of
 *     the range for cur_mark's serial (mark non-null) or through the owner-flagged
 *     ids of cur's pairs (mark null).
 * Together they equal rg_mf_pairs + rg_mf_apply over the same rows, bit for bit.
 * Not for adaptive hinge (its backward needs the global max first). */
int rg_mf_step_front(void *stream, const rg_mf_tables_t *tables, const rg_mf_batch_t *cur, rg_mf_work_t *work,
                     const rg_mf_mark_t *cur_mark, const rg_opt_t *opt, int64_t cold_begin, int64_t cold_end,
                     const rg_mf_batch_t *next, const rg_mf_work_t *next_work, const rg_mf_mark_t *next_mark);
/* The cold-row part of rg_mf_step_front as its own launch (rows in range whose
 * stamp is not mark->serial; weight decay only), for a two-stream schedule. */
int rg_mf_step_cold(void *stream, const rg_mf_tables_t *tables, const rg_mf_mark_t *mark, const rg_opt_t *opt,
                    int64_t row_begin, int64_t row_end);
int rg_mf_step_hot(void *stream, const rg_mf_tables_t *tables, const rg_mf_batch_t *cur, rg_mf_work_t *work,
                   const rg_mf_mark_t *mark, const rg_opt_t *opt, int64_t row_begin, int64_t row_end,
                   const rg_mf_loss_t *loss);

/* Forward of all pairs of the step, the loss terms, dL/dz, and the per-row
 * contribution lists (+ planned partials) consumed by rg_mf_apply / rg_mf_grads.
 * backward = 0 computes the loss only (validation, implicit.py:366). */
int rg_mf_pairs(void *stream, const rg_mf_tables_t *tables, const rg_mf_batch_t *batch,
                rg_mf_work_t *work, int32_t backward);

/* Rows are numbered users [0, U) then items [U, U + I); [row_begin, row_end)
 * selects the rows a call touches (row_end < 0: all).  Item rows run first. */

/* Gradient gather (pull from the contribution lists) + optimizer update of EVERY
 * row in the range (coupled weight decay touches all rows).  loss: optional. */
int rg_mf_apply(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, const rg_opt_t *opt,
                int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss);

/* rg_mf_apply and the rg_mf_prepare of the NEXT step (optional: next null) in one
 * launch (the prepare runs in extra workgroups beside the HBM-bound update), so a
 * training step needs no side stream and no per-step cross-stream event. */
int rg_mf_apply_prepare(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, const rg_opt_t *opt,
                        int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss, const rg_mf_batch_t *next,
                        const rg_mf_work_t *next_work);

/* An MT19937 walk to run inside another launch (one extra workgroup): advances
 * `state` (CPython getstate()[1] layout, device) by nwords raw words into out
 * (nwords + RG_MT_PAD words), copying the entry state to state_before (optional) --
 * rg_mt_generate's work, without a launch or stream of its own. */
typedef struct rg_mt_gen {
    uint32_t *state, *out, *state_before;
    int64_t nwords;                 /* 0: no walk */
} rg_mt_gen_t;

/* rg_mf_apply_prepare plus, in one more workgroup of the same launch, the MT walk of a
 * later step's words (gen may be null).  The single-GPU native step uses it so the
 * sampler stream needs neither a generator stream nor a per-step event. */
int rg_mf_apply_prepare_gen(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, const rg_opt_t *opt,
                            int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss,
                            const rg_mf_batch_t *next, const rg_mf_work_t *next_work, const rg_mt_gen_t *gen);

/* Pipelined single-GPU step (A/B build only, -DRG_AB=1: measured 4x slower than the split
 * step; the product library refuses it and the stepper never selects it): ONE
 * launch that runs
 *   the dense update of step t (tables t -> tables' out set, as rg_mf_apply),
 *   the pair pass of step t+1 (pair_b / pair_w, prepared with claimed slots; it reads the
 *     rows this launch writes and waits, in the launch, until every row it reads is written),
 *   the prepare of step t+2 (optional: next null; claims in next_w->row_count and appends
 *     every user it claims a first slot of to pipe->hot_out / *pipe->nhot_out).
 * Replaces run_train_iteration's forward/backward (implicit.py:348-361) of step t+1 and the
 * optimizer step (implicit.py:363) of step t, overlapped.  pair_w's scratch (lists, overflow
 * accumulators, partials, planned partials) must not alias w's.  Loss: pointwise, bpr, hinge. */
typedef struct rg_mf_pipe {
    const int32_t *hot_users;   /* users step t+1's pair pass reads (rg_mf_prepare_hot of step t+1) */
    const int32_t *nhot;        /* [1] their number */
    const int32_t *counts_next; /* step t+1's claim counts (a user with a claim is one of them) */
    int32_t *gate;              /* [1] 0 on entry (this launch's hot-row counter) */
    int32_t *gate_next;         /* [1] set to 0 (the next launch's gate) */
    int32_t *nhot_free;         /* [1] set to 0 (the hot-list length the launch after next appends to) */
    int32_t *hot_out, *nhot_out;/* step t+2's hot list (next != null); *nhot_out 0 on entry */
    int32_t *err;               /* [1] set to 1 if a pair workgroup's bounded wait ran out */
} rg_mf_pipe_t;
int rg_mf_pipe_step(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, const rg_opt_t *opt,
                    const rg_mf_loss_t *loss, const rg_mf_batch_t *pair_batch, rg_mf_work_t *pair_work,
                    const rg_mf_batch_t *next, const rg_mf_work_t *next_work, const rg_mf_pipe_t *pipe,
                    const rg_mt_gen_t *gen);
/* rg_mf_prepare with claimed slots that also lists the users it claims a first slot of
 * (hot_out, *nhot_out; 0 on entry): the first step of a pipelined sequence. */
int rg_mf_prepare_hot(void *stream, const rg_mf_batch_t *batch, const rg_mf_work_t *work, int32_t *hot_out,
                      int32_t *nhot_out);

/* The single-GPU step as TWO launches per step t (opt-in, RG_PIPE2=1, for pointwise / bpr / hinge via
 * rg_mf_stepper_train_ahead; measured slower than the split step), replacing run_train_iteration (implicit.py:347-364) of
 * step t+1 up to its backward and the optimizer step (implicit.py:363, spotlight/optimizers.py:10-16)
 * of step t, with step t+1's latency-bound pair pass beside the HBM-bound update of the rows it does
 * not read:
 *   rg_mf_pipe2_hot:  step t's dense update (as rg_mf_apply) of every item row and of the users in
 *                     hot_users[0 .. *nhot) (step t+1's hot list); step t's loss; *nhot_clear = 0
 *                     (optional: the list the cold launch's prepare appends to); gen: a later unit's
 *                     MT walk in one workgroup (optional).  hot_cap >= *nhot sizes the grid.
 *   rg_mf_pipe2_cold: step t+1's pair pass (pair_batch / pair_work: prepared with claims in
 *                     counts_next, which must be pair_work->row_count; it reads the tables' OUT set,
 *                     rows the hot launch wrote), the prepare of step t+2 (optional: next null;
 *                     claims in next_work->row_count, its hot list to hot_out / *nhot_out), gen, and
 *                     step t's dense update of every user with counts_next[u] == 0.
 * Per-row and per-column arithmetic is rg_mf_apply's / rg_mf_pairs', so the results are bit-identical
 * to the split step.  pair_work's scratch (lists, overflow accumulators, partials, planned partials,
 * counts) must not alias work's.  Loss: pointwise, bpr, hinge. */
int rg_mf_pipe2_hot(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, const rg_opt_t *opt,
                    const rg_mf_loss_t *loss, const int32_t *hot_users, const int32_t *nhot, int64_t hot_cap,
                    int32_t *nhot_clear, const rg_mt_gen_t *gen);
int rg_mf_pipe2_cold(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, const rg_opt_t *opt,
                     const rg_mf_batch_t *pair_batch, rg_mf_work_t *pair_work, const int32_t *counts_next,
                     const rg_mf_batch_t *next, const rg_mf_work_t *next_work, int32_t *hot_out, int32_t *nhot_out,
                     const rg_mt_gen_t *gen);

/* Pull the DATA gradient (no weight decay) of the rows in range into the flat
 * buffer grad_dev = [n*dim row grads | n bias grads | loss], n = row_end - row_begin
 * (the loss slot is written when loss->out is non-null).  Resets the lists like
 * rg_mf_apply.  The caller all-reduces grad_dev across ranks (RCCL). */
int rg_mf_grads(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, float *grad_dev,
                int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss);

/* Replicated data-parallel step (one process per GPU, every rank holds every row;
 * the reference-exact layout of SURVEY §8e): the flat gradient is RANK-MAJOR so that
 * ncclReduceScatter hands rank s the summed gradient of exactly its row shard --
 * chunk s (rg_mf_grad_chunk floats, a multiple of 4) holds
 *   [user rows s*Us .. (s+1)*Us | item rows s*Is .. (s+1)*Is] (dim floats each),
 *   their biases (Us + Is), the loss;
 * Us * world >= num_users, Is * world >= num_items (rows past the tables stay zero).
 * rg_mf_grads_sharded pulls every row's data gradient (the lists of rg_mf_pairs) into
 * that layout and writes this rank's loss share into every chunk's loss slot (the
 * reduce-scatter sums it); rg_mf_apply_shard updates rank `rank`'s rows from its
 * (summed) chunk into the *_out tables; an all-gather of the four *_out tables
 * (counts Us*dim, Is*dim, Us, Is; tables allocated with world*Us / world*Is rows)
 * completes the step. */
int64_t rg_mf_grad_chunk(int64_t shard_users, int64_t shard_items, int32_t dim);
int rg_mf_grads_sharded(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, float *grad_dev,
                        int64_t shard_users, int64_t shard_items, int32_t world, const rg_mf_loss_t *loss);
int rg_mf_apply_shard(void *stream, const rg_mf_tables_t *tables, const float *grad_dev, const rg_opt_t *opt,
                      int64_t shard_users, int64_t shard_items, int32_t world, int32_t rank, float *loss_out_dev);

/* The owner-sharded step's item update split the same way (dp_mode 2 with shard_items = Is > 0):
 * rg_mf_grads_item_shard writes the item rows' data gradient rank-major, chunk s =
 * [item rows s*Is .. (s+1)*Is (dim floats each) | their Is biases | the loss share], each chunk
 * rg_mf_item_grad_chunk(Is, dim) floats; after a reduce-scatter rg_mf_apply_item_shard updates
 * items [rank*Is, min((rank+1)*Is, num_items)) into item_w_out / item_b_out, and an all-gather of
 * those two tables (counts Is*dim, Is; allocated with world*Is rows) completes the item update. */
int64_t rg_mf_item_grad_chunk(int64_t shard_items, int32_t dim);
int rg_mf_grads_item_shard(void *stream, const rg_mf_tables_t *tables, rg_mf_work_t *work, float *grad_dev,
                           int64_t shard_items, int32_t world, const rg_mf_loss_t *loss);
int rg_mf_apply_item_shard(void *stream, const rg_mf_tables_t *tables, const float *grad_dev, const rg_opt_t *opt,
                           int64_t shard_items, int32_t world, int32_t rank, float *loss_out_dev);

/* ------------------------------------------------------------------------------
 * Owner-sharded data-parallel step (dp_mode 2; rg_owner.hip), reference-exact: R ranks
 * at batch B compute the reference's step at batch R*B (one global CPython stream of
 * n*R*B draws over the FULL pool, contiguous global batches, global loss means;
 * implicit.py:262, :290, :351-354), with only the items replicated:
 *   rank r owns the users u with u % R == r (its tables hold them as local rows u / R,
 *   then every item); every rank walks the global draw and keeps the pairs whose user
 *   it owns (rg_mf_owner_prepare);
 *   rg_mf_owner_scores: the scores of its pairs into a zeroed global score vector
 *   [(1 + n) * GC] (pair gp = c: positive of column c, (1 + k) * GC + c: its negative k);
 *   -> all-reduce (sum; every slot has exactly one writer, so the sum is exact) ->
 *   rg_mf_owner_back: dL/dz of its pairs from the column's scores (the BPR / hinge
 *   pairing couples a column's positive with its negatives), contribution lists, planned
 *   item partials, loss partials (this rank's share);
 *   -> rg_mf_grads over the item rows (+ loss) -> all-reduce -> rg_mf_apply_dense of the
 *   items beside rg_mf_apply of the user rows.
 * Per step a rank exchanges 4 (1 + n) GC bytes of scores and the (I (d + 1) + 1)-float
 * item gradient, instead of the (U + I)(d + 1) floats of the replicated layout.
 * Not for adaptive hinge (global max over all negatives).
 * ---------------------------------------------------------------------------- */
typedef struct rg_mf_owner_batch {
    const int64_t *pos_user, *pos_item;  /* the GLOBAL batch's positives (global ids), column order */
    int64_t n_pos;                       /* positives in the global batch (<= global_cols) */
    int64_t global_cols;                 /* GC = batch_size * world */
    const int32_t *plan_perm, *plan_pos_slot;   /* this rank's planned positives (rg_mf_plans_build
                                                   with the owner filter); plan_item_slot_off in work */
    int64_t n_planned;
    const uint32_t *words;               /* 2 * n_neg * GC raw MT19937 words of the step */
    const int32_t *pool;                 /* the FULL negative pool, int32 (user, item) global ids */
    int64_t pool_len;
    int32_t n_neg, loss;
    int32_t world, rank;
    int32_t *neg_rec;                    /* [4 * rg_mf_owner_rec_len(GC, n_neg)] prepared records */
    int32_t *seg_count;                  /* [rg_mf_owner_segments(GC, n_neg)] */
    float *scores;                       /* [(1 + n_neg) * GC] (+ 4 for the adaptive hinge: max, its
                                            pair, the active count -- rg_mf_owner_adapt) */
    int32_t *claim_count;                /* non-null (not the adaptive hinge): rg_mf_owner_prepare claims
                                            each kept draw's two list slots here (local user row, and
                                            claim_num_users + item) and keeps them in its record, and
                                            rg_mf_owner_back appends there without atomics; the work's
                                            row_count of the step must be this array (alternate two
                                            between consecutive steps, as rg_mf_work_t claim_num_users) */
    int64_t claim_num_users;             /* this rank's user rows */
} rg_mf_owner_batch_t;

int64_t rg_mf_owner_segments(int64_t global_cols, int32_t n_neg);
/* Adaptive hinge, after the score exchange: the global max negative (largest score, first
 * draw on ties) and the active-positive count, computed from the full score vector on every
 * rank (no further exchange), into scores[(1 + n_neg) * GC + {0, 1, 2}]; rg_mf_owner_back
 * then gives the positives the hinge against it and the max's owner its gradient. */
int rg_mf_owner_adapt(void *stream, const rg_mf_owner_batch_t *b);
int64_t rg_mf_owner_rec_len(int64_t global_cols, int32_t n_neg);
/* float loss partials rg_mf_owner_back writes (upper bound over any n_planned <= GC) */
int64_t rg_mf_owner_partials_len(int64_t global_cols, int32_t n_neg, int32_t dim, int32_t world);
/* the partials a step with n_planned planned positives actually writes */
int64_t rg_mf_owner_partials_used(int64_t global_cols, int32_t n_neg, int32_t dim, int32_t world,
                                  int64_t n_planned);
int rg_mf_owner_prepare(void *stream, const rg_mf_owner_batch_t *batch);
/* tables: this rank's (num_users = its local users) */
int rg_mf_owner_scores(void *stream, const rg_mf_tables_t *tables, const rg_mf_owner_batch_t *batch);
int rg_mf_owner_back(void *stream, const rg_mf_tables_t *tables, const rg_mf_owner_batch_t *batch,
                     rg_mf_work_t *work);
/* run_val_iteration's loss (implicit.py:366-379) of the step from its EXCHANGED score vector
 * (every rank computes the same value; one workgroup, fixed order) */
int rg_mf_owner_loss(void *stream, const rg_mf_owner_batch_t *batch, float *loss_out_dev);

/* Optimizer update of the rows in range from a (summed) flat gradient
 * (+ weight_decay * p).  loss_out_dev (optional) receives grad_dev's loss slot. */
int rg_mf_apply_dense(void *stream, const rg_mf_tables_t *tables, const float *grad_dev, const rg_opt_t *opt,
                      int64_t row_begin, int64_t row_end, float *loss_out_dev);

/* loss = sum(partials[:,0]) * inv_a + sum(partials[:,1]) * inv_b  (one block). */
int rg_loss_finalize(void *stream, const float *partials_dev, int64_t n_partials,
                     double inv_a, double inv_b, float *loss_out_dev);

/* Scores sigmoid(<U[u],I[i]> + ub[u] + ib[i]) for n pairs (ids int64). */
int rg_mf_scores(void *stream, const float *user_w, const float *item_w,
                 const float *user_b, const float *item_b, int32_t dim,
                 const int64_t *users, const int64_t *items, int64_t n, float *out);

/* ------------------------------------------------------------------------------
 * Lazy dense pass.  The reference's dense coupled-L2 optimizer moves EVERY
 * row every step (optimizers.py:10-16 over sparse=False tables, mf_spotlight.py:55); a
 * user row no pair touches gets the cold update opt(p, grad = wd * p) only.  The lazy
 * pass defers those cold updates: a user row is processed at step t iff it has a data
 * gradient at t (list count), the NEXT step's pair pass reads it (a mark the next step's
 * prepare wrote), or the pass is a full one; a processed row first applies its skipped
 * cold updates in step order with each step's own Adam constants (the eager pass's exact
 * operation sequence), so every row any kernel reads is bit-identical to the eager
 * pass's, and rg_mf_lazy_flush brings every row up to date (before validation, predict,
 * a checkpoint, the end of a fit).  Item rows are always processed.
 * ---------------------------------------------------------------------------- */
typedef struct rg_mf_lazy {
    int32_t *last_rel;         /* [num_users] last step applied to each user row, minus base */
    int32_t *umark;            /* [num_users] step whose pair pass reads the row (prepare marks) */
    const float *step_consts;  /* [2 * n_consts] Adam (step_size, bias_correction2_sqrt) of absolute step s */
    int64_t n_consts;
    int64_t base;              /* absolute step of last_rel == 0 */
    int64_t step;              /* rg_mf_apply_lazy: the step applied; rg_mf_lazy_flush: the step caught up to */
    int32_t full;              /* rg_mf_apply_lazy: process every user row */
    int32_t pad_;
    uint64_t *rows_done;       /* optional: += user rows processed (diagnostics; contended) */
} rg_mf_lazy_t;

/* The pair pass of this step (rg_mf_pairs, backward) and the prepare of `next` in one
 * launch; the prepare stores umark[user] = umark_step for every pair's user. */
int rg_mf_pairs_prepare(void *stream, const rg_mf_tables_t *t, const rg_mf_batch_t *b, rg_mf_work_t *w,
                        const rg_mf_batch_t *next, const rg_mf_work_t *next_w, int32_t *umark, int32_t umark_step);
/* Lazy dense pass of step lazy->step over every row (items always, users by the rule
 * above), loss finalisation, optional MT walk; writes the *_out tables. */
int rg_mf_apply_lazy(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                     const rg_mf_loss_t *loss, const rg_mf_lazy_t *lazy, const rg_mt_gen_t *gen);
/* Every user row caught up to step lazy->step, into the tables' IN side (the current set;
 * a row whose value is in the other set is read from the *_out side). */
int rg_mf_lazy_flush(void *stream, const rg_mf_tables_t *t, const rg_opt_t *opt, const rg_mf_lazy_t *lazy);

/* ------------------------------------------------------------------------------
 * RCCL communicator (rg_comm.cpp) for the user-sharded data-parallel step: one
 * process per GPU; rank 0 makes the id, the caller broadcasts it (torch.distributed),
 * every rank creates its communicator on `device`.
 * ---------------------------------------------------------------------------- */
#define RG_COMM_ID_BYTES 128
int rg_comm_unique_id(uint8_t *out, int64_t len);
void *rg_comm_create(const uint8_t *id, int32_t world, int32_t rank, int32_t device);
/* One-GPU stand-in for rank `rank` of a `world`-rank communicator (bench.py
 * --emulate-rank): every collective is a same-size local copy out and back on the
 * communicator stream (data unchanged), placed and fenced like the RCCL path. */
void *rg_comm_create_local(int32_t world, int32_t rank, int32_t device);
/* Host-staged stand-in (tests: two processes sharing one GPU, where RCCL refuses a second
 * rank on a device): each all-reduce runs on the communicator stream, placed and fenced like
 * the RCCL one, as a D2H copy into pinned staging, a host callback fn(ctx, host_buf, n)
 * (stream-ordered, hipLaunchHostFunc; must sum host_buf over the ranks in place and return
 * 0; no HIP calls), and an H2D copy back.  All-reduce only; n <= max_floats. */
typedef int (*rg_host_allreduce_fn)(void *ctx, float *host_buf, int64_t n);
void *rg_comm_create_host(int32_t world, int32_t rank, int32_t device, int64_t max_floats,
                          rg_host_allreduce_fn fn, void *ctx);
/* Host-staged stand-in only: the owner step's MT word all-gather (a rank's slice of each step's
 * words to every rank, bit for bit), called synchronously on the stepper's host thread:
 * fn(ctx, send, n, recv) must gather n words from every rank into recv[world * n] in rank order
 * and return 0 (tests: a gloo all_gather on a group of its own). */
typedef int (*rg_host_gather_fn)(void *ctx, const uint32_t *send, int64_t n, uint32_t *recv);
int rg_comm_set_host_gather(void *comm, rg_host_gather_fn fn, void *ctx);
int rg_comm_destroy(void *comm);
/* What the native communicator reports: ncclCommCount / ncclCommUserRank of an RCCL
 * communicator (is_rccl = 1), or the configured world / rank of a local / host-staged stand-in
 * (is_rccl = 0). */
int rg_comm_info(void *comm, int32_t *count, int32_t *user_rank, int32_t *is_rccl);
/* In-place sum over ranks, stream-ordered with respect to `stream` (runs on the
 * communicator's own stream between two events). */
int rg_comm_allreduce_sum_f32(void *comm, void *stream, float *buf_dev, int64_t n);
/* In-place reduce-scatter (sum): rank r receives the sum of every rank's chunk r at
 * buf_dev + r * chunk.  On `stream` itself. */
int rg_comm_reduce_scatter_f32(void *comm, void *stream, float *buf_dev, int64_t chunk);
/* In-place all-gather of n buffers in one group: rank r's counts[k] floats at
 * bufs[k] + r * counts[k] go to every rank.  On `stream` itself. */
int rg_comm_allgather_f32(void *comm, void *stream, int32_t n, float *const *bufs_dev, const int64_t *counts);

/* ------------------------------------------------------------------------------
 * Native step runtime (rg_stepper.cpp): one call per training step enqueues
 *   gen stream:   rg_mt_generate of the stream chunk two steps ahead
 *   prep stream:  rg_mf_prepare of the NEXT step (draws -> pool pairs)
 *   main stream:  rg_mf_pairs -> rg_mf_apply of the current step
 * Replaces the loop body implicit.py:290-298 / run_train_iteration :347-364.
 *
 * User-sharded data parallelism (item_grad != NULL): this rank's tables hold its
 * own users (rows [0, num_users)) and every item (replicated).  The step becomes
 *   rg_mf_pairs -> rg_mf_grads(item rows -> item_grad) -> [comm: all-reduce on the
 *   communicator stream] || rg_mf_apply(user rows) -> rg_mf_apply_dense(item rows)
 * so the only exchange is the item gradient, overlapped with the user update.
 * ---------------------------------------------------------------------------- */
typedef struct rg_mf_stepper_config {
    rg_mf_tables_t tables[2];       /* tables[k]: reads set k, writes set 1 - k */
    rg_mf_work_t work;              /* plan_* fields are set per step */
    uint32_t *mt_state;             /* [625] CPython getstate()[1] layout; the stepper owns its
                                       word ring (3 chunks of 2*n_neg*global_cols words) */
    int32_t *pairs[2];              /* [(1 + n_neg) * cols * 2] each */
    const int32_t *pool;
    int64_t pool_len;
    int32_t n_neg, loss;
    int64_t cols, col_offset, global_cols;   /* draw layout: j = (q-1)*global_cols + col_offset + col */
    int64_t neg_cols;               /* negatives per draw row over every rank (loss denominator) */
    float *item_grad;               /* [num_items*(dim+1) + 1] (shard_items > 0 in dp_mode 2:
                                       [world * rg_mf_item_grad_chunk(shard_items, dim)]): the
                                       user-sharded DP step when non-null */
    void *comm;                     /* rg_comm_create handle (NULL: single rank, no exchange) */
    rg_opt_t opt;                   /* kind + fp32 hyper-parameters */
    double lr_d, beta1_d, beta2_d;  /* the same as Python floats (Adam bias corrections) */
    int64_t step;                   /* optimizer steps already taken */
    int64_t n_partials;
    int32_t current_set;
    int32_t gen_mode;               /* 0: MT words walked inside the step's dense pass when that hides
                                       them (rg_mf_stepper_train); 1: the consumer has no such pass
                                       (NeuMF, data-parallel NCF): 8-step slots on the generator
                                       stream; 2: the consumer's own tail launch walks them when
                                       that hides them (single-GPU NCF: rg_mf_stepper_tail_gen +
                                       rg_ncf_tail), otherwise as 1; 3: as 2 without the stepper's
                                       test, made by the caller (NeuMF: the GMF tables' pass) */
    /* dp_mode 1: the replicated, reference-exact data-parallel step (rg_mf_grads_sharded ->
     * reduce-scatter -> rg_mf_apply_shard -> all-gather), rank `rank` of `world`; every rank
     * consumes columns [col_offset, col_offset + cols) of one global draw of global_cols
     * columns.  grad_buf: [world * rg_mf_grad_chunk(shard_users, shard_items, dim)]. */
    int32_t dp_mode, rank, world, pad2_;
    int64_t shard_users, shard_items;
    float *grad_buf;
    /* dp_mode 2: the owner-sharded step (rg_mf_owner_*, reference-exact): tables[k] hold this
     * rank's users (local rows u / world) and every item; cols = global_cols = GC and
     * col_offset = 0 (every rank walks the whole global draw); item_grad is the exchanged
     * item gradient; per-unit buffers (unit parity) of the prepared records, their segment
     * counts and the score vector the first exchange sums. */
    int32_t *owner_rec[2];          /* [4 * rg_mf_owner_rec_len(GC, n_neg)] each */
    int32_t *owner_seg[2];          /* [rg_mf_owner_segments(GC, n_neg)] each */
    float *owner_scores[2];         /* [(1 + n_neg) * GC] each */
} rg_mf_stepper_config_t;

typedef struct rg_mf_step_in {
    const int64_t *pos_user, *pos_item;
    int64_t n_pos, global_pos;
    const int32_t *plan_perm, *plan_pos_slot, *plan_item_slot_off;   /* optional plan */
    int64_t n_planned;              /* dp_mode 2: this rank's planned positives (plan required);
                                       pos_user / pos_item / n_pos are then the GLOBAL batch */
} rg_mf_step_in_t;

void *rg_mf_stepper_create(const rg_mf_stepper_config_t *config);
/* How the stepper produces its MT words: 0 one walk of every word, 1 jump-ahead head + parallel
 * tail segments of the whole global draw (data-parallel steps), 2 this rank's slice of every
 * step's draw + a jump, the slices all-gathered (the owner step over a communicator). */
int32_t rg_mf_stepper_mt_mode(void *stepper);
int rg_mf_stepper_destroy(void *stepper);
/* One fused training step on `stream`; `next` (optional) = the following step's
 * inputs, whose words and pairs are produced ahead on the side stream.  Optional
 * events (hipEvent_t) are recorded around rg_mf_apply. */
int rg_mf_stepper_train(void *stepper, void *stream, const rg_mf_step_in_t *cur, const rg_mf_step_in_t *next,
                        float *loss_out_dev, void *ev_apply_begin, void *ev_apply_end);
/* rg_mf_stepper_train with two steps of lookahead: the pipelined single-GPU step
 * (rg_mf_pipe_step) runs step t's dense update, step t+1's pair pass (`next`) and step t+2's
 * prepare (`next2`, optional) in one launch; a later call whose input is not the `next` given
 * here, or any acquire, drops what ran ahead.  Other configurations: rg_mf_stepper_train. */
int rg_mf_stepper_train_ahead(void *stepper, void *stream, const rg_mf_step_in_t *cur, const rg_mf_step_in_t *next,
                              const rg_mf_step_in_t *next2, float *loss_out, void *ev_apply_begin,
                              void *ev_apply_end);
/* 1 if the stepper runs the pipelined step (rg_mf_stepper_train_ahead), 0 if not. */
int rg_mf_stepper_pipelined(void *stepper);
/* *err_out = 1 if a pipelined launch's pair workgroups ran out of their bounded wait (synchronises). */
int rg_mf_stepper_pipe_error(void *stepper, int32_t *err_out);
/* Words + pairs of `cur` for an external consumer on `stream` (validation, split
 * data-parallel steps); *batch_out / *work_out are ready for rg_mf_pairs.
 * Follow the consumer's launch with rg_mf_stepper_release. */
int rg_mf_stepper_acquire(void *stepper, void *stream, const rg_mf_step_in_t *cur, rg_mf_batch_t *batch_out,
                          rg_mf_work_t *work_out);
int rg_mf_stepper_release(void *stepper, void *stream);
/* After a step's release: prepare the next unit's pairs for `next` on the side stream now
 * (ordered after the work `stream` holds), so the next acquire with the same input finds
 * them ready.  A different input there prepares again. */
int rg_mf_stepper_prefetch(void *stepper, void *stream, const rg_mf_step_in_t *next);
/* The same prepare enqueued on `stream` itself (no side stream, no events): for callers that
 * enqueue it after their step's last kernel (the NCF / NeuMF engines). */
int rg_mf_stepper_prefetch_inline(void *stepper, void *stream, const rg_mf_step_in_t *next);
/* The bookkeeping of rg_mf_stepper_prefetch_inline without its launch: fills the batch / work
 * of the next unit's prepare, which the caller launches on `stream` inside another kernel
 * (rg_ncf_tail).  Returns 1 (launch it), 0 (already prepared) or an error status. */
int rg_mf_stepper_prefetch_args(void *stepper, void *stream, const rg_mf_step_in_t *next, rg_mf_batch_t *batch_out,
                                rg_mf_work_t *work_out);
/* After a step's release, gen_mode 2 / 3: when the MT words of the unit after the next one are due,
 * fills *gen_out with their walk -- which the caller enqueues on `stream` before any other
 * work there (rg_ncf_tail's first workgroup) -- and returns 1; returns 0 (nothing to walk:
 * *gen_out zeroed) or an error status. */
int rg_mf_stepper_tail_gen(void *stepper, void *stream, rg_mt_gen_t *gen_out);
/* The replicated data-parallel step (dp_mode 1) in two halves around a caller-run
 * exchange (comm == NULL; tests, gloo): dp_begin = prepare / pairs / release / the next
 * step's prepare / rg_mf_grads_sharded into grad_buf; the caller reduce-scatters grad_buf;
 * dp_end = rg_mf_apply_shard of this rank's chunk + flip of the table sets; the caller
 * then all-gathers the four current tables.  With a communicator rg_mf_stepper_train
 * runs both halves and both collectives itself. */
int rg_mf_stepper_dp_begin(void *stepper, void *stream, const rg_mf_step_in_t *cur, const rg_mf_step_in_t *next,
                           float *loss_out_dev);
int rg_mf_stepper_dp_end(void *stepper, void *stream, float *loss_out_dev);
/* The owner-sharded step (dp_mode 2) in three parts around caller-run all-reduces (sum)
 * (comm == NULL; tests, gloo); with a communicator rg_mf_stepper_train runs all of it:
 *   owner_begin: prepare (unless prefetched) + rg_mf_owner_scores of `cur` -> the caller
 *     all-reduces rg_mf_stepper_owner_buffers' scores (pointwise: no exchange needed);
 *   owner_mid: rg_mf_owner_back + rg_mf_grads of the item rows into item_grad -> the caller
 *     all-reduces item_grad;
 *   owner_end: the user rows' update with `next`'s owner prepare in the same launch, then
 *     the items from item_grad; flips the sets. */
int rg_mf_stepper_owner_begin(void *stepper, void *stream, const rg_mf_step_in_t *cur);
int rg_mf_stepper_owner_mid(void *stepper, void *stream, float *loss_out_dev);
/* (ev_begin / ev_end optional hipEvent_t recorded around the user rows' update launch) */
int rg_mf_stepper_owner_end(void *stepper, void *stream, const rg_mf_step_in_t *next, float *loss_out_dev,
                            void *ev_begin, void *ev_end);
/* the current unit's score vector and its length (floats) */
int rg_mf_stepper_owner_scores(void *stepper, float **scores_out, int64_t *len_out);
/* Validation (run_val_iteration) in the owner layout: owner_begin of `cur` (same draw stream),
 * the caller all-reduces the scores, owner_val_end writes the batch's loss; with a
 * communicator rg_mf_stepper_owner_val does all three. */
int rg_mf_stepper_owner_val_end(void *stepper, void *stream, float *loss_out_dev);
int rg_mf_stepper_owner_val(void *stepper, void *stream, const rg_mf_step_in_t *cur, float *loss_out_dev);
/* Optimizer scalars for optimizer step `step` (1-based). */
int rg_mf_stepper_opt(void *stepper, int64_t step, rg_opt_t *opt_out);
int rg_mf_stepper_state(void *stepper, int32_t *current_set, int64_t *step);
/* After an external update: flip the ping-pong sets and count optimizer steps. */
int rg_mf_stepper_advance(void *stepper, int32_t flip_sets, int64_t steps);
/* direction 0: copy the MT state after the last consumed word to host_state[625];
 * 1: load host_state into the device state (drops words generated ahead).  Synchronises. */
int rg_mf_stepper_sync_mt(void *stepper, uint32_t *host_state, int32_t direction);
/* Lazy split step (single rank; RG_LAZY=0 disables): bring every user row up to the
 * current step in the current set (rg_mf_lazy_flush; no-op when none lags).  The
 * stepper flushes by itself before an external consumer (acquire) and before a step
 * whose pairs it did not prepare; callers that read the tables directly (predict, a
 * checkpoint, set_params) call it first. */
int rg_mf_stepper_flush(void *stepper, void *stream);
/* Diagnostics: *rows_out = user rows the lazy passes processed since the last call
 * (synchronises; then reset); `enable` turns the counting on for later steps.  Returns 1
 * if the stepper runs the lazy pass, 0 if not. */
int rg_mf_stepper_lazy_count(void *stepper, int32_t enable, uint64_t *rows_out);

/* ------------------------------------------------------------------------------
 * NCF MLP (rg_ncf.hip): spotlight/dnn_models/mlp.py:5-46 trained by
 * implicit.py:347-364, layers [2E, E, ..., 8] -> 1 (ncf_spotlight.py:53-56),
 * E in {8, 16, 32, 64}.  A step is
 *   rg_mf_prepare -> rg_ncf_pairs (fused forward + loss + backward, MFMA) ->
 *   rg_ncf_update (MLP gradient reduce + optimizer) -> rg_ncf_apply (embeddings)
 * (adaptive hinge: rg_ncf_pairs(scores) -> rg_ncf_adapt_dp -> rg_ncf_pairs(given dp)).
 * ---------------------------------------------------------------------------- */
typedef struct rg_ncf_model {
    float *user_w, *item_w;                 /* [U, E], [I, E]; updated in place */
    float *user_w_m, *user_w_v, *item_w_m, *item_w_v;
    float *mlp, *mlp_m, *mlp_v;             /* flat MLP parameters, named_parameters() order */
    int64_t num_users, num_items;
    int32_t dim;
    int32_t mf_dim;                         /* NeuMF: GMF embedding dim M (0: plain MLP) */
    /* NeuMF GMF tables embedding_user_mf / embedding_item_mf [U, M], [I, M] + optimizer state */
    float *mf_user_w, *mf_item_w, *mf_user_m, *mf_user_v, *mf_item_m, *mf_item_v;
} rg_ncf_model_t;

typedef struct rg_ncf_work {
    float *contrib;                         /* [tiles * rows_per_tile * 2E] per-example input gradients */
    float *mlp_partials;                    /* [rg_ncf_blocks * rg_ncf_mlp_len] */
    float *scores;                          /* [tiles * rows_per_tile] (scores phase) */
    float *dp;                              /* [tiles * rows_per_tile] (given-dp phase) */
    const uint8_t *mask_pos, *mask_neg;     /* recorded dropout masks [rows][rg_ncf_mask_units] or null */
    uint64_t seed;                          /* dropout hash seed when no masks are given */
    int32_t training;                       /* 0: eval (no dropout) */
    int32_t tile_rows;                      /* rg_ncf_rows_per_tile(dim, mf_dim): the layout of
                                               contrib / scores / dp (rg_ncf_pairs checks it) */
    /* NeuMF only: per-example GMF gradient rows [tiles * rows_per_tile * 2M] (user | item),
     * overflow rows [(U + I) * M] (zero between steps), planned positive partials [cols * M] */
    float *mf_contrib;
    int64_t *mf_hot_grad;                   /* int64 fixed point, as rg_mf_work_t.hot_grad */
    float *mf_part_row;
} rg_ncf_work_t;

int64_t rg_ncf_mlp_len(int32_t dim);
/* NeuMF flat parameters (tower layers, then affine_output (1 x (8 + M)) and its bias) */
int64_t rg_neumf_param_len(int32_t dim, int32_t mf_dim);
int64_t rg_ncf_mask_units(int32_t dim);
/* Tile geometry of a model: rows per tile (48 for the E = 64 MLP's wave kernel since round 5,
 * RG_NCF_WAVE_ROWS; 32 for the other towers and NeuMF), columns per tile (also the plan's units
 * per block), tiles.
 * ABI 2 (rg_version "abi=2"): these three take (dim, mf_dim) / (n_neg, dim, mf_dim) /
 * (cols, n_neg, dim, mf_dim); ABI 1 took fewer arguments. */
int64_t rg_ncf_rows_per_tile(int32_t dim, int32_t mf_dim);
int64_t rg_ncf_cols_per_tile(int32_t n_neg, int32_t dim, int32_t mf_dim);
int64_t rg_ncf_tiles(int64_t cols, int32_t n_neg, int32_t dim, int32_t mf_dim);
/* workgroups of rg_ncf_pairs (= weight-gradient partials): tiles, capped at 256 x the workgroups
 * per CU that the dim's LDS allows (1 for the E = 64 MLP, up to 4) */
int64_t rg_ncf_blocks(int64_t cols, int32_t n_neg, int32_t dim, int32_t mf_dim);
/* phase 0: fused step (pointwise / bpr / hinge); 1: forward scores only; 2: fused with given dL/dp;
 * 3: forward + loss partials only (validation, run with training = 0) */
int rg_ncf_pairs(void *stream, const rg_ncf_model_t *model, const rg_mf_batch_t *batch, rg_mf_work_t *work,
                 rg_ncf_work_t *ncf_work, int32_t phase);
int rg_ncf_adapt_dp(void *stream, const rg_mf_batch_t *batch, rg_ncf_work_t *ncf_work, float *loss_partials);
/* Adaptive hinge over several ranks (data-parallel NCF / NeuMF): this rank's largest
 * negative (score, draw index) into slot `rank` of a zeroed [world * 4] float buffer
 * (the caller then SUM all-reduces it: one writer per slot, so it acts as an all-gather),
 * its local row in *local_row; then the positives' dp against the global maximum, this
 * rank's active-positive count in *count (SUM all-reduce it) and loss share; then the
 * winning rank sets the maximum's dp = global count / global_pos. */
int rg_ncf_adapt_local(void *stream, const rg_mf_batch_t *b, const rg_mf_work_t *w, rg_ncf_work_t *nw,
                       float *slots, int32_t rank, int32_t world, int32_t *local_row);
int rg_ncf_adapt_global(void *stream, const rg_mf_batch_t *b, rg_ncf_work_t *nw, const float *slots,
                        int32_t world, float *count, float *loss_partials);
int rg_ncf_adapt_winner(void *stream, const rg_mf_batch_t *b, rg_ncf_work_t *nw, const float *slots,
                        int32_t world, int32_t rank, const int32_t *local_row, const float *count);
int rg_ncf_update(void *stream, const rg_ncf_model_t *model, const rg_ncf_work_t *ncf_work, int64_t nparts,
                  const rg_opt_t *opt, const float *loss_partials, const rg_mf_loss_t *loss);
/* Data-parallel NCF / NeuMF step (replicated, reference-exact: R ranks take column slices of
 * the global batch of ONE draw stream and equal the single process at batch R*B):
 *   rg_ncf_mlp_grad   the MLP weight-gradient reduce of rg_ncf_update without the update:
 *                     grad[0, P) and this rank's loss share (loss->inv_*: global means) in grad[P]
 *   rg_ncf_grads      the embedding rows' data gradient pulled into grad = [nr*D | nr | 0]
 *                     (nr = row_end - row_begin; gmf = 1: NeuMF GMF tables, whose lists are kept
 *                     for the MLP tables' pass that follows)
 * the caller all-reduces the buffers, then
 *   rg_ncf_mlp_apply  the MLP update from grad (loss_out <- grad[P]),
 *   rg_ncf_apply_dense every row's in-place update from its summed gradient. */
int rg_ncf_mlp_grad(void *stream, const rg_ncf_model_t *model, const rg_ncf_work_t *ncf_work, int64_t nparts,
                    const float *loss_partials, const rg_mf_loss_t *loss, float *grad);
int rg_ncf_mlp_apply(void *stream, const rg_ncf_model_t *model, const float *grad, const rg_opt_t *opt,
                     float *loss_out);
int rg_ncf_grads(void *stream, const rg_ncf_model_t *model, rg_mf_work_t *work, const rg_ncf_work_t *ncf_work,
                 float *grad, int64_t row_begin, int64_t row_end, int32_t gmf);
int rg_ncf_apply_dense(void *stream, const rg_ncf_model_t *model, const float *grad, const rg_opt_t *opt,
                       int64_t row_begin, int64_t row_end, int32_t gmf);
/* Embedding rows [row_begin, row_end) (users then items): pull + optimizer, in place. */
int rg_ncf_apply(void *stream, const rg_ncf_model_t *model, rg_mf_work_t *work, const float *contrib,
                 const rg_opt_t *opt, int64_t row_begin, int64_t row_end);
/* The tail of a single-GPU NCF / NeuMF step in ONE launch (NeuMF: after its GMF tables' pass,
 * a launch of its own, as in rg_neumf_apply): the next step's
 * prepare (rg_mf_prepare of next / next_work; next = NULL: none), rg_ncf_update (the MLP
 * weight-gradient reduce + optimizer, with the step's loss) and rg_ncf_apply (every embedding
 * row's pull + optimizer) -- the same sums as the three separate calls; gen (optional, from
 * rg_mf_stepper_tail_gen): a later unit's MT walk in the launch's first workgroup. */
int rg_ncf_tail(void *stream, const rg_ncf_model_t *model, rg_mf_work_t *work, const rg_ncf_work_t *ncf_work,
                int64_t nparts, const rg_opt_t *opt, const float *loss_partials, const rg_mf_loss_t *loss,
                const rg_mf_batch_t *next, const rg_mf_work_t *next_work, const rg_mt_gen_t *gen);
/* Every check rg_ncf_tail makes that does not depend on the stepper's outputs (next, gen), with no
 * launch: call it BEFORE rg_mf_stepper_prefetch_args / rg_mf_stepper_tail_gen, which commit the
 * next unit and the MT ring slot, so a tail that would be refused never leaves the stepper holding
 * a prepare or a walk that was not launched.  RG_OK or the status rg_ncf_tail would return. */
int rg_ncf_tail_validate(const rg_ncf_model_t *model, rg_mf_work_t *work, const rg_ncf_work_t *ncf_work,
                         int64_t nparts, const rg_opt_t *opt, const float *loss_partials, const rg_mf_loss_t *loss);
/* NeuMF (spotlight/dnn_models/neuMF.py:7-55): rg_ncf_pairs / rg_ncf_update run with
 * model->mf_dim > 0 (the affine_output sees cat(tower, U_mf[u] * I_mf[i])); this applies
 * the GMF tables, then the MLP tables (as rg_ncf_apply). */
#define RG_NEUMF_MAX_MF_DIM 128
int rg_neumf_apply(void *stream, const rg_ncf_model_t *model, rg_mf_work_t *work, const rg_ncf_work_t *ncf_work,
                   const rg_opt_t *opt, int64_t row_begin, int64_t row_end);

/* ------------------------------------------------------------------------------
 * Evaluation top-k (rg_eval.hip): the first k entries of argsort(-scores) per row, as
 * precision_recall_score / hit_ratio / map_at_k read them (spotlight/evaluation.py:
 * 108-213, 278-353).  scores [rows][ld] (device, fp32), out_idx [rows][k] (device,
 * int32, rank order; equal scores: lower column first; NaN ranks last), 1 <= k <= 32.
 * ---------------------------------------------------------------------------- */
int rg_topk_rows(void *stream, const float *scores, int64_t rows, int64_t cols, int64_t ld, int32_t k,
                 int32_t *out_idx);

/* ------------------------------------------------------------------------------
 * Negative pool (rg_pool.cpp, host code): spotlight/sampling.py:46-70
 * get_negative_samples, continuing NumPy's legacy global MT19937 (mt_key[624], mt_pos
 * from np.random.get_state(), advanced in place).  users / items of n draws
 * (np.random.choice), then the has_key redraws in index order against the training CSR
 * (indptr [U + 1], column-sorted indices, summed ratings; all three null: no redraws).
 * ---------------------------------------------------------------------------- */
int rg_pool_build(uint32_t *mt_key, int32_t *mt_pos, int64_t n, int64_t num_users, int64_t num_items,
                  const int64_t *indptr, const int32_t *indices, const float *ratings, int64_t *out_users,
                  int64_t *out_items);

/* ---------------------------------------------------------------- cGAN (C4)
 * The generator / discriminator of spotlight/dnn_models/cGAN_models.py as
 * slate_generation.py:46-54 builds them (G hidden [H/2, H], D hidden [2H, H, H/2])
 * and the two training iterations of CGANs.py (rg_gan.hip, GEMMs in rg_gemm.hip):
 *   rg_gan_d_step  replaces CGAN.train_discriminator_iteration (CGANs.py:410-457)
 *   rg_gan_g_step  replaces CGAN.train_generator_iteration     (CGANs.py:370-408)
 *   rg_gan_generate replaces generator.forward(inference=True) (cGAN_models.py:52-62)
 * Parameters live in two flat fp32 buffers laid out by rg_gan_layout (blocks in the
 * reference's tensor order; D's layers.0.weight is split into its E history
 * columns W1E and its S*N slate columns W1S, row stride ks); optimizer state
 * buffers (m, v) cover [0, g_off[RG_GAN_G_RM1]) and [0, d_off[RG_GAN_D_END]). */
typedef struct rg_gan_dims {
    int32_t num_items;   /* N; the padding id (history) is N */
    int32_t slate_size;  /* S */
    int32_t hidden;      /* H (gan_hidden_layer) */
    int32_t emb_dim;     /* E (gan_embedding_dim) */
    int32_t z_dim;       /* Z (noise_dim, 100) */
    int32_t batch_max;   /* largest batch a workspace serves */
} rg_gan_dims_t;

enum rg_gan_g_block {
    RG_GAN_G_WH = 0,   /* mult_heads.head_s.weight stacked: [S*N][H] (+ zero rows up to ks) */
    RG_GAN_G_BH,       /* mult_heads.head_s.bias stacked: [S*N] (+ zeros up to ks) */
    RG_GAN_G_EMB,      /* embedding_layer.weight [N+1][E] */
    RG_GAN_G_W1,       /* layers.0.weight [H/2][kz] (kz = Z+E rounded up to 4, zero pad) */
    RG_GAN_G_B1, RG_GAN_G_GAMMA1, RG_GAN_G_BETA1,
    RG_GAN_G_W2,       /* layers.4.weight [H][H/2] */
    RG_GAN_G_B2, RG_GAN_G_GAMMA2, RG_GAN_G_BETA2,
    RG_GAN_G_RM1, RG_GAN_G_RV1, RG_GAN_G_RM2, RG_GAN_G_RV2,   /* BatchNorm buffers (not optimized) */
    RG_GAN_G_END
};
enum rg_gan_d_block {
    RG_GAN_D_W1S = 0,  /* layers.0.weight[:, E:] [2H][ks] (ks = S*N rounded up to 4) */
    RG_GAN_D_EMB,      /* embedding_layer.weight [N+1][E] */
    RG_GAN_D_W1E,      /* layers.0.weight[:, :E] [2H][E] */
    RG_GAN_D_B1, RG_GAN_D_W2, RG_GAN_D_B2, RG_GAN_D_W3, RG_GAN_D_B3, RG_GAN_D_W4, RG_GAN_D_B4,
    RG_GAN_D_END
};
enum rg_gan_ws_view {
    RG_GAN_WS_FAKE = 0,   /* G(z) of the last step: [rows][ks] */
    RG_GAN_WS_DOUT,       /* D outputs of the last step: D step [real rows | fake rows], G step [fake rows] */
    RG_GAN_WS_END
};

/* Offsets (floats) of the blocks; g_off[RG_GAN_G_END] / d_off[RG_GAN_D_END] are the
 * buffer lengths.  strides[0] = kz, strides[1] = ks. */
int rg_gan_layout(const rg_gan_dims_t *dims, int64_t *g_off, int64_t *d_off, int64_t *strides);
/* The workspace must be zero-filled once before its first use (padding columns are
 * read as zeros and never written). */
int64_t rg_gan_workspace_bytes(const rg_gan_dims_t *dims);
/* Offset (bytes) of a named intermediate inside the workspace. */
int64_t rg_gan_workspace_offset(const rg_gan_dims_t *dims, int32_t view);

typedef struct rg_gan_model {
    rg_gan_dims_t dims;
    float *g, *g_m, *g_v;   /* m / v may be NULL when the optimizer does not use them */
    float *d, *d_m, *d_v;
} rg_gan_model_t;

typedef struct rg_gan_batch {
    int32_t rows;                  /* <= dims.batch_max */
    int32_t hist_len;              /* L */
    const int32_t *hist;           /* [rows][L] item ids, padding = N */
    const int32_t *slates;         /* [rows][S] real slates (D step) */
    /* history items grouped for the embedding backward (deterministic order):
     * unique items [n_hist_items], offsets [n_hist_items + 1], batch rows */
    const int32_t *hist_items, *hist_off, *hist_rows;
    int32_t n_hist_items;
    int32_t n_hits;                /* rows * S */
    /* real-slate columns s*N + slates[b][s], sorted by (column, b), and their rows;
     * hit_tile_off[t] = first hit with column >= 128 t, t = 0 .. ceil(S*N / 128) */
    const int32_t *hit_col, *hit_row, *hit_tile_off;
} rg_gan_batch_t;

typedef struct rg_gan_noise {
    const float *z;                /* [rows][Z] uniform [0, 1) (torch.rand) */
    /* recorded dropout masks [rows][width] in the reference's call order
     * (D step: D(real) x3, G x2, D(fake) x3; G step: G x2, D(fake) x3), or NULL:
     * then a counter-based hash of (seed, call, layer, row, unit) keeps with 1 - p */
    const uint8_t *masks[8];
    uint64_t seed;
} rg_gan_noise_t;

/* out: [0] d_loss = mean D(fake) - mean D(real), [1] mean D(real), [2] mean D(fake). */
int rg_gan_d_step(void *stream, const rg_gan_model_t *model, void *workspace, const rg_gan_batch_t *batch,
                  const rg_gan_noise_t *noise, const rg_opt_t *opt, float *out);
/* out: [0] g_loss = -mean D(G(z)).  slates (optional, [rows][S] float item ids): the
 * eval-mode generator on the same z after the update (CGANs.py:404-406). */
int rg_gan_g_step(void *stream, const rg_gan_model_t *model, void *workspace, const rg_gan_batch_t *batch,
                  const rg_gan_noise_t *noise, const rg_opt_t *opt, float *out, float *slates);
/* Eval-mode generator (BatchNorm running stats, no dropout): argmax slates [rows][S]. */
int rg_gan_generate(void *stream, const rg_gan_model_t *model, void *workspace, const rg_gan_batch_t *batch,
                    const float *z, float *slates);

/* fp32 MFMA GEMM used by the cGAN (test entry): C = A B^T with A [M][K] (a_kmajor) or
 * [K][M], B [N][K] (b_kmajor) or [K][N]; post 0 none / 1 tanh; splits > 1 uses work
 * [splits * M * N] and a fixed-order reduction. */
int rg_gemm_f32(void *stream, const float *A, int64_t lda, int32_t a_kmajor, const float *B, int64_t ldb,
                int32_t b_kmajor, int64_t M, int64_t N, int64_t K, float *C, int64_t ldc, const float *bias,
                int32_t post, int32_t splits, float *work);

/* The cGAN's weight-gradient GEMM fused with an in-place RMSprop update of P [M][N]
 * (row stride ldp) and its square average V (test / measurement entry). */
int rg_gemm_f32_rms(void *stream, const float *A, int64_t lda, int32_t a_kmajor, const float *B, int64_t ldb,
                    int32_t b_kmajor, int64_t M, int64_t N, int64_t K, float *P, float *V, int64_t ldp, float lr,
                    float alpha, float eps);

/* The optimizer GEMM's form (W1S / WH weight gradient fused with the update; test /
 * measurement entry): mode 0 the 3-workgroup-per-CU kernel with the update in its epilogue
 * (the product), 1 the wave-specialised persistent kernel (matrix, loader and update waves of
 * one workgroup overlap; measured slower, A/B build only: -1 and rg_last_error elsewhere),
 * < 0 leaves it.  Returns the form in force before the call.  Both give identical bits. */
int rg_gemm_ws_mode(int32_t mode);

/* Milliseconds between two timing events (hipEvent_t) recorded on a stream. */
int rg_event_elapsed_ms(void *ev_begin, void *ev_end, float *ms);

/* Thread-local description of the last error. */
const char *rg_last_error(void);

/* Library build identification (gfx target, ABI version). */
const char *rg_version(void);
/* Build flags: RG_BUILD_AB = an A/B build (build.py --variant NAME -DRG_AB=1) carrying the
 * measured-slower alternatives behind RG_* environment switches; the product
 * library returns 0 and reads none of those switches. */
#define RG_BUILD_AB 1
int32_t rg_build_flags(void);

#ifdef __cplusplus
}
#endif
#endif /* RG_HIP_H */
