/*
 * mf_hip.h -- C ABI of libmf_hip.so, the MI355X (gfx950) implementation of
 * the SGD latent-factor update loop of SHEEPididoo/matrix-factorization.
 *
 * Drop-in boundary.  The reference crosses from Python into native (numba
 * JIT) code at exactly three functions of
 * matrix_factorization/kernel_matrix_factorization.py and four of
 * matrix_factorization/baseline_model.py; each entry point below replaces
 * one of them (file:line of the reference cited per function).  The
 * reference passes NumPy arrays that the callee mutates in place; here the
 * caller passes device pointers (HBM, e.g. torch-ROCm tensor storage) that
 * the callee mutates in place, plus an explicit hipStream_t.
 *
 * Conventions
 *   - every function returns 0 on success, a MF_ERR_* code otherwise;
 *     mf_last_error() returns a thread-local message for the last failure;
 *   - device pointers are caller-owned; no entry point allocates device
 *     memory except where a workspace size is documented;
 *   - `dtype` selects the parameter/rating storage type: MF_F32 or MF_F64;
 *     ids are int32 (internal ids 0..n-1, -1 = unknown where allowed);
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *     all kernels are enqueued asynchronously on it, no host sync unless the
 *     optional timing output is requested;
 *   - host-side schedulers (mf_sched_*) take host pointers and never touch
 *     the GPU.
 */
#ifndef MF_HIP_H
#define MF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MF_ABI_VERSION 1

enum {
    MF_OK = 0,
    MF_ERR_INVALID = 1,   /* bad argument (shape, enum, range)             */
    MF_ERR_HIP = 2,       /* HIP runtime error                             */
    MF_ERR_CAPACITY = 3,  /* caller-provided output buffer too small        */
    MF_ERR_NOMEM = 4      /* host allocation failed (schedulers)            */
};

enum { MF_F32 = 0, MF_F64 = 1 };

/* kernel codes: KernelMF(kernel=...) kernel_matrix_factorization.py:56,66 */
enum { MF_LINEAR = 0, MF_SIGMOID = 1, MF_RBF = 2 };

/* flags for mf_sgd_epoch */
enum {
    MF_FLAG_XCD_SWIZZLE = 1,  /* map consecutive tiles of a batch onto one XCD */
    MF_FLAG_NT_USER = 2,      /* stream user rows/biases/triples non-temporally */
    MF_FLAG_NT_ITEM = 4,      /* (unused by the current kernels)                */
    MF_FLAG_XCD_CLAIM = 8,    /* workgroups claim the tiles of the item slice of
                                 the XCD they run on (needs `workspace`)        */
    MF_FLAG_PERSISTENT = 16,  /* mf_sgd_epoch_strata: the whole epoch in one
                                 launch, item slabs resident in LDS (needs
                                 `workspace`; falls back to one launch per
                                 stratum when the grid cannot be co-resident) */
    MF_FLAG_DEEP_PIPE = 32,   /* with MF_FLAG_PERSISTENT: user rows gathered two
                                 steps ahead (blocks of few steps)               */
    MF_FLAG_NO_COOP = 64,     /* with MF_FLAG_PERSISTENT: plain launch instead of
                                 hipLaunchCooperativeKernel (diagnostic A/B; the
                                 occupancy check is then the only guard)         */
    MF_FLAG_NARROW = 128,     /* strata: a plan built for mf_strata_slots_waves(k,
                                 dtype, 4) runs on 4-wave workgroups whose lane
                                 groups are half as wide (two vectors per lane;
                                 FP32, n_factors a multiple of 4 up to 32) */
    MF_FLAG_L2_HANDOFF = 256, /* with MF_FLAG_PERSISTENT and an XCD-class stratum
                                 order: a block whose user range goes next to a
                                 workgroup on the SAME XCD (checked at run time
                                 from the XCC ids the workgroups publish) stores
                                 its user rows plainly, so they stay in that
                                 XCD's L2 for the successor's loads; before a
                                 hand-off to another XCD the producer writes its
                                 XCD's L2 back (agent release).  Needs rows of a
                                 whole number of 128-B lines and a 128-B aligned
                                 P; ignored otherwise (and with user-range
                                 classes C > 1). */
    MF_FLAG_NO_EARLY_POLL = 512, /* with MF_FLAG_PERSISTENT and classes C > 1: wait
                                 for each position's user range at its start
                                 instead of polling it once during the previous
                                 block (diagnostic A/B) */
    MF_FLAG_STREAM = 1024,    /* with MF_FLAG_PERSISTENT, MF_FLAG_DEEP_PIPE and
                                 classes C > 1: the stream form -- one software
                                 pipeline through all positions of the launch
                                 (the next block's triples and user rows loaded
                                 while the current block's last steps apply,
                                 the bias slices double-buffered in LDS); the
                                 same sequential order, bit for bit */
    MF_FLAG_PREPARE = 2048,   /* mf_sgd_epoch_strata: no launch -- only the
                                 launcher's one-time runtime work for this plan
                                 (kernel attributes, the co-residency query),
                                 so the first epoch does not pay it; the
                                 parameter pointers are not touched */
    /* mf_sgd_epoch_strata: bits 24..27 = C - 1, the plan's user-range classes
       (mf_strata_plan_build_classes; 0 = C = 1, the plain B x B plan) */
    MF_FLAG_CLASSES_SHIFT = 24
};
/* Jobs of one mf_permute_rows launch. */
#define MF_PERMUTE_MAX_JOBS 4
/* Largest number of user-range classes a strata plan may have. */
#define MF_STRATA_MAX_CLASSES 4

const char* mf_last_error(void);
int mf_abi_version(void);
/* One empty kernel launch per translation unit of this library on `stream`,
 * and one cooperative launch: makes the runtime load the code objects for
 * the current device now (the engine calls it while it is built) instead of
 * inside the first training epoch.  flags & MF_FLAG_NO_COOP: no cooperative
 * launch (rocprofv3's dispatch interception crashes on one). */
int mf_warmup(int32_t flags, void* stream);
/* Up to MF_PERMUTE_MAX_JOBS row arrays permuted in one launch (the relabelled
 * strata plans' parameter moves): job j has n_rows[j]
 * rows of row_bytes[j] bytes (a multiple of 4); mode 0 gathers dst[r] =
 * src[idx[r]], mode 1 scatters dst[idx[r]] = src[r].  DEVICE pointers in
 * HOST arrays of n_jobs; idx[j] has n_rows[j] entries in [0, n_rows[j]). */
int mf_permute_rows(int32_t n_jobs, void* const* dst, const void* const* src,
                    const int64_t* const* idx, const int64_t* n_rows,
                    const int32_t* row_bytes, int32_t mode, void* stream);
/* Largest n_factors the kernels accept (inclusive). */
int mf_max_factors(void);

/*
 * One SGD epoch over a conflict-free batch schedule.
 *
 * Replaces the body of one epoch of `_sgd`
 * (kernel_matrix_factorization.py:369-425: the sweep that calls
 * kernel_{linear,sigmoid,rbf}_sgd_update, kernels.py:108-327, once per
 * rating).  The reference visits ratings in one sequential order.  Here that
 * order is given as batches: batch b holds the ratings at schedule positions
 * [batch_offsets[b], batch_offsets[b+1]); no two ratings of a batch share a
 * user row (when update_user_params) or an item row (when
 * update_item_params), so every batch is applied in parallel and the result
 * equals the sequential sweep in the order
 *     batch_seq[0], batch_seq[1], ...   (each batch in any internal order).
 * The schedulers below produce such batches (exactly for a given
 * permutation, or by edge colouring for throughput).
 *
 *   user_ids, item_ids, ratings  device, n_ratings each (ratings: dtype)
 *   order          device, nullable: schedule position -> rating index; when
 *                  NULL, position p is rating p (ratings pre-sorted)
 *   batch_offsets  HOST, n_batches + 1 positions (non-decreasing, last <= n)
 *   batch_seq      HOST, nullable, n_seq batch indices: launch order (a full
 *                  epoch passes a permutation of 0..n_batches-1; a prefix
 *                  applies a partial epoch).  NULL = 0, 1, ..., n_batches-1
 *                  and n_seq is ignored
 *   user_biases / item_biases      device, dtype, n_users / n_items
 *   user_features / item_features  device, dtype, row-major
 *                  (n_users, n_factors) / (n_items, n_factors)
 *   kernel, gamma, lr, reg, min_rating, max_rating
 *                  as KernelMF (a = min_rating, c = max_rating - min_rating,
 *                  kernel_matrix_factorization.py:405-406)
 *   update_user_params / update_item_params   as _sgd (:336-337)
 *   flags          MF_FLAG_* bits; bits 16..23 = timing stride S (0 = 1)
 *   workspace      device, nullable: >= mf_sgd_workspace_bytes(launches)
 *                  bytes, required by MF_FLAG_XCD_CLAIM (tile counters,
 *                  zeroed by the call on `stream`)
 *   kernel_ms      host, nullable, 2 doubles: when given, every S-th launch
 *                  is bracketed by hipEvents on `stream`, the stream is
 *                  synchronised, kernel_ms[0] = summed time (ms) of the
 *                  bracketed launches and kernel_ms[1] = their count.
 */
int mf_sgd_epoch(const int32_t* user_ids, const int32_t* item_ids,
                 const void* ratings, int64_t n_ratings, const int32_t* order,
                 const int64_t* batch_offsets, int32_t n_batches,
                 const int32_t* batch_seq, int32_t n_seq,
                 double global_mean, void* user_biases,
                 void* item_biases, void* user_features, void* item_features,
                 int32_t n_users, int32_t n_items, int32_t n_factors,
                 int32_t kernel, int32_t dtype, double gamma, double lr,
                 double reg, double min_rating, double max_rating,
                 int32_t update_user_params, int32_t update_item_params,
                 int32_t flags, void* workspace, size_t workspace_bytes,
                 void* stream, double* kernel_ms);
size_t mf_sgd_workspace_bytes(int32_t n_launch);

/*
 * One epoch (or the strata listed in strata_seq) of the STRATIFIED sweep:
 * the throughput form of `_sgd`'s loop (kernel_matrix_factorization.py:
 * 371-425), same per-rating updates (kernels.py:108-327).  The plan comes
 * from mf_strata_plan_build: B user ranges and B item ranges
 * (user_bounds/item_bounds, DEVICE, B+1 each); block (s, w) = user range
 * (w+s) mod B x item range w is a grid of (block_steps[s*B+w+1] -
 * block_steps[s*B+w]) steps x n_slots rating slots (block_steps: DEVICE,
 * B*B+1); the triples (user_ids/item_ids/ratings, DEVICE, n_positions =
 * block_steps[B*B] * n_slots each) are stored in plan order, an idle slot
 * holding user id -1.  n_slots must equal mf_strata_slots(n_factors, dtype).
 * Stratum strata_seq[t] (HOST, n_seq entries) is one launch of B
 * workgroups; workgroup w stages item range w (rows + biases) and the bias
 * slice of its user range in LDS and applies the block's steps starting at
 * step (mix(seed, block) mod n_steps), one LDS barrier apart.
 * max_block_items / max_block_users size the LDS (mf_strata_lds_bytes must
 * not exceed mf_strata_lds_limit()).  flags: MF_FLAG_PERSISTENT runs the
 * strata of strata_seq in ONE launch: workgroup w keeps item slab w in LDS
 * throughout and, before each stratum, waits for the workgroup that last
 * applied the same user range (bounded wait; on timeout it sets an error
 * flag that mf_strata_status reports); it needs workspace (DEVICE, >=
 * mf_strata_workspace_bytes(n_blocks, n_seq) bytes, zero-initialised once by
 * the caller -- and zeroed WHOLE again after a reported failure, since the
 * position counters in it grow across launches) and is used only when
 * n_seq <= 256 and all n_blocks workgroups fit on the device at once, else
 * the call falls back to one launch per stratum.  The result
 * is the same sequential order either way.  kernel_ms (HOST, optional):
 * elapsed ms of the whole call and the launch count (synchronises).
 *
 * User-range classes (flags bits 24..27 = C - 1, a plan from
 * mf_strata_plan_build_classes): C*B user ranges, B item ranges, C*B strata;
 * block (s, w) = user range (s + C*w) mod C*B x item range w, so stratum s
 * touches the user ranges of class s mod C only.  The persistent kernel
 * then needs strata_seq to cycle through the classes (seq[t] mod C ==
 * seq[t mod C] mod C, the first C entries of distinct classes): a user range
 * used at position t was last used at t - C, so every hand-off has C - 1
 * whole blocks of slack (no waiting on the chain's jitter); any other order
 * runs as one launch per stratum.  n_seq may then be up to 1024.
 */
int mf_sgd_epoch_strata(const int32_t* user_ids, const int32_t* item_ids,
                        const void* ratings, int64_t n_positions, int32_t n_blocks,
                        const int32_t* user_bounds, const int32_t* item_bounds,
                        const int64_t* block_steps, int32_t n_slots,
                        int32_t max_block_items, int32_t max_block_users,
                        const int32_t* strata_seq, int32_t n_seq, uint32_t seed,
                        double global_mean, void* user_biases, void* item_biases,
                        void* user_features, void* item_features, int32_t n_users,
                        int32_t n_items, int32_t n_factors, int32_t kernel, int32_t dtype,
                        double gamma, double lr, double reg, double min_rating,
                        double max_rating, int32_t update_user_params,
                        int32_t update_item_params, int32_t flags, void* workspace,
                        size_t workspace_bytes, void* stream, double* kernel_ms);
/*
 * The same epoch in DELTA-OUT form, for user-sharded data parallelism (every
 * rank holds a replica of the item rows and biases; no
 * counterpart in the single-process reference): item_features / item_biases
 * are left at their values before the call, and item_delta (DEVICE, n_items
 * x n_factors) / item_bias_delta (DEVICE, n_items; unused by rbf) receive
 * the local update (value after the epoch - value before).  The caller
 * all-reduces the deltas and adds them damped with mf_replica_apply, scale =
 * min(1/2, 2/world) (distributed.default_delta_scale: the plain sum diverges
 * at N >= 4 on C3).  This is the "delta" exchange; the default "rotate"
 * exchange needs no delta form (ranks pass item ranges instead, each applied
 * in place by mf_sgd_epoch_strata on its rows of Q / b_i).
 * The persistent kernel writes the delta where it would write the slab back;
 * the per-stratum fallback keeps the start values in the delta buffers and
 * swaps at the end.  User rows and biases are updated in place as usual.
 */
int mf_sgd_epoch_strata_delta(const int32_t* user_ids, const int32_t* item_ids,
                              const void* ratings, int64_t n_positions, int32_t n_blocks,
                              const int32_t* user_bounds, const int32_t* item_bounds,
                              const int64_t* block_steps, int32_t n_slots,
                              int32_t max_block_items, int32_t max_block_users,
                              const int32_t* strata_seq, int32_t n_seq, uint32_t seed,
                              double global_mean, void* user_biases, void* item_biases,
                              void* user_features, void* item_features, int32_t n_users,
                              int32_t n_items, int32_t n_factors, int32_t kernel,
                              int32_t dtype, double gamma, double lr, double reg,
                              double min_rating, double max_rating,
                              int32_t update_user_params, int32_t update_item_params,
                              int32_t flags, void* workspace, size_t workspace_bytes,
                              void* item_delta, void* item_bias_delta, void* stream,
                              double* kernel_ms);
size_t mf_strata_workspace_bytes(int32_t n_blocks, int32_t n_seq);
/* Synchronises `stream` and reports whether a persistent strata sweep using
 * `workspace` gave up waiting (MF_ERR_HIP) since the workspace was zeroed. */
int mf_strata_status(const void* workspace, int32_t n_blocks, void* stream);
size_t mf_strata_lds_bytes(int32_t max_block_items, int32_t max_block_users,
                           int32_t n_factors, int32_t dtype);
int32_t mf_strata_lds_limit(void);
/* Diagnostic (tools/strata_probe.py): when `probe` (DEVICE, 4 * n_seq * B
 * int64) is set, the persistent strata kernel records s_memrealtime stamps
 * (100 MHz) per (position t, workgroup w) at [(t*B + w)*4 + q]: q = 0 wait
 * start, 1 wait end, 2 block end, 3 signal.  NULL turns it off (default). */
int mf_strata_set_probe(int64_t* probe);
/* Test hook: the next n_launches persistent strata launches of this process
 * start with their error word set, as if a neighbour wait had timed out, so
 * callers can exercise their recovery (KernelMF.fit / distributed.fit_sharded
 * replay the epochs as per-stratum launches).  0 turns it off. */
int mf_strata_inject_fail(int32_t n_launches);
/* Rating slots per step of the strata kernel for (n_factors, dtype); -1 on
 * invalid arguments. */
int32_t mf_strata_slots(int32_t n_factors, int32_t dtype);
/* The same for a workgroup of `waves` waves: 16 (the default) or, FP32 with
 * n_factors <= 64 or FP64 with n_factors <= 64, 8 -- a plan built with that
 * many slots runs the
 * 8-wave kernels (blocks whose step count is set by the item degree, not by
 * the slot count); 4 = the narrow form of the 8-wave plan (same slot count,
 * run with MF_FLAG_NARROW; FP32, n_factors a multiple of 4 up to 32); -1
 * where the layout has no such kernels. */
int32_t mf_strata_slots_waves(int32_t n_factors, int32_t dtype, int32_t waves);

/*
 * Sum of squared training errors, sum_j (r_j - pred_j)^2, accumulated in
 * FP64 -- replaces `_calculate_rmse` (kernel_matrix_factorization.py:240-317;
 * rmse = sqrt(sse / n_ratings), :315).  The sum is written to the DEVICE
 * double *sse_out (no host sync).  `workspace` is a device buffer of at
 * least mf_sse_workspace_bytes(n_ratings) bytes.  Deterministic: the same
 * inputs give the same bits.
 * slice_offsets (HOST, nullable, n_slices + 1 <= 129 entries): the ratings
 * are ordered by mf_sched_slices; slice x is walked by the workgroups
 * b % n_slices == x (XCD-local Q slices).  NULL = one slice.  n_slices > 8
 * and a multiple of 8 (mf_sched_tiles): the tiles are walked in phases of 8,
 * by a resident grid for FP64 (MF_SSE_PHASED=0: dispatch-ordered phases).
 * n_users / n_items: rows of user_features / item_features (every id must
 * be below them).
 */
size_t mf_sse_workspace_bytes(int64_t n_ratings);
int mf_sse(const int32_t* user_ids, const int32_t* item_ids,
           const void* ratings, int64_t n_ratings, double global_mean,
           const void* user_biases, const void* item_biases,
           const void* user_features, const void* item_features,
           int32_t n_users, int32_t n_items,
           int32_t n_factors, int32_t kernel, int32_t dtype, double gamma,
           double min_rating, double max_rating,
           const int64_t* slice_offsets, int32_t n_slices, void* workspace,
           double* sse_out, void* stream);
/* mf_sse with its grid capped at max_blocks workgroups of 256 threads (0 = no
 * cap; at least n_slices): the pass then leaves CUs free for a kernel running
 * beside it on another stream (the rotation schedule runs epoch e's RMSE
 * beside epoch e+1's sub-epochs).  The same sum up to
 * FP64 rounding (another grouping of the per-workgroup partial sums). */
int mf_sse_capped(const int32_t* user_ids, const int32_t* item_ids,
                  const void* ratings, int64_t n_ratings, double global_mean,
                  const void* user_biases, const void* item_biases,
                  const void* user_features, const void* item_features,
                  int32_t n_users, int32_t n_items,
                  int32_t n_factors, int32_t kernel, int32_t dtype, double gamma,
                  double min_rating, double max_rating,
                  const int64_t* slice_offsets, int32_t n_slices, void* workspace,
                  int32_t max_blocks, double* sse_out, void* stream);

/*
 * Predictions for (user, item) pairs -- replaces `_predict`
 * (kernel_matrix_factorization.py:448-541).  An id of -1 is unknown: zero
 * bias and an all-zero factor vector (:487-499).  Clipped to
 * [min_rating, max_rating] when bound_ratings (:532-536).  `out` is a device
 * array of n_pairs values of `dtype`.
 */
int mf_predict(const int32_t* user_ids, const int32_t* item_ids,
               int64_t n_pairs, double global_mean, const void* user_biases,
               const void* item_biases, const void* user_features,
               const void* item_features, int32_t n_factors, int32_t kernel,
               int32_t dtype, double gamma, double min_rating,
               double max_rating, int32_t bound_ratings, void* out,
               void* stream);

/*
 * Top-`amount` items for each of n_query users (scores = unbounded
 * prediction of every item, as recommend() scores them,
 * recommender_base.py:245-260).  Exclusions (recommend's items_known,
 * :245-250) as a DEVICE CSR list, both nullable: the items
 * exclude_items[exclude_ptr[q] .. exclude_ptr[q+1]) (int32, each user's list
 * SORTED ASCENDING -- the kernels binary-search it; ids outside [0, n_items)
 * ignored) are skipped for query q.  An unsorted list makes the result
 * undefined (items may come back although listed).  Ties are broken by
 * the lower item id (the order a stable sort_values gives; the reference's
 * default quicksort leaves tie order unspecified, :259).  out_items (int32) /
 * out_scores (dtype): device, n_query * amount.  Rows with fewer than
 * `amount` candidates are padded with id -1.  The workspace grows with
 * n_query * n_items: callers chunk the users.
 * workspace: device, >= mf_topk_workspace_bytes(n_query, n_items, amount).
 */
size_t mf_topk_workspace_bytes(int32_t n_query, int32_t n_items,
                               int32_t amount);
int mf_topk(const int32_t* query_users, int32_t n_query, double global_mean,
            const void* user_biases, const void* item_biases,
            const void* user_features, const void* item_features,
            int32_t n_items, int32_t n_factors, int32_t kernel, int32_t dtype,
            double gamma, double min_rating, double max_rating,
            const int64_t* exclude_ptr, const int32_t* exclude_items,
            int32_t amount, void* workspace,
            int32_t* out_items, void* out_scores, void* stream);

/*
 * The same top-k through an MFMA filter (linear kernel, float32, n_factors a
 * multiple of 4 in [4, 64], 1 <= amount <= 64: mf_topk_mm_supported): scores
 * of 64-user x 32-item tiles on v_mfma_f32_32x32x2_f32 (another summation
 * order than predict) only select candidates -- every item whose exact score
 * can reach the top `amount` within a per-user error bound -- which are then
 * rescored with predict's arithmetic and ranked exactly as mf_topk ranks
 * them.  *overflow (device int32, the caller zeroes it) is OR-ed with 1 when
 * a candidate band outgrew its list (masses of near-equal scores): the
 * results are then not guaranteed and the caller re-runs mf_topk.  Items
 * whose score is NaN are never candidates here (mf_topk ranks them last).
 * Exclusion lists as for mf_topk: each user's list sorted ascending.
 * workspace: device, >= mf_topk_mm_workspace_bytes(n_query, n_items).
 */
int32_t mf_topk_mm_supported(int32_t n_factors, int32_t kernel, int32_t dtype,
                             int32_t amount);
size_t mf_topk_mm_workspace_bytes(int32_t n_query, int32_t n_items);
int mf_topk_mm(const int32_t* query_users, int32_t n_query, double global_mean,
               const void* user_biases, const void* item_biases,
               const void* user_features, const void* item_features,
               int32_t n_items, int32_t n_factors, int32_t kernel, int32_t dtype,
               const int64_t* exclude_ptr, const int32_t* exclude_items,
               int32_t amount, void* workspace, int32_t* out_items,
               void* out_scores, int32_t* overflow, void* stream);

/* ---------------- BaselineModel (bias-only), baseline_model.py ---------- */

/* One bias-SGD epoch over a conflict-free batch schedule: replaces one epoch
 * of baseline_model.py `_sgd` (:250-266).  Same schedule contract as
 * mf_sgd_epoch. */
int mf_bias_sgd_epoch(const int32_t* user_ids, const int32_t* item_ids,
                      const void* ratings, int64_t n_ratings,
                      const int32_t* order, const int64_t* batch_offsets,
                      int32_t n_batches, const int32_t* batch_seq,
                      int32_t n_seq,
                      double global_mean, void* user_biases,
                      void* item_biases, int32_t dtype, double lr, double reg,
                      int32_t update_user_params, int32_t update_item_params,
                      void* stream);

/* Bias-model SSE, replaces baseline_model.py `_calculate_rmse` (:183-212). */
int mf_bias_sse(const int32_t* user_ids, const int32_t* item_ids,
                const void* ratings, int64_t n_ratings, double global_mean,
                const void* user_biases, const void* item_biases,
                int32_t dtype, void* workspace, double* sse_out, void* stream);

/*
 * One alternating-least-squares epoch of the bias model: replaces one epoch
 * of baseline_model.py `_als` (:326-348).  Sums are taken per id in the
 * reference's order through CSR lists:
 *   user_ptr (n_users+1) / user_list: rating indices of each user, ascending
 *   item_ptr (n_items+1) / item_list: rating indices of each item, ascending
 * (all device, int64 ptr / int32 list), so results are bit-identical to the
 * sequential reference loop.  Counts are the list lengths (:317-323).
 */
int mf_bias_als_epoch(const int32_t* user_ids, const int32_t* item_ids,
                      const void* ratings, double global_mean,
                      void* user_biases, void* item_biases, int32_t n_users,
                      int32_t n_items, const int64_t* user_ptr,
                      const int32_t* user_list, const int64_t* item_ptr,
                      const int32_t* item_list, int32_t dtype, double reg,
                      void* stream);

/* Bias-model prediction, replaces baseline_model.py `_predict` (:365-417). */
int mf_bias_predict(const int32_t* user_ids, const int32_t* item_ids,
                    int64_t n_pairs, double global_mean,
                    const void* user_biases, const void* item_biases,
                    int32_t dtype, double min_rating, double max_rating,
                    int32_t bound_ratings, void* out, void* stream);

/* ---------------- factor-model ALS (BASELINE config 5) ------------------ */

/*
 * One half-sweep of alternating least squares for the factor model: solves,
 * for every entity e (users with the item side fixed, or items with the user
 * side fixed), the regularised normal equations of its factor row and bias
 *     (sum_n y_n y_n^T + reg I) [w_e; b_e] = sum_n t_n y_n,
 *     y_n = [other_features[o_n]; 1],  t_n = r_n - global_mean - other_biases[o_n]
 * No reference counterpart: it extends the bias-only ALS of
 * baseline_model.py:283-362 (`_als`, whose per-entity update
 * (reg + n_e) b_e = sum t_n, :328-337, is the k = 0 case) to the latent
 * factors of KernelMF's linear kernel.
 *   entity_ptr      DEVICE, n_entities + 1 (int64): CSR offsets
 *   other_ids       DEVICE, the other side's id per rating, CSR order
 *   ratings         DEVICE, float, CSR order
 *   other_biases / other_features   DEVICE, float, (n_other) / (n_other, k)
 *   biases / features               DEVICE, float, written: (n_entities) /
 *                                   (n_entities, k)
 * Entities without ratings keep their parameters (update_users re-solves
 * only the users present in its data).  The Gramian runs on f32-input MFMA
 * (v_mfma_f32_32x32x2_f32), the solve is an LDS elimination in f32.  dtype must be MF_F32; 1 <= n_factors <=
 * mf_als_max_factors().
 */
int mf_als_sweep(const int64_t* entity_ptr, const int32_t* other_ids,
                 const void* ratings, int32_t n_entities, double global_mean,
                 const void* other_biases, const void* other_features,
                 void* biases, void* features, int32_t n_factors, int32_t dtype,
                 double reg, void* stream);
int32_t mf_als_max_factors(void);
/* Profiling probe: mf_als_sweep that also writes 4 wall-clock stamps
 * (s_memrealtime, 100 MHz) per entity to probe[4 * n_entities] (DEVICE):
 * start, Gramian done, elimination done, end (entities without ratings:
 * untouched). */
int mf_als_sweep_probe(const int64_t* entity_ptr, const int32_t* other_ids,
                       const void* ratings, int32_t n_entities, double global_mean,
                       const void* other_biases, const void* other_features,
                       void* biases, void* features, int32_t n_factors, int32_t dtype,
                       double reg, void* stream, int64_t* probe);

/* ---------------- multi-GPU replica exchange ----------------------------- */

/*
 * Element-wise helper around the per-epoch all-reduce of the replicated item
 * parameters (user-sharded data parallelism, "delta" exchange, DESIGN.md
 * section 6; no
 * counterpart in the single-process reference):
 *   mode 0 (MF_DELTA_TAKE):  cur[j] = cur[j] - base[j]   (local update delta)
 *   mode 1 (MF_DELTA_APPLY): cur[j] = cur[j] + base[j]   (base + summed delta)
 * cur, base: device, n values of dtype.
 */
enum { MF_DELTA_TAKE = 0, MF_DELTA_APPLY = 1 };
int mf_replica_delta(void* cur, const void* base, int64_t n, int32_t dtype,
                     int32_t mode, void* stream);
/* cur[j] = cur[j] + scale * delta[j] (device, n values of dtype): applies
 * the all-reduced item deltas; scale = min(1/2, 2/world) is the default of
 * the delta exchange (distributed.default_delta_scale) -- the plain sum
 * (scale 1) overshoots once each rank's local epoch moves an item most of the
 * way to its local optimum (measured at C3: N = 4 and 8 diverge), plain
 * averaging (1/world) under-steps. */
int mf_replica_apply(void* cur, const void* delta, int64_t n, int32_t dtype, double scale,
                     void* stream);

/* ---------------- host-side schedulers (no GPU) -------------------------- */

/*
 * Exact-order schedule.  Given the visit order of one epoch (the row order
 * of X after `np.random.shuffle(X)`, kernel_matrix_factorization.py:371),
 * assign every rating the level 1 + max(level of the previous rating of the
 * same user, ... of the same item) and group positions by level.  Applying
 * the levels in increasing order (mf_sgd_epoch) is bit-for-bit the
 * reference's sequential sweep.  use_user / use_item drop a row family
 * from the conflict test when it is not written (update_users passes
 * use_item = 0, kernel_matrix_factorization.py:234).
 *
 *   order            host, nullable, n: visit order (rating indices)
 *   sched_out        host, n: rating indices grouped by level, each level
 *                    in visit order
 *   level_offsets    host, capacity `offsets_cap` (>= n_levels + 1)
 *   n_levels_out     host
 */
int mf_sched_levels(const int32_t* user_ids, const int32_t* item_ids,
                    int64_t n, const int64_t* order, int32_t n_users,
                    int32_t n_items, int32_t use_user, int32_t use_item,
                    int32_t* sched_out, int64_t* level_offsets,
                    int64_t offsets_cap, int32_t* n_levels_out);

/*
 * The exact-order schedule at scale (replaces the per-epoch host cost of
 * `np.random.shuffle(X)` + the sequential sweep's order,
 * kernel_matrix_factorization.py:369-425).  The visit order is cut into
 * n_chunks contiguous chunks (<= 0: min(16, cores) from 2^20 ratings, else
 * 1) levelled on as many threads, each chunk's levels placed after all of
 * the earlier chunks'.  Every level is conflict-free and every rating's
 * level is above each earlier rating of its user and item, so the levels
 * applied in order (mf_sgd_epoch) give the same bits as mf_sched_levels'
 * greedy levels -- more levels (the sum of the chunk depths), built in a
 * fraction of the time.  order: 32-bit rating indices, n < 2^31.
 * sched_out[lo_c, hi_c) holds chunk c's ratings (the chunk's own range of
 * visit positions), by level, each level in visit order.
 */
int mf_sched_levels_chunked(const int32_t* user_ids, const int32_t* item_ids,
                            int64_t n, const int32_t* order, int32_t n_users,
                            int32_t n_items, int32_t use_user, int32_t use_item,
                            int32_t n_chunks, int32_t* sched_out, int64_t* level_offsets,
                            int64_t offsets_cap, int32_t* n_levels_out);

/*
 * Throughput schedule.  Greedy edge colouring of the bipartite rating graph
 * (no two ratings of one colour share a user or an item), ratings visited
 * item by item.  Output: rating indices grouped by colour, each colour sorted
 * by item id (so a batch walks Q in address order), plus colour offsets.
 * Any order of colours is a valid sequential order of the ratings.
 *   colour count <= max user degree + max item degree - 1 (offsets_cap must
 *   be at least that + 1).
 */
int mf_sched_color(const int32_t* user_ids, const int32_t* item_ids,
                   int64_t n, int32_t n_users, int32_t n_items,
                   int32_t* sched_out, int64_t* color_offsets,
                   int64_t offsets_cap, int32_t* n_colors_out);

/*
 * Evaluation order for the read-only passes (mf_sse, mf_sse_sliced).  Items
 * are cut into n_slices contiguous id ranges (n_slices = 8: one per XCD, so
 * one slice of Q fits an XCD's 4 MiB L2); ratings are grouped by slice and,
 * inside a slice, by user (consecutive ratings share the user's P row).
 *   sched_out      host, n: rating indices in that order
 *   slice_offsets  host, n_slices + 1
 */
int mf_sched_slices(const int32_t* user_ids, const int32_t* item_ids,
                    int64_t n, int32_t n_users, int32_t n_items,
                    int32_t n_slices, int32_t* sched_out,
                    int64_t* slice_offsets);

/*
 * Tiled evaluation order (replaces the per-rating loop order of
 * _calculate_rmse, kernel_matrix_factorization.py:240-317, which any order
 * serves: the pass is read-only).  Users are cut into n_chunks contiguous id
 * ranges of about equal rating counts, items into n_slices id ranges; tile
 * c * n_slices + s holds the ratings of user chunk c and item slice s, users
 * ascending inside a tile.  With n_slices a multiple of 8 and the offsets
 * passed to mf_sse, the FP64 pass walks the tiles in phases of 8 (one per
 * XCD) with a resident grid (k_sse_phased), so each XCD's L2 holds one
 * 1/n_slices item slice at a time.
 *   n_chunks * n_slices <= 128
 *   sched_out      host, n: rating indices in that order
 *   tile_offsets   host, n_chunks * n_slices + 1
 */
int mf_sched_tiles(const int32_t* user_ids, const int32_t* item_ids,
                   int64_t n, int32_t n_users, int32_t n_items,
                   int32_t n_chunks, int32_t n_slices, int32_t* sched_out,
                   int64_t* tile_offsets);

/*
 * Plan of the stratified sweep (mf_sgd_epoch_strata), host only.
 * user_bounds / item_bounds (HOST, n_blocks+1 each, non-decreasing from 0 to
 * n_users / n_items) cut the ids into B contiguous ranges; block (s, w) =
 * user range (w+s) mod B x item range w.  Inside a block every user is owned
 * by one of n_slots rating slots (largest degree first onto the least loaded
 * slot) and the ratings are edge-coloured as a bipartite (slot, item)
 * multigraph with exactly D = max(slot load, item degree) colours, one step
 * per colour: no step holds a slot or an item twice.
 *   mf_strata_plan_build      plans all blocks into an opaque handle
 *   mf_strata_plan_positions  n_positions = (total steps) * n_slots
 *   mf_strata_plan_fetch      sched_out[n_positions] = rating index per
 *                             position, -1 = idle slot (block-major, step-
 *                             major, slot-minor); block_steps[B*B+1] = step
 *                             offsets of the blocks
 *   mf_strata_plan_free
 */
typedef struct mf_strata_plan mf_strata_plan;
/* The same with n_classes user-range classes: user_bounds has
 * n_classes * n_blocks + 1 entries, block_steps (fetch) n_classes * n_blocks^2
 * + 1; block (s, w), s < n_classes * n_blocks, = user range (s + n_classes*w)
 * mod (n_classes * n_blocks) x item range w.  n_classes = 1 is
 * mf_strata_plan_build. */
int mf_strata_plan_build_classes(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                                 int32_t n_users, int32_t n_items, int32_t n_blocks,
                                 int32_t n_classes, const int32_t* user_bounds,
                                 const int32_t* item_bounds, int32_t n_slots,
                                 mf_strata_plan** plan_out);
/* mf_strata_plan_build_classes over n_cands (slots, waves) kernel shapes
 * (1..8): the step counts of each (no colouring) pick the shape of least
 * steps * waves (ties: the earlier one), the first one outright when its plan
 * fills at least fill_stop of its positions (n / (steps * slots); 0 = never);
 * only the pick is planned in full.  *picked = its index.  The plan is the
 * one mf_strata_plan_build_classes builds with that shape's slot count. */
int mf_strata_plan_build_pick(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                              int32_t n_users, int32_t n_items, int32_t n_blocks,
                              int32_t n_classes, const int32_t* user_bounds,
                              const int32_t* item_bounds, const int32_t* slot_cands,
                              const int32_t* wave_cands, int32_t n_cands, double fill_stop,
                              int32_t* picked, mf_strata_plan** plan_out);
int mf_strata_plan_build(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                         int32_t n_users, int32_t n_items, int32_t n_blocks,
                         const int32_t* user_bounds, const int32_t* item_bounds,
                         int32_t n_slots, mf_strata_plan** plan_out);
int64_t mf_strata_plan_positions(const mf_strata_plan* plan);
int mf_strata_plan_fetch(const mf_strata_plan* plan, int32_t* sched_out,
                         int64_t* block_steps);
void mf_strata_plan_free(mf_strata_plan* plan);

/* ---------------------------------------------------------------------------
 * fit() preprocessing, host only (mf_prep.cpp).  Replaces the three costly
 * steps of RecommenderBase._preprocess_data (recommender_base.py:97-173 of
 * the reference) for integer ids, with identical results:
 *
 * mf_legacy_shuffle      numpy.random.RandomState.shuffle(data) of a 1-D
 *     8-byte array, drawn from the MT19937 state (key[624], *pos) given and
 *     advancing it exactly as NumPy does (numpy 2.2 mtrand _shuffle_raw +
 *     random_interval).  On arange(n) this is permutation(n), which is the
 *     draw of X.sample(frac=1, replace=False) (recommender_base.py:131 =
 *     RandomState.choice(n, n, replace=False)); on the row order it is the
 *     per-epoch np.random.shuffle (kernel_matrix_factorization.py:371).
 *     n <= 2^32 + 1 (NumPy's 32-bit draw branch); MF_ERR_INVALID otherwise.
 * mf_legacy_permutation  out = np.random.permutation(n) (int64), the same
 *     draws as mf_legacy_shuffle of arange(n), swapped on 4-byte elements
 *     while n < 2^31.
 * mf_pairs_duplicated    *has_dup = 1 iff two rows hold the same (a, b)
 *     pair of integer ids (X.duplicated(subset=[user_id, item_id]).sum()
 *     != 0, :127-128).
 * mf_factorize           pd.factorize(vals, sort=False) of integer ids, as
 *     X[col].unique() + the id map of the shuffled frame (:135-140):
 *     uniques[0..*n_uniques) in first-appearance order (capacity n) and
 *     codes[p] = position of vals[p] in uniques.
 * mf_id_range            *lo / *hi = min / max of vals (n > 0).
 * mf_first_appearance    pd.factorize(vals[perm], sort=False) given dense ids
 *     of the unshuffled column: dense[p] - base in [0, n_dense) (the ids
 *     themselves when they span a small range, else mf_factorize's codes of
 *     the unshuffled column), n_dense <= 2^32 - 1.  codes[t] = code of row
 *     perm[t]; order[0..*n_uniques) = the dense ids in code order (capacity
 *     n_dense), so uniques = base + order or the unshuffled uniques[order].
 * mf_gather              dst[p] = src[idx[p]], idx[p] in [0, n_src), for
 *     elem_bytes 4 or 8.
 * Threads: min(16, cores) unless MF_HOST_THREADS is set. */
int mf_legacy_shuffle(uint32_t* mt_key, int32_t* mt_pos, int64_t* data, int64_t n);
/* mf_legacy_shuffle on a 1-D array of 4-byte elements: the same draws and
 * swaps (they depend on n only), half the bytes moved; the exact schedule's
 * per-epoch np.random.shuffle of the row order (kernel_matrix_factorization.py:371)
 * runs on 32-bit rating indices. */
int mf_legacy_shuffle_i32(uint32_t* mt_key, int32_t* mt_pos, int32_t* data, int64_t n);
int mf_legacy_permutation(uint32_t* mt_key, int32_t* mt_pos, int64_t* out, int64_t n);
/* np.random.shuffle of n elements in two parts (the exact schedule's
 * per-epoch shuffle, kernel_matrix_factorization.py:371, with its swaps on the
 * GPU): mf_legacy_shuffle_draws makes the draws only -- targets[d] = the
 * position swapped with n-1-d, d = 0 .. n-2 -- advancing the MT19937 state
 * exactly as the whole shuffle does; mf_legacy_apply_swaps_i32 applies swaps
 * d_begin .. n-2 of them, in order, on the host; mf_shuffle_swaps_device
 * (device pointers; stream a hipStream_t) applies swaps 0 .. d_end-1 on the
 * GPU by rounds of deterministic reservations (the same result as in
 * order): reservations = n zeroed 64-bit words kept between calls, tag_io =
 * the next round tag (start at 1; advanced), workspace >=
 * mf_shuffle_swaps_workspace_bytes(n). */
int mf_legacy_shuffle_draws(uint32_t* mt_key, int32_t* mt_pos, int64_t n, uint32_t* targets);
int mf_legacy_apply_swaps_i32(const uint32_t* targets, int64_t n, int64_t d_begin, int32_t* data);
size_t mf_shuffle_swaps_workspace_bytes(int64_t n);
int mf_shuffle_swaps_device(const uint32_t* targets, int64_t n, int64_t d_end, int32_t* data,
                            unsigned long long* reservations, void* workspace, uint64_t* tag_io,
                            void* stream);
int mf_pairs_duplicated(const int64_t* a, const int64_t* b, int64_t n, int32_t* has_dup);
int mf_factorize(const int64_t* vals, int64_t n, int64_t* codes, int64_t* uniques,
                 int64_t* n_uniques);
int mf_id_range(const int64_t* vals, int64_t n, int64_t* lo, int64_t* hi);
int mf_first_appearance(const int64_t* dense, int64_t base, int64_t n_dense, const int64_t* perm,
                        int64_t n, int64_t* codes, int64_t* order, int64_t* n_uniques);
int mf_gather(const void* src, int64_t n_src, int32_t elem_bytes, const int64_t* idx, int64_t n,
              void* dst);
/* mf_gather with 32-bit indices: the relabelled strata plans' host ids
 * (user x -> pu[x] over 10^8 int32 ids, engine.py _build_regroup). */
int mf_gather_i32(const void* src, int64_t n_src, int32_t elem_bytes, const int32_t* idx,
                  int64_t n, void* dst);
/* dst[p] = (int32)src[p] for ids in [0, bound) (else MF_ERR_INVALID; bound
 * <= 2^31), and dst[p] = (float)src[p]: the engine's host ids and FP32
 * ratings from fit()'s int64 codes and float64 ratings, threaded
 * (kernel_matrix_factorization.py _make_engine). */
int mf_ids_to_i32(const int64_t* src, int64_t n, int64_t bound, int32_t* dst);
int mf_f64_to_f32(const double* src, int64_t n, float* dst);
/* 64-bit fingerprint of a HOST buffer (threaded, not cryptographic): lets the
 * estimator tell whether the device copy of a parameter array is still the
 * NumPy attribute's content (the reference predicts from the live arrays,
 * kernel_matrix_factorization.py:148-160). */
uint64_t mf_fingerprint(const void* data, int64_t n_bytes);

#ifdef __cplusplus
}
#endif

#endif /* MF_HIP_H */
