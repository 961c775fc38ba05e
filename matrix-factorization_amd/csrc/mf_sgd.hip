// mf_sgd.hip -- C ABI of the KernelMF hot path (include/mf_hip.h):
//   mf_sgd_epoch  -> k_sgd_batch  (mf_rows.hpp; one launch per batch)
//   mf_sse        -> k_sse_owned (mf_rows.hpp)
//   mf_predict    -> k_read       (this file)
//
// Compiled with -ffp-contract=off: every scalar expression rounds like the
// reference's FP64 evaluation of the same expression; only the k-long sums
// follow a fixed DPP order instead of BLAS ddot's.
#include <atomic>
#include <algorithm>
#include <type_traits>
#include <vector>

#include "mf_rows.hpp"
#include "mf_strata.hpp"
#include "mf_dispatch.hpp"

namespace mf {

template <typename T, int V> struct Tile {
    static constexpr int U = V >= 4 ? 1 : (V == 2 ? 2 : 4);
};

// Batched prediction (_predict, kernel_matrix_factorization.py:448-541):
// -1 ids read as a zero bias and an all-zero factor row (:487-499).
template <typename T, int GS, int V, int KERN, bool SSE>
__global__ __launch_bounds__(kBlock) void k_read(ReadArgs<T> A, SliceTab S) {
    constexpr int R = kWave / GS;
    constexpr int U = Tile<T, V>::U;
    constexpr int RPW = U * R;
    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS;
    const int l = lane % GS;
    const int k = A.k;
    const Hyper<T> h = A.h;
    const int x_slice = blockIdx.x % S.n;
    const int64_t bps = gridDim.x / S.n;                 // blocks per slice
    const int64_t s_end = S.off[x_slice + 1];
    const int64_t nwaves = bps * kWavesPerBlock;
    const int64_t wave = (int64_t)(blockIdx.x / S.n) * kWavesPerBlock + threadIdx.x / kWave;
    double acc = 0.0;

    for (int64_t w0 = S.off[x_slice] + wave * RPW; w0 < s_end; w0 += nwaves * RPW) {
        const int nw = (int)min((int64_t)RPW, s_end - w0);
        int uu[U], ii[U];
        bool have[U];
        T p[U][V], q[U][V], bu[U], bi[U];
#pragma unroll
        for (int x = 0; x < U; ++x) {
            const int idx = x * R + g;
            have[x] = idx < nw;
            const int64_t j = w0 + (have[x] ? idx : 0);
            uu[x] = A.u[j];
            ii[x] = A.i[j];
            const bool uk = have[x] && uu[x] >= 0;
            const bool ik = have[x] && ii[x] >= 0;
            const T* pr = A.P + (int64_t)(uk ? uu[x] : 0) * k;
            const T* qr = A.Q + (int64_t)(ik ? ii[x] : 0) * k;
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int f = l + v * GS;
                p[x][v] = (uk && f < k) ? pr[f] : (T)0;
                q[x][v] = (ik && f < k) ? qr[f] : (T)0;
            }
            if constexpr (KERN != MF_RBF) {
                bu[x] = uk ? A.Bu[uu[x]] : (T)0;
                bi[x] = ik ? A.Bi[ii[x]] : (T)0;
            } else {
                bu[x] = bi[x] = (T)0;
            }
        }
#pragma unroll
        for (int x = 0; x < U; ++x) {
            T s = (T)0;
#pragma unroll
            for (int v = 0; v < V; ++v) {
                if constexpr (KERN == MF_RBF) {
                    const T d = p[x][v] - q[x][v];
                    s = s + d * d;
                } else {
                    s = s + p[x][v] * q[x][v];
                }
            }
            s = group_sum<GS>(s);
            T pred = predict_one<T, KERN>(s, bu[x], bi[x], h);
            if (have[x] && l == 0) {
                const int64_t j = w0 + x * R + g;
                if constexpr (SSE) {
                    const T err = A.r[j] - pred;             // :313
                    acc += (double)err * (double)err;
                } else {
                    if (A.bound) {                           // :532-536
                        if (pred > h.hi) pred = h.hi;
                        else if (pred < h.lo) pred = h.lo;
                    }
                    A.out[j] = pred;
                }
            }
        }
    }

    if constexpr (SSE) {
        // deterministic block reduction: wave butterfly, then 4 partials
        acc = wave_sum(acc);
        __shared__ double red[kWavesPerBlock];
        if (lane == 0) red[threadIdx.x / kWave] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
#pragma unroll
            for (int w = 0; w < kWavesPerBlock; ++w) t += red[w];
            A.partials[blockIdx.x] = t;
        }
    }
}

// Training SSE, streaming form.  Each wave owns a contiguous run of its
// slice; triples arrive 64 at a time in three coalesced loads (lane j holds
// rating j of the chunk) and the NEXT chunk's triples are loaded before the
// current chunk is consumed, so the only exposed latency is the row gather
// (U groups of R ratings in flight).  In mf_sched_slices order consecutive
// ratings share the user's P row (L1/L2 hits) and a slice's Q rows stay in
// one XCD's L2.
// Fixed-order sum of the per-block partials (one block).
__global__ __launch_bounds__(kBlock) void k_sum_partials(const double* part, int n,
                                                         double* out) {
    double t = 0.0;
    for (int j = threadIdx.x; j < n; j += kBlock) t += part[j];
    t = wave_sum(t);
    __shared__ double red[kWavesPerBlock];
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < kWavesPerBlock; ++w) s += red[w];
        *out = s;
    }
}

inline int read_bps(const SliceTab& S, int rpw) {
    int64_t mx = 0;
    for (int x = 0; x < S.n; ++x) mx = std::max(mx, S.off[x + 1] - S.off[x]);
    const int64_t waves = (mx + rpw - 1) / rpw;
    const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    return (int)std::max<int64_t>(1, std::min<int64_t>(blocks, kSseMaxBlocks / S.n));
}

struct ReadLaunch {
    const int32_t* u; const int32_t* i; const void* r; int64_t n;
    double mu; const void* bu; const void* bi; const void* P; const void* Q;
    int32_t k; double gamma, lo, hi; int32_t bound; void* out;
    double* partials; double* sse_out; hipStream_t stream; SliceTab S;

    template <typename T, int GS, int V, int KERN>
    int run() {
        constexpr int RPW = Tile<T, V>::U * (kWave / GS);
        ReadArgs<T> a;
        a.u = u; a.i = i; a.r = static_cast<const T*>(r);
        a.P = static_cast<const T*>(P); a.Q = static_cast<const T*>(Q);
        a.Bu = static_cast<const T*>(bu); a.Bi = static_cast<const T*>(bi);
        a.n = n; a.k = k; a.bound = bound; a.out = static_cast<T*>(out);
        a.partials = partials;
        a.h = make_hyper<T>(mu, 0.0, 0.0, gamma, lo, hi);
        const int blocks = read_bps(S, RPW) * S.n;
        hipLaunchKernelGGL((k_read<T, GS, V, KERN, false>), dim3(blocks), dim3(kBlock), 0,
                           stream, a, S);
        MF_HIP_CHECK(hipGetLastError());
        return MF_OK;
    }
};

}  // namespace mf

using namespace mf;

extern "C" int mf_max_factors(void) { return kMaxFactors; }

extern "C" size_t mf_sgd_workspace_bytes(int32_t n_launch) {
    return n_launch > 0 ? sizeof(int32_t) * 8 * (size_t)n_launch : 0;
}

extern "C" int mf_sgd_epoch(const int32_t* user_ids, const int32_t* item_ids,
                            const void* ratings, int64_t n_ratings,
                            const int32_t* order, const int64_t* batch_offsets,
                            int32_t n_batches, const int32_t* batch_seq,
                            int32_t n_seq, double global_mean, void* user_biases,
                            void* item_biases, void* user_features,
                            void* item_features, int32_t n_users,
                            int32_t n_items, int32_t n_factors, int32_t kernel,
                            int32_t dtype, double gamma, double lr, double reg,
                            double min_rating, double max_rating,
                            int32_t update_user_params,
                            int32_t update_item_params, int32_t flags,
                            void* workspace, size_t workspace_bytes,
                            void* stream, double* kernel_ms) {
    if (n_ratings < 0 || n_batches < 0 || n_users < 0 || n_items < 0 ||
        (batch_seq && n_seq < 0)) {
        set_error("negative size");
        return MF_ERR_INVALID;
    }
    if (n_batches > 0 && !batch_offsets) {
        set_error("batch_offsets is NULL");
        return MF_ERR_INVALID;
    }
    for (int32_t b = 0; b < n_batches; ++b) {
        if (batch_offsets[b] < 0 || batch_offsets[b + 1] < batch_offsets[b] ||
            batch_offsets[b + 1] > n_ratings) {
            set_error("batch_offsets[%d..%d] = %lld..%lld invalid for n_ratings=%lld", b, b + 1,
                      (long long)batch_offsets[b], (long long)batch_offsets[b + 1],
                      (long long)n_ratings);
            return MF_ERR_INVALID;
        }
    }
    const int32_t n_launch = batch_seq ? n_seq : n_batches;
    for (int32_t q = 0; batch_seq && q < n_seq; ++q) {
        if (batch_seq[q] < 0 || batch_seq[q] >= n_batches) {
            set_error("batch_seq[%d] = %d out of range [0, %d)", q, batch_seq[q], n_batches);
            return MF_ERR_INVALID;
        }
    }
    if (n_ratings > 0 && (!user_ids || !item_ids || !ratings)) {
        set_error("NULL triple array");
        return MF_ERR_INVALID;
    }
    if (kernel_ms) { kernel_ms[0] = 0.0; kernel_ms[1] = 0.0; }
    if (n_launch == 0 || n_ratings == 0) return MF_OK;
    int32_t* claim = nullptr;
    if (flags & MF_FLAG_XCD_CLAIM) {
        if (!workspace || workspace_bytes < mf_sgd_workspace_bytes(n_launch)) {
            set_error("MF_FLAG_XCD_CLAIM needs a workspace of mf_sgd_workspace_bytes(%d) bytes",
                      n_launch);
            return MF_ERR_INVALID;
        }
        claim = static_cast<int32_t*>(workspace);
    }
    SgdParams P{user_ids, item_ids, ratings, order, batch_offsets, batch_seq, n_launch,
                global_mean, user_biases, item_biases, user_features, item_features,
                n_factors, kernel, gamma, lr, reg, min_rating, max_rating,
                update_user_params ? 1 : 0, update_item_params ? 1 : 0, flags,
                (hipStream_t)stream, kernel_ms, claim, n_users};
    if (dtype == MF_F32) return sgd_launch_f32(P);
    if (dtype == MF_F64) return sgd_launch_f64(P);
    set_error("unknown dtype code %d", dtype);
    return MF_ERR_INVALID;
}

extern "C" size_t mf_strata_lds_bytes(int32_t max_block_items, int32_t max_block_users,
                                      int32_t n_factors, int32_t dtype) {
    if (max_block_items < 0 || max_block_users < 0 || n_factors < 0) return 0;
    return dtype == MF_F32 ? strata_lds_bytes<float>(max_block_items, max_block_users, n_factors)
                           : strata_lds_bytes<double>(max_block_items, max_block_users, n_factors);
}

extern "C" int32_t mf_strata_lds_limit(void) { return kLdsLimit; }

namespace mf {
static int64_t* g_strata_probe = nullptr;
int64_t* strata_probe_ptr() { return g_strata_probe; }
static std::atomic<int32_t> g_strata_inject{0};
bool strata_inject_fail() {
    int32_t v = g_strata_inject.load();
    while (v > 0)
        if (g_strata_inject.compare_exchange_weak(v, v - 1)) return true;
    return false;
}
}  // namespace mf

extern "C" int mf_strata_set_probe(int64_t* probe) {
    mf::g_strata_probe = probe;
    return MF_OK;
}

extern "C" int mf_strata_inject_fail(int32_t n_launches) {
    if (n_launches < 0) {
        set_error("mf_strata_inject_fail: n_launches < 0");
        return MF_ERR_INVALID;
    }
    mf::g_strata_inject.store(n_launches);
    return MF_OK;
}

extern "C" size_t mf_strata_workspace_bytes(int32_t n_blocks, int32_t n_seq) {
    return n_blocks > 0 && n_seq >= 0 ? strata_ws_bytes(n_blocks, n_seq) : 0;
}

// One empty launch: the runtime loads the library's code object for the
// device at the first launch of any of its kernels (tens of ms for this
// library), which otherwise lands in the first training epoch.
__global__ void k_warmup() {}

extern "C" int mf_warmup(int32_t flags, void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    const LaunchTrace lt;
    hipLaunchKernelGGL(k_warmup, dim3(1), dim3(64), 0, s);
    lt.mark("warmup: sgd unit");
    touch_rows_f32(s);
    touch_rows_f64(s);
    lt.mark("warmup: rows units");
    touch_strata_f32(s);
    touch_strata_f64(s);
    lt.mark("warmup: strata units");
    touch_bias(s);
    touch_topk(s);
    touch_als(s);
    lt.mark("warmup: other units");
    if (!(flags & MF_FLAG_NO_COOP)) {   // the cooperative launch path (persistent sweeps)
        void* no_args[1] = {nullptr};
        (void)hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_warmup), dim3(1),
                                         dim3(64), no_args, 0u, s);
        (void)hipGetLastError();
    }
    lt.mark("warmup: cooperative");
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MF_OK : hip_fail(e, "mf_warmup");
}

extern "C" int mf_strata_status(const void* workspace, int32_t n_blocks, void* stream) {
    if (!workspace || n_blocks < 1) {
        set_error("mf_strata_status: NULL workspace");
        return MF_ERR_INVALID;
    }
    int32_t err = 0;
    MF_HIP_CHECK(hipMemcpyAsync(&err, static_cast<const int32_t*>(workspace) + n_blocks,
                                sizeof(int32_t), hipMemcpyDeviceToHost, (hipStream_t)stream));
    MF_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    if (err != 0) {
        set_error("persistent strata sweep: a workgroup gave up waiting for its neighbour "
                  "(workgroups not co-resident?); the parameters are invalid");
        return MF_ERR_HIP;
    }
    return MF_OK;
}

extern "C" int32_t mf_strata_slots_waves(int32_t n_factors, int32_t dtype, int32_t waves) {
    if (n_factors < 0 || n_factors > kMaxFactors || (dtype != MF_F32 && dtype != MF_F64) ||
        (waves != 16 && waves != 8 && waves != 4)) {
        set_error("mf_strata_slots_waves: n_factors=%d / dtype=%d / waves=%d invalid", n_factors,
                  dtype, waves);
        return -1;
    }
    if (dtype == MF_F32) {
        StrataSlots<float> f{waves};
        return dispatch_rows<float>(n_factors, MF_LINEAR, f);
    }
    StrataSlots<double> f{waves};
    return dispatch_rows<double>(n_factors, MF_LINEAR, f);
}

extern "C" int32_t mf_strata_slots(int32_t n_factors, int32_t dtype) {
    return mf_strata_slots_waves(n_factors, dtype, 16);
}

static int strata_epoch(const int32_t* user_ids, const int32_t* item_ids,
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
                                   void* stream, double* kernel_ms, void* dq, void* dbi) {
    if (n_positions < 0 || n_blocks < 0 || n_seq < 0 || n_users < 0 || n_items < 0 ||
        max_block_items < 0 || max_block_users < 0 || n_slots < 1) {
        set_error("negative size");
        return MF_ERR_INVALID;
    }
    if (kernel_ms) { kernel_ms[0] = 0.0; kernel_ms[1] = 0.0; }
    if (n_seq == 0 || n_positions == 0) return MF_OK;
    if (n_blocks == 0 || !strata_seq || !user_bounds || !item_bounds || !block_steps ||
        !user_ids || !item_ids || !ratings) {
        set_error("NULL plan or triple array");
        return MF_ERR_INVALID;
    }
    const int n_cls = strata_classes(flags);       // user-range classes: C*B strata
    if (n_cls > MF_STRATA_MAX_CLASSES) {
        set_error("user-range classes %d > %d", n_cls, MF_STRATA_MAX_CLASSES);
        return MF_ERR_INVALID;
    }
    if ((int64_t)n_cls * n_blocks * n_blocks >= ((int64_t)1 << 31)) {
        set_error("n_blocks=%d too large", n_blocks);
        return MF_ERR_INVALID;
    }
    for (int32_t t = 0; t < n_seq; ++t) {
        if (strata_seq[t] < 0 || strata_seq[t] >= n_cls * n_blocks) {
            set_error("strata_seq[%d] = %d out of range [0, %d)", t, strata_seq[t],
                      n_cls * n_blocks);
            return MF_ERR_INVALID;
        }
    }
    if (!(flags & MF_FLAG_PREPARE) &&
        (!user_features || !item_features || (kernel != MF_RBF && (!user_biases || !item_biases)))) {
        set_error("NULL parameter array");
        return MF_ERR_INVALID;
    }
    StrataParams P{user_ids, item_ids, ratings, user_bounds, item_bounds, block_steps,
                   n_blocks, n_slots, max_block_items, max_block_users,
                   strata_seq, n_seq, seed, global_mean, user_biases, item_biases,
                   user_features, item_features, n_factors, kernel, gamma, lr, reg,
                   min_rating, max_rating, update_user_params ? 1 : 0,
                   update_item_params ? 1 : 0, flags, workspace, workspace_bytes, n_users,
                   (hipStream_t)stream, kernel_ms, n_items, dq, dbi, n_positions};
    if (dtype == MF_F32) return strata_launch_f32(P);
    if (dtype == MF_F64) return strata_launch_f64(P);
    set_error("unknown dtype code %d", dtype);
    return MF_ERR_INVALID;
}

extern "C" int mf_sgd_epoch_strata(const int32_t* user_ids, const int32_t* item_ids,
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
                                   void* stream, double* kernel_ms) {
    return strata_epoch(user_ids, item_ids, ratings, n_positions, n_blocks, user_bounds,
                        item_bounds, block_steps, n_slots, max_block_items, max_block_users,
                        strata_seq, n_seq, seed, global_mean, user_biases, item_biases,
                        user_features, item_features, n_users, n_items, n_factors, kernel, dtype,
                        gamma, lr, reg, min_rating, max_rating, update_user_params,
                        update_item_params, flags, workspace, workspace_bytes, stream, kernel_ms,
                        nullptr, nullptr);
}

extern "C" int mf_sgd_epoch_strata_delta(
    const int32_t* user_ids, const int32_t* item_ids, const void* ratings, int64_t n_positions,
    int32_t n_blocks, const int32_t* user_bounds, const int32_t* item_bounds,
    const int64_t* block_steps, int32_t n_slots, int32_t max_block_items,
    int32_t max_block_users, const int32_t* strata_seq, int32_t n_seq, uint32_t seed,
    double global_mean, void* user_biases, void* item_biases, void* user_features,
    void* item_features, int32_t n_users, int32_t n_items, int32_t n_factors, int32_t kernel,
    int32_t dtype, double gamma, double lr, double reg, double min_rating, double max_rating,
    int32_t update_user_params, int32_t update_item_params, int32_t flags, void* workspace,
    size_t workspace_bytes, void* item_delta, void* item_bias_delta, void* stream,
    double* kernel_ms) {
    if (!item_delta || (kernel != MF_RBF && !item_bias_delta)) {
        set_error("mf_sgd_epoch_strata_delta: NULL delta buffer");
        return MF_ERR_INVALID;
    }
    return strata_epoch(user_ids, item_ids, ratings, n_positions, n_blocks, user_bounds,
                        item_bounds, block_steps, n_slots, max_block_items, max_block_users,
                        strata_seq, n_seq, seed, global_mean, user_biases, item_biases,
                        user_features, item_features, n_users, n_items, n_factors, kernel, dtype,
                        gamma, lr, reg, min_rating, max_rating, update_user_params,
                        update_item_params, flags, workspace, workspace_bytes, stream, kernel_ms,
                        item_delta, item_bias_delta);
}

extern "C" size_t mf_sse_workspace_bytes(int64_t n_ratings) {
    (void)n_ratings;
    return sizeof(double) * (size_t)kSseMaxBlocks;
}

extern "C" int mf_sse_capped(const int32_t* user_ids, const int32_t* item_ids,
                             const void* ratings, int64_t n_ratings,
                             double global_mean, const void* user_biases,
                             const void* item_biases, const void* user_features,
                             const void* item_features, int32_t n_users, int32_t n_items,
                             int32_t n_factors, int32_t kernel, int32_t dtype, double gamma,
                             double min_rating, double max_rating,
                             const int64_t* slice_offsets, int32_t n_slices, void* workspace,
                             int32_t max_blocks, double* sse_out, void* stream) {
    if (n_ratings < 0 || !sse_out || !workspace || n_users < 0 || n_items < 0 ||
        (slice_offsets && (n_slices < 1 || n_slices > kMaxSlices))) {
        set_error("mf_sse: bad arguments (n_slices must be in [1, %d])", kMaxSlices);
        return MF_ERR_INVALID;
    }
    SliceTab S;
    if (slice_offsets) {
        S.n = n_slices;
        for (int x = 0; x <= n_slices; ++x) S.off[x] = slice_offsets[x];
        for (int x = 0; x < n_slices; ++x) {
            if (S.off[x] < 0 || S.off[x + 1] < S.off[x] || S.off[n_slices] > n_ratings) {
                set_error("mf_sse: slice_offsets invalid");
                return MF_ERR_INVALID;
            }
        }
    } else {
        S.n = 1; S.off[0] = 0; S.off[1] = n_ratings;
    }
    if (n_ratings == 0) {
        MF_HIP_CHECK(hipMemsetAsync(sse_out, 0, sizeof(double), (hipStream_t)stream));
        return MF_OK;
    }
    if (max_blocks < 0) {
        set_error("mf_sse_capped: max_blocks < 0");
        return MF_ERR_INVALID;
    }
    SseParams P{user_ids, item_ids, ratings, n_ratings, global_mean, user_biases,
                item_biases, user_features, item_features, n_users, n_items, n_factors,
                kernel, gamma, min_rating, max_rating, (double*)workspace, sse_out,
                (hipStream_t)stream, S, max_blocks};
    if (dtype == MF_F32) return sse_launch_f32(P);
    if (dtype == MF_F64) return sse_launch_f64(P);
    set_error("unknown dtype code %d", dtype);
    return MF_ERR_INVALID;
}

extern "C" int mf_sse(const int32_t* user_ids, const int32_t* item_ids,
                      const void* ratings, int64_t n_ratings,
                      double global_mean, const void* user_biases,
                      const void* item_biases, const void* user_features,
                      const void* item_features, int32_t n_users, int32_t n_items,
                      int32_t n_factors, int32_t kernel, int32_t dtype, double gamma,
                      double min_rating, double max_rating,
                      const int64_t* slice_offsets, int32_t n_slices, void* workspace,
                      double* sse_out, void* stream) {
    return mf_sse_capped(user_ids, item_ids, ratings, n_ratings, global_mean, user_biases,
                         item_biases, user_features, item_features, n_users, n_items,
                         n_factors, kernel, dtype, gamma, min_rating, max_rating,
                         slice_offsets, n_slices, workspace, 0, sse_out, stream);
}

extern "C" int mf_predict(const int32_t* user_ids, const int32_t* item_ids,
                          int64_t n_pairs, double global_mean,
                          const void* user_biases, const void* item_biases,
                          const void* user_features, const void* item_features,
                          int32_t n_factors, int32_t kernel, int32_t dtype,
                          double gamma, double min_rating, double max_rating,
                          int32_t bound_ratings, void* out, void* stream) {
    if (n_pairs < 0 || (n_pairs > 0 && !out)) {
        set_error("mf_predict: bad arguments");
        return MF_ERR_INVALID;
    }
    if (n_pairs == 0) return MF_OK;
    SliceTab S;
    S.n = 1; S.off[0] = 0; S.off[1] = n_pairs;
    ReadLaunch L{user_ids, item_ids, nullptr, n_pairs, global_mean, user_biases,
                 item_biases, user_features, item_features, n_factors, gamma,
                 min_rating, max_rating, bound_ratings ? 1 : 0, out, nullptr,
                 nullptr, (hipStream_t)stream, S};
    return dispatch(dtype, n_factors, kernel, L);
}
