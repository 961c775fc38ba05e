// mf_sgd.hip -- gfx950 kernels for the KernelMF hot path:
//   k_sgd_batch : one conflict-free batch of SGD updates
//                 (kernels.py:108-327 applied to every rating of the batch)
//   k_sse       : sum of squared training errors (_calculate_rmse,
//                 kernel_matrix_factorization.py:240-317)
//   k_predict   : batched prediction (_predict, :448-541)
// and their C-ABI launchers (include/mf_hip.h).
//
// Compiled with -ffp-contract=off: every scalar expression rounds like the
// reference's FP64 evaluation of the same expression; only the k-long sums
// (group_sum) follow a fixed butterfly order instead of BLAS ddot's.
#include <algorithm>
#include <vector>

#include "mf_common.hpp"

namespace mf {

// ---------------------------------------------------------------- SGD batch
template <typename T>
struct SgdArgs {
    const int32_t* u;
    const int32_t* i;
    const T* r;
    const int32_t* order;   // nullable: position -> rating index
    T* P;
    T* Q;
    T* Bu;
    T* Bi;
    int64_t off;            // first schedule position of this batch
    int64_t n;              // ratings in this batch
    int32_t k;
    int32_t upd_user;
    int32_t upd_item;
    int32_t swizzle;
    Hyper<T> h;
};

// Tile shape per KPAD: ratings in flight per wave (U groups of R ratings)
// and iterations per wave.
template <int V> struct Tile {
    static constexpr int U = V >= 4 ? 1 : (V == 2 ? 2 : 4);
    static constexpr int ITERS = 2;
};

template <typename T, int GS, int V, int KERN>
__global__ __launch_bounds__(kBlock) void k_sgd_batch(SgdArgs<T> A) {
    constexpr int R = kWave / GS;
    constexpr int U = Tile<V>::U;
    constexpr int ITERS = Tile<V>::ITERS;
    constexpr int RPW = U * R * ITERS;       // ratings per wave
    static_assert(RPW <= kWave, "one lane per rating for the triple loads");

    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS;
    const int l = lane % GS;
    const int64_t blk = A.swizzle ? xcd_swizzle(blockIdx.x, gridDim.x)
                                  : (int64_t)blockIdx.x;
    const int64_t wave = blk * kWavesPerBlock + (threadIdx.x / kWave);
    const int64_t w0 = wave * RPW;
    if (w0 >= A.n) return;
    const int nw = (int)min((int64_t)RPW, A.n - w0);
    const int k = A.k;
    const Hyper<T> h = A.h;

    // coalesced triple loads: lane j holds rating w0 + j of the batch
    int tu = 0, ti = 0;
    T tr = (T)0;
    if (lane < nw) {
        const int64_t pos = A.off + w0 + lane;
        const int64_t j = A.order ? (int64_t)A.order[pos] : pos;
        tu = A.u[j];
        ti = A.i[j];
        tr = A.r[j];
    }

#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
        int uu[U], ii[U];
        bool have[U];
        T rr[U], bu[U], bi[U];
        T p[U][V], q[U][V];
#pragma unroll
        for (int x = 0; x < U; ++x) {
            const int idx = it * U * R + x * R + g;
            have[x] = idx < nw;
            if constexpr (GS == kWave) {
                uu[x] = rl_i32(tu, idx);
                ii[x] = rl_i32(ti, idx);
                rr[x] = rl_f(tr, idx);
            } else {
                uu[x] = bcast_i32(tu, idx);
                ii[x] = bcast_i32(ti, idx);
                rr[x] = bcast_f(tr, idx);
            }
            const T* pr = A.P + (int64_t)uu[x] * k;
            const T* qr = A.Q + (int64_t)ii[x] * k;
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int f = l + v * GS;
                const bool ok = have[x] && f < k;
                p[x][v] = ok ? pr[f] : (T)0;
                q[x][v] = ok ? qr[f] : (T)0;
            }
            if constexpr (KERN != MF_RBF) {
                bu[x] = have[x] ? A.Bu[uu[x]] : (T)0;
                bi[x] = have[x] ? A.Bi[ii[x]] : (T)0;
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

            T e, d = (T)1;
            if constexpr (KERN == MF_LINEAR) {
                // kernels.py:148-156
                const T pred = ((h.mu + bi[x]) + bu[x]) + s;
                e = pred - rr[x];
            } else if constexpr (KERN == MF_SIGMOID) {
                // kernels.py:226-236 (derivative without the c factor)
                const T lin = ((h.mu + bu[x]) + bi[x]) + s;
                const T ex = dexp<T>(-lin);
                const T sg = (T)1 / ((T)1 + ex);
                const T pred = h.a + h.c * sg;
                e = pred - rr[x];
                d = (sg * sg) * ex;
            } else {
                // kernels.py:302-310 (no biases, no c factor)
                const T E = dexp<T>((-h.gamma) * s);
                const T pred = h.a + h.c * E;
                e = pred - rr[x];
                d = ((T)2 * E) * h.gamma;
            }

            const bool lead = have[x] && l == 0;
            if constexpr (KERN == MF_LINEAR) {
                // kernels.py:159-163
                if (A.upd_user && lead) A.Bu[uu[x]] = bu[x] - h.lr * (e + h.reg * bu[x]);
                if (A.upd_item && lead) A.Bi[ii[x]] = bi[x] - h.lr * (e + h.reg * bi[x]);
            } else if constexpr (KERN == MF_SIGMOID) {
                // kernels.py:239-245
                if (A.upd_user && lead) A.Bu[uu[x]] = bu[x] - h.lr * (e * d + h.reg * bu[x]);
                if (A.upd_item && lead) A.Bi[ii[x]] = bi[x] - h.lr * (e * d + h.reg * bi[x]);
            }

            T* pw = A.P + (int64_t)uu[x] * k;
            T* qw = A.Q + (int64_t)ii[x] * k;
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int f = l + v * GS;
                if (!(have[x] && f < k)) continue;
                const T pf = p[x][v], qf = q[x][v];
                T np, nq;
                if constexpr (KERN == MF_LINEAR) {          // kernels.py:166-178
                    np = pf - h.lr * (e * qf + h.reg * pf);
                    nq = qf - h.lr * (e * pf + h.reg * qf);
                } else if constexpr (KERN == MF_SIGMOID) {  // kernels.py:248-260
                    np = pf - h.lr * (e * (qf * d) + h.reg * pf);
                    nq = qf - h.lr * (e * (pf * d) + h.reg * qf);
                } else {                                    // kernels.py:313-325
                    np = pf - h.lr * (e * (d * (qf - pf)) + h.reg * pf);
                    nq = qf - h.lr * (e * (d * (pf - qf)) + h.reg * qf);
                }
                if (A.upd_user) pw[f] = np;
                if (A.upd_item) qw[f] = nq;
            }
        }
    }
}

// ------------------------------------------------------------ predictors
// kernels.py:21-105.  `s` is the group-reduced dot product (linear/sigmoid)
// or squared distance (rbf).
template <typename T, int KERN>
__device__ __forceinline__ T predict_one(T s, T bu, T bi, const Hyper<T>& h) {
    if constexpr (KERN == MF_LINEAR) {
        return ((h.mu + bi) + bu) + s;                       // kernels.py:42-44
    } else if constexpr (KERN == MF_SIGMOID) {
        const T lin = ((h.mu + bu) + bi) + s;                // kernels.py:73-75
        const T sg = (T)1 / ((T)1 + dexp<T>(-lin));          // kernels.py:17
        return h.a + h.c * sg;                               // kernels.py:77
    } else {
        return h.a + h.c * dexp<T>((-h.gamma) * s);          // kernels.py:102-104
    }
}

// Rating/pair source for the read-only kernels.
template <typename T>
struct ReadArgs {
    const int32_t* u;
    const int32_t* i;
    const T* r;           // ratings (k_sse) or nullptr
    const T* P;
    const T* Q;
    const T* Bu;
    const T* Bi;
    int64_t n;
    int32_t k;
    int32_t bound;        // k_predict: clip
    T* out;               // k_predict: predictions
    double* partials;     // k_sse: one per block
    Hyper<T> h;
};

template <typename T, int GS, int V, int KERN, bool SSE>
__global__ __launch_bounds__(kBlock) void k_read(ReadArgs<T> A) {
    constexpr int R = kWave / GS;
    constexpr int U = Tile<V>::U;
    constexpr int RPW = U * R;
    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS;
    const int l = lane % GS;
    const int k = A.k;
    const Hyper<T> h = A.h;
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    double acc = 0.0;

    for (int64_t w0 = wave * RPW; w0 < A.n; w0 += nwaves * RPW) {
        const int nw = (int)min((int64_t)RPW, A.n - w0);
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
        acc = group_sum<kWave>(acc);
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

// Fixed-order sum of the per-block partials (one block).
__global__ __launch_bounds__(kBlock) void k_sum_partials(const double* part, int n,
                                                         double* out) {
    double t = 0.0;
    for (int j = threadIdx.x; j < n; j += kBlock) t += part[j];
    t = group_sum<kWave>(t);
    __shared__ double red[kWavesPerBlock];
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < kWavesPerBlock; ++w) s += red[w];
        *out = s;
    }
}

constexpr int kSseMaxBlocks = 2048;

inline int read_blocks(int64_t n, int rpw) {
    const int64_t waves = (n + rpw - 1) / rpw;
    const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    return (int)std::max<int64_t>(1, std::min<int64_t>(blocks, kSseMaxBlocks));
}

}  // namespace mf

#include "mf_dispatch.hpp"

namespace mf {

struct SgdLaunch {
    const int32_t* u; const int32_t* i; const void* r; const int32_t* order;
    const int64_t* offs; const int32_t* seq; int32_t nb;
    double mu; void* bu; void* bi; void* P; void* Q; int32_t k;
    double gamma, lr, reg, lo, hi; int32_t uu, ui, flags;
    hipStream_t stream; double* kernel_ms;

    template <typename T, int GS, int V, int KERN>
    int run() {
        constexpr int R = kWave / GS;
        constexpr int RPW = Tile<V>::U * R * Tile<V>::ITERS;
        SgdArgs<T> a;
        a.u = u; a.i = i; a.r = static_cast<const T*>(r); a.order = order;
        a.P = static_cast<T*>(P); a.Q = static_cast<T*>(Q);
        a.Bu = static_cast<T*>(bu); a.Bi = static_cast<T*>(bi);
        a.k = k; a.upd_user = uu; a.upd_item = ui;
        a.swizzle = (flags & MF_FLAG_XCD_SWIZZLE) ? 1 : 0;
        a.h = make_hyper<T>(mu, lr, reg, gamma, lo, hi);
        std::vector<hipEvent_t> ev;
        if (kernel_ms) {
            ev.resize(2 * (size_t)nb);
            for (auto& e : ev) MF_HIP_CHECK(hipEventCreate(&e));
        }
        int rc = MF_OK;
        for (int32_t s = 0; s < nb; ++s) {
            const int32_t b = seq ? seq[s] : s;
            a.off = offs[b];
            a.n = offs[b + 1] - offs[b];
            if (a.n <= 0) continue;
            const int64_t waves = (a.n + RPW - 1) / RPW;
            const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
            if (kernel_ms) { hipError_t e = hipEventRecord(ev[2 * s], stream); if (e) { rc = hip_fail(e, "hipEventRecord"); break; } }
            hipLaunchKernelGGL((k_sgd_batch<T, GS, V, KERN>), dim3((unsigned)blocks),
                               dim3(kBlock), 0, stream, a);
            if (kernel_ms) { hipError_t e = hipEventRecord(ev[2 * s + 1], stream); if (e) { rc = hip_fail(e, "hipEventRecord"); break; } }
        }
        hipError_t le = hipGetLastError();
        if (rc == MF_OK && le != hipSuccess) rc = hip_fail(le, "k_sgd_batch launch");
        if (kernel_ms) {
            double tot = 0.0;
            if (rc == MF_OK) {
                hipError_t e = hipStreamSynchronize(stream);
                if (e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize");
            }
            for (int32_t s = 0; rc == MF_OK && s < nb; ++s) {
                const int32_t b = seq ? seq[s] : s;
                if (offs[b + 1] - offs[b] <= 0) continue;
                float ms = 0.f;
                hipError_t e = hipEventElapsedTime(&ms, ev[2 * s], ev[2 * s + 1]);
                if (e != hipSuccess) { rc = hip_fail(e, "hipEventElapsedTime"); break; }
                tot += ms;
            }
            for (auto& e : ev) (void)hipEventDestroy(e);
            if (rc == MF_OK) *kernel_ms = tot;
        }
        return rc;
    }
};

struct ReadLaunch {
    const int32_t* u; const int32_t* i; const void* r; int64_t n;
    double mu; const void* bu; const void* bi; const void* P; const void* Q;
    int32_t k; double gamma, lo, hi; int32_t bound; void* out;
    double* partials; double* sse_out; hipStream_t stream;

    template <typename T, int GS, int V, int KERN>
    int run() {
        constexpr int RPW = Tile<V>::U * (kWave / GS);
        ReadArgs<T> a;
        a.u = u; a.i = i; a.r = static_cast<const T*>(r);
        a.P = static_cast<const T*>(P); a.Q = static_cast<const T*>(Q);
        a.Bu = static_cast<const T*>(bu); a.Bi = static_cast<const T*>(bi);
        a.n = n; a.k = k; a.bound = bound; a.out = static_cast<T*>(out);
        a.partials = partials;
        a.h = make_hyper<T>(mu, 0.0, 0.0, gamma, lo, hi);
        const int blocks = read_blocks(n, RPW);
        if (sse_out) {
            hipLaunchKernelGGL((k_read<T, GS, V, KERN, true>), dim3(blocks), dim3(kBlock), 0,
                               stream, a);
            hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(kBlock), 0, stream,
                               (const double*)partials, blocks, sse_out);
        } else {
            hipLaunchKernelGGL((k_read<T, GS, V, KERN, false>), dim3(blocks), dim3(kBlock), 0,
                               stream, a);
        }
        MF_HIP_CHECK(hipGetLastError());
        return MF_OK;
    }
};

}  // namespace mf

using namespace mf;

extern "C" int mf_max_factors(void) { return kMaxFactors; }

extern "C" int mf_sgd_epoch(const int32_t* user_ids, const int32_t* item_ids,
                            const void* ratings, int64_t n_ratings,
                            const int32_t* order, const int64_t* batch_offsets,
                            const int32_t* batch_seq, int32_t n_batches,
                            double global_mean, void* user_biases,
                            void* item_biases, void* user_features,
                            void* item_features, int32_t n_users,
                            int32_t n_items, int32_t n_factors, int32_t kernel,
                            int32_t dtype, double gamma, double lr, double reg,
                            double min_rating, double max_rating,
                            int32_t update_user_params,
                            int32_t update_item_params, int32_t flags,
                            void* stream, double* kernel_ms) {
    if (n_ratings < 0 || n_batches < 0 || n_users < 0 || n_items < 0) {
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
        if (batch_seq && (batch_seq[b] < 0 || batch_seq[b] >= n_batches)) {
            set_error("batch_seq[%d] = %d out of range", b, batch_seq[b]);
            return MF_ERR_INVALID;
        }
    }
    if (n_ratings > 0 && (!user_ids || !item_ids || !ratings)) {
        set_error("NULL triple array");
        return MF_ERR_INVALID;
    }
    if (kernel_ms) *kernel_ms = 0.0;
    if (n_batches == 0 || n_ratings == 0) return MF_OK;
    SgdLaunch L{user_ids, item_ids, ratings, order, batch_offsets, batch_seq, n_batches,
                global_mean, user_biases, item_biases, user_features, item_features,
                n_factors, gamma, lr, reg, min_rating, max_rating,
                update_user_params ? 1 : 0, update_item_params ? 1 : 0, flags,
                (hipStream_t)stream, kernel_ms};
    return dispatch(dtype, n_factors, kernel, L);
}

extern "C" size_t mf_sse_workspace_bytes(int64_t n_ratings) {
    (void)n_ratings;
    return sizeof(double) * (size_t)kSseMaxBlocks;
}

extern "C" int mf_sse(const int32_t* user_ids, const int32_t* item_ids,
                      const void* ratings, int64_t n_ratings,
                      double global_mean, const void* user_biases,
                      const void* item_biases, const void* user_features,
                      const void* item_features, int32_t n_factors,
                      int32_t kernel, int32_t dtype, double gamma,
                      double min_rating, double max_rating, void* workspace,
                      double* sse_out, void* stream) {
    if (n_ratings < 0 || !sse_out || !workspace) {
        set_error("mf_sse: bad arguments");
        return MF_ERR_INVALID;
    }
    if (n_ratings == 0) {
        MF_HIP_CHECK(hipMemsetAsync(sse_out, 0, sizeof(double), (hipStream_t)stream));
        return MF_OK;
    }
    ReadLaunch L{user_ids, item_ids, ratings, n_ratings, global_mean, user_biases,
                 item_biases, user_features, item_features, n_factors, gamma,
                 min_rating, max_rating, 0, nullptr, (double*)workspace, sse_out,
                 (hipStream_t)stream};
    return dispatch(dtype, n_factors, kernel, L);
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
    ReadLaunch L{user_ids, item_ids, nullptr, n_pairs, global_mean, user_biases,
                 item_biases, user_features, item_features, n_factors, gamma,
                 min_rating, max_rating, bound_ratings ? 1 : 0, out, nullptr,
                 nullptr, (hipStream_t)stream};
    return dispatch(dtype, n_factors, kernel, L);
}
