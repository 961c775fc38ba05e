// mf_bias.hip -- BaselineModel (bias-only) kernels, baseline_model.py.
//
// The bias model is the k = 0 member of the family: one scalar per user and
// per item.  One lane per rating; SGD uses the same conflict-free batch
// schedules as the factor model; ALS sums each id's ratings sequentially in
// the reference's row order through CSR lists, so results are bit-identical
// to the reference loop (baseline_model.py:326-348).
#include "mf_common.hpp"

namespace mf {

template <typename T>
__global__ __launch_bounds__(kBlock) void k_bias_sgd(const int32_t* __restrict__ u,
                                                     const int32_t* __restrict__ it,
                                                     const T* __restrict__ r,
                                                     const int32_t* __restrict__ order,
                                                     int64_t off, int64_t n, T mu, T* bu, T* bi,
                                                     T lr, T reg, int upd_user, int upd_item) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n) return;
    const int64_t pos = off + t;
    const int64_t j = order ? (int64_t)order[pos] : pos;
    const int32_t uu = u[j], ii = it[j];
    const T pred = (mu + bu[uu]) + bi[ii];                       // :259
    const T err = r[j] - pred;                                   // :260
    if (upd_user) bu[uu] = bu[uu] + lr * (err - reg * bu[uu]);   // :264
    if (upd_item) bi[ii] = bi[ii] + lr * (err - reg * bi[ii]);   // :266
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_bias_sse(const int32_t* __restrict__ u,
                                                     const int32_t* __restrict__ it,
                                                     const T* __restrict__ r, int64_t n, T mu,
                                                     const T* __restrict__ bu,
                                                     const T* __restrict__ bi,
                                                     double* partials) {
    double acc = 0.0;
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * kBlock) {
        const T pred = (mu + bu[u[j]]) + bi[it[j]];               // :207
        const T err = r[j] - pred;                                // :208
        acc += (double)err * (double)err;
    }
    acc = wave_sum(acc);
    __shared__ double red[kWavesPerBlock];
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < kWavesPerBlock; ++w) s += red[w];
        partials[blockIdx.x] = s;
    }
}

__global__ void k_sum_partials_bias(const double* part, int n, double* out) {
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

// One half-sweep of the bias ALS: for every id x of the solved side,
//   b[x] = (sum over its ratings j, in row order, of (r_j - mu) - other[o_j])
//          / (reg + count_x)
// baseline_model.py:329-337 (users) and :340-348 (items).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_bias_als_half(const int32_t* __restrict__ other_ids,
                                                          const T* __restrict__ r, T mu,
                                                          const int64_t* __restrict__ ptr,
                                                          const int32_t* __restrict__ list,
                                                          const T* __restrict__ other, T* b,
                                                          int32_t n_ids, T reg) {
    const int32_t x = blockIdx.x * kBlock + threadIdx.x;
    if (x >= n_ids) return;
    T s = (T)0;
    const int64_t e = ptr[x + 1];
    for (int64_t p = ptr[x]; p < e; ++p) {
        const int32_t j = list[p];
        s += (r[j] - mu) - other[other_ids[j]];
    }
    const T cnt = (T)(e - ptr[x]);
    b[x] = s / (reg + cnt);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_bias_predict(const int32_t* __restrict__ u,
                                                         const int32_t* __restrict__ it,
                                                         int64_t n, T mu,
                                                         const T* __restrict__ bu,
                                                         const T* __restrict__ bi, int bound,
                                                         T lo, T hi, T* out) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    T pred = mu;                                                  // :400
    if (u[j] != -1) pred += bu[u[j]];                             // :402-403
    if (it[j] != -1) pred += bi[it[j]];                           // :404-405
    if (bound) {                                                  // :408-412
        if (pred > hi) pred = hi;
        else if (pred < lo) pred = lo;
    }
    out[j] = pred;
}

constexpr int kBiasSseBlocks = 1024;

template <typename T>
static int bias_sgd_run(const int32_t* u, const int32_t* it, const void* r, const int32_t* order,
                        const int64_t* offs, const int32_t* seq, int32_t nb, double mu, void* bu,
                        void* bi, double lr, double reg, int uu, int ui, hipStream_t s) {
    for (int32_t q = 0; q < nb; ++q) {
        const int32_t b = seq ? seq[q] : q;
        const int64_t n = offs[b + 1] - offs[b];
        if (n <= 0) continue;
        hipLaunchKernelGGL(k_bias_sgd<T>, dim3((unsigned)((n + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, s, u, it, (const T*)r, order, offs[b], n, (T)mu,
                           (T*)bu, (T*)bi, (T)lr, (T)reg, uu, ui);
    }
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}

}  // namespace mf

using namespace mf;

extern "C" int mf_bias_sgd_epoch(const int32_t* user_ids, const int32_t* item_ids,
                                 const void* ratings, int64_t n_ratings, const int32_t* order,
                                 const int64_t* batch_offsets, int32_t n_batches,
                                 const int32_t* batch_seq, int32_t n_seq,
                                 double global_mean, void* user_biases,
                                 void* item_biases, int32_t dtype, double lr, double reg,
                                 int32_t update_user_params, int32_t update_item_params,
                                 void* stream) {
    if (n_ratings < 0 || n_batches < 0 || (n_batches > 0 && !batch_offsets)) {
        set_error("mf_bias_sgd_epoch: bad arguments");
        return MF_ERR_INVALID;
    }
    for (int32_t b = 0; b < n_batches; ++b) {
        if (batch_offsets[b] < 0 || batch_offsets[b + 1] < batch_offsets[b] ||
            batch_offsets[b + 1] > n_ratings) {
            set_error("mf_bias_sgd_epoch: invalid batch %d", b);
            return MF_ERR_INVALID;
        }
    }
    const int32_t n_launch = batch_seq ? n_seq : n_batches;
    for (int32_t q = 0; batch_seq && q < n_seq; ++q) {
        if (batch_seq[q] < 0 || batch_seq[q] >= n_batches) {
            set_error("mf_bias_sgd_epoch: batch_seq[%d] out of range", q);
            return MF_ERR_INVALID;
        }
    }
    if (n_ratings == 0 || n_launch <= 0) return MF_OK;
    hipStream_t s = (hipStream_t)stream;
    const int uu = update_user_params ? 1 : 0, ui = update_item_params ? 1 : 0;
    if (dtype == MF_F32)
        return bias_sgd_run<float>(user_ids, item_ids, ratings, order, batch_offsets, batch_seq,
                                   n_launch, global_mean, user_biases, item_biases, lr, reg, uu,
                                   ui, s);
    if (dtype == MF_F64)
        return bias_sgd_run<double>(user_ids, item_ids, ratings, order, batch_offsets, batch_seq,
                                    n_launch, global_mean, user_biases, item_biases, lr, reg,
                                    uu, ui, s);
    set_error("unknown dtype code %d", dtype);
    return MF_ERR_INVALID;
}

extern "C" int mf_bias_sse(const int32_t* user_ids, const int32_t* item_ids, const void* ratings,
                           int64_t n_ratings, double global_mean, const void* user_biases,
                           const void* item_biases, int32_t dtype, void* workspace,
                           double* sse_out, void* stream) {
    if (n_ratings < 0 || !workspace || !sse_out) {
        set_error("mf_bias_sse: bad arguments");
        return MF_ERR_INVALID;
    }
    hipStream_t s = (hipStream_t)stream;
    if (n_ratings == 0) {
        MF_HIP_CHECK(hipMemsetAsync(sse_out, 0, sizeof(double), s));
        return MF_OK;
    }
    const int64_t need = (n_ratings + kBlock - 1) / kBlock;
    const int blocks = (int)(need < kBiasSseBlocks ? need : kBiasSseBlocks);
    double* part = (double*)workspace;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(k_bias_sse<float>, dim3(blocks), dim3(kBlock), 0, s, user_ids,
                           item_ids, (const float*)ratings, n_ratings, (float)global_mean,
                           (const float*)user_biases, (const float*)item_biases, part);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(k_bias_sse<double>, dim3(blocks), dim3(kBlock), 0, s, user_ids,
                           item_ids, (const double*)ratings, n_ratings, global_mean,
                           (const double*)user_biases, (const double*)item_biases, part);
    else {
        set_error("unknown dtype code %d", dtype);
        return MF_ERR_INVALID;
    }
    hipLaunchKernelGGL(k_sum_partials_bias, dim3(1), dim3(kBlock), 0, s, (const double*)part,
                       blocks, sse_out);
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}

extern "C" int mf_bias_als_epoch(const int32_t* user_ids, const int32_t* item_ids,
                                 const void* ratings, double global_mean, void* user_biases,
                                 void* item_biases, int32_t n_users, int32_t n_items,
                                 const int64_t* user_ptr, const int32_t* user_list,
                                 const int64_t* item_ptr, const int32_t* item_list,
                                 int32_t dtype, double reg, void* stream) {
    if (n_users < 0 || n_items < 0 || !user_ptr || !item_ptr) {
        set_error("mf_bias_als_epoch: bad arguments");
        return MF_ERR_INVALID;
    }
    hipStream_t s = (hipStream_t)stream;
    const unsigned gu = (unsigned)((n_users + kBlock - 1) / kBlock);
    const unsigned gi = (unsigned)((n_items + kBlock - 1) / kBlock);
#define MF_ALS(T)                                                                              \
    do {                                                                                       \
        if (gu) hipLaunchKernelGGL(k_bias_als_half<T>, dim3(gu), dim3(kBlock), 0, s, item_ids, \
                                   (const T*)ratings, (T)global_mean, user_ptr, user_list,     \
                                   (const T*)item_biases, (T*)user_biases, n_users, (T)reg);   \
        if (gi) hipLaunchKernelGGL(k_bias_als_half<T>, dim3(gi), dim3(kBlock), 0, s, user_ids, \
                                   (const T*)ratings, (T)global_mean, item_ptr, item_list,     \
                                   (const T*)user_biases, (T*)item_biases, n_items, (T)reg);   \
    } while (0)
    if (dtype == MF_F32) MF_ALS(float);
    else if (dtype == MF_F64) MF_ALS(double);
    else {
        set_error("unknown dtype code %d", dtype);
        return MF_ERR_INVALID;
    }
#undef MF_ALS
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}

extern "C" int mf_bias_predict(const int32_t* user_ids, const int32_t* item_ids, int64_t n_pairs,
                               double global_mean, const void* user_biases,
                               const void* item_biases, int32_t dtype, double min_rating,
                               double max_rating, int32_t bound_ratings, void* out,
                               void* stream) {
    if (n_pairs < 0 || (n_pairs > 0 && !out)) {
        set_error("mf_bias_predict: bad arguments");
        return MF_ERR_INVALID;
    }
    if (n_pairs == 0) return MF_OK;
    hipStream_t s = (hipStream_t)stream;
    const unsigned g = (unsigned)((n_pairs + kBlock - 1) / kBlock);
    if (dtype == MF_F32)
        hipLaunchKernelGGL(k_bias_predict<float>, dim3(g), dim3(kBlock), 0, s, user_ids,
                           item_ids, n_pairs, (float)global_mean, (const float*)user_biases,
                           (const float*)item_biases, bound_ratings ? 1 : 0, (float)min_rating,
                           (float)max_rating, (float*)out);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(k_bias_predict<double>, dim3(g), dim3(kBlock), 0, s, user_ids,
                           item_ids, n_pairs, global_mean, (const double*)user_biases,
                           (const double*)item_biases, bound_ratings ? 1 : 0, min_rating,
                           max_rating, (double*)out);
    else {
        set_error("unknown dtype code %d", dtype);
        return MF_ERR_INVALID;
    }
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}

// ---------------------------------------------------------------------------
// Replica exchange helper (multi-GPU): cur -= base / cur += base, 16-B lanes.
namespace mf {
template <typename T>
__global__ __launch_bounds__(kBlock) void k_replica_delta(T* __restrict__ cur,
                                                          const T* __restrict__ base, int64_t n,
                                                          int mode) {
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * kBlock) {
        const T b = base[j];
        cur[j] = mode == MF_DELTA_TAKE ? cur[j] - b : cur[j] + b;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_replica_apply(T* __restrict__ cur,
                                                          const T* __restrict__ delta, int64_t n,
                                                          T scale) {
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * kBlock)
        cur[j] = cur[j] + scale * delta[j];
}
}  // namespace mf

extern "C" int mf_replica_apply(void* cur, const void* delta, int64_t n, int32_t dtype,
                                double scale, void* stream) {
    if (n < 0 || (n > 0 && (!cur || !delta))) {
        set_error("mf_replica_apply: bad arguments");
        return MF_ERR_INVALID;
    }
    if (n == 0) return MF_OK;
    hipStream_t s = (hipStream_t)stream;
    const int64_t need = (n + kBlock - 1) / kBlock;
    const unsigned g = (unsigned)(need < 4096 ? need : 4096);
    if (dtype == MF_F32)
        hipLaunchKernelGGL(k_replica_apply<float>, dim3(g), dim3(kBlock), 0, s, (float*)cur,
                           (const float*)delta, n, (float)scale);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(k_replica_apply<double>, dim3(g), dim3(kBlock), 0, s, (double*)cur,
                           (const double*)delta, n, scale);
    else {
        set_error("unknown dtype code %d", dtype);
        return MF_ERR_INVALID;
    }
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}

extern "C" int mf_replica_delta(void* cur, const void* base, int64_t n, int32_t dtype,
                                int32_t mode, void* stream) {
    if (n < 0 || (n > 0 && (!cur || !base)) || (mode != MF_DELTA_TAKE && mode != MF_DELTA_APPLY)) {
        set_error("mf_replica_delta: bad arguments");
        return MF_ERR_INVALID;
    }
    if (n == 0) return MF_OK;
    hipStream_t s = (hipStream_t)stream;
    const int64_t need = (n + kBlock - 1) / kBlock;
    const unsigned g = (unsigned)(need < 4096 ? need : 4096);
    if (dtype == MF_F32)
        hipLaunchKernelGGL(k_replica_delta<float>, dim3(g), dim3(kBlock), 0, s, (float*)cur,
                           (const float*)base, n, mode);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(k_replica_delta<double>, dim3(g), dim3(kBlock), 0, s, (double*)cur,
                           (const double*)base, n, mode);
    else {
        set_error("unknown dtype code %d", dtype);
        return MF_ERR_INVALID;
    }
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}

// ---------------------------------------------------------------------------
// Relabelled strata plans (engine._epoch_regroup): the
// parameters move into a plan's labelling and back -- up to 4 row arrays (P,
// Q, b_u, b_i) permuted in ONE launch.  Job j: rows of row_bytes[j] bytes;
// gather (mode 0): dst[r] = src[idx[r]], scatter (mode 1): dst[idx[r]] =
// src[r].  16-B accesses where a row is a whole number of them, else 8 / 4 B.
namespace mf {
struct PermJobs {
    const char* src[MF_PERMUTE_MAX_JOBS];
    char* dst[MF_PERMUTE_MAX_JOBS];
    const int64_t* idx[MF_PERMUTE_MAX_JOBS];
    int64_t rows[MF_PERMUTE_MAX_JOBS];
    int32_t row_bytes[MF_PERMUTE_MAX_JOBS];
    int32_t n;
    int32_t mode;
};

template <typename V>
__device__ __forceinline__ void permute_job(const PermJobs& J, int j, int64_t t0, int64_t stride) {
    const int per = J.row_bytes[j] / (int)sizeof(V);               // vectors per row
    const int64_t total = J.rows[j] * per;
    const V* src = reinterpret_cast<const V*>(J.src[j]);
    V* dst = reinterpret_cast<V*>(J.dst[j]);
    for (int64_t t = t0; t < total; t += stride) {
        const int64_t r = t / per;
        const int c = (int)(t - r * per);
        const int64_t o = J.idx[j][r];
        if (J.mode == 0) dst[r * per + c] = src[o * per + c];
        else dst[o * per + c] = src[r * per + c];
    }
}

__global__ __launch_bounds__(kBlock) void k_permute_rows(PermJobs J) {
    const int j = blockIdx.y;
    const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int rb = J.row_bytes[j];
    const uintptr_t al = reinterpret_cast<uintptr_t>(J.src[j]) | reinterpret_cast<uintptr_t>(J.dst[j]);
    if (rb % 16 == 0 && al % 16 == 0) permute_job<uint4>(J, j, t0, stride);
    else if (rb % 8 == 0 && al % 8 == 0) permute_job<uint2>(J, j, t0, stride);
    else permute_job<uint32_t>(J, j, t0, stride);
}
void touch_bias(hipStream_t s) { hipLaunchKernelGGL(k_touch<5>, dim3(1), dim3(64), 0, s); }

}  // namespace mf

extern "C" int mf_permute_rows(int32_t n_jobs, void* const* dst, const void* const* src,
                               const int64_t* const* idx, const int64_t* n_rows,
                               const int32_t* row_bytes, int32_t mode, void* stream) {
    if (n_jobs < 0 || n_jobs > MF_PERMUTE_MAX_JOBS || (mode != 0 && mode != 1) ||
        (n_jobs > 0 && (!dst || !src || !idx || !n_rows || !row_bytes))) {
        set_error("mf_permute_rows: bad arguments");
        return MF_ERR_INVALID;
    }
    PermJobs J{};
    J.mode = mode;
    int64_t most = 0;
    for (int32_t j = 0; j < n_jobs; ++j) {
        if (n_rows[j] < 0 || row_bytes[j] <= 0 || row_bytes[j] % 4 != 0 ||
            (n_rows[j] > 0 && (!dst[j] || !src[j] || !idx[j]))) {
            set_error("mf_permute_rows: job %d invalid", j);
            return MF_ERR_INVALID;
        }
        if (n_rows[j] == 0) continue;
        J.src[J.n] = static_cast<const char*>(src[j]);
        J.dst[J.n] = static_cast<char*>(dst[j]);
        J.idx[J.n] = idx[j];
        J.rows[J.n] = n_rows[j];
        J.row_bytes[J.n] = row_bytes[j];
        most = std::max<int64_t>(most, n_rows[j] * (row_bytes[j] / 4));
        ++J.n;
    }
    if (J.n == 0) return MF_OK;
    const int64_t need = (most / 4 + kBlock - 1) / kBlock;            // ~one 16-B access per thread
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(need, 8192));
    hipLaunchKernelGGL(k_permute_rows, dim3(g, (unsigned)J.n), dim3(kBlock), 0,
                       (hipStream_t)stream, J);
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}
