// mf_topk.hip -- batched recommend(): score every item for a set of users and
// keep the best `amount` per user (recommender_base.py:214-271 scores all
// candidate items with predict(bound_ratings=False) and sorts descending).
//
// Stage 1 (k_topk_scores): one wave per (user, chunk of items); the user's
//   factor row stays in registers, item rows stream from HBM/L2; each score
//   becomes a 64-bit order-preserving key (1 = NaN); k_topk_exclude then
//   zeroes the keys of the excluded (user, item) pairs (CSR list).
// Stage 2 (k_topk_select): one workgroup per user: 8-pass radix select of
//   the amount-th key (LDS histograms), collect, bitonic sort in LDS by
//   (score desc, item id asc).
#include <climits>

#include "mf_common.hpp"

namespace mf {

constexpr int kTopkMaxAmount = 2048;
constexpr int kTopkItemsPerWave = 256;

__device__ __forceinline__ uint64_t order_key(double s) {
    if (s != s) return 1ull;                       // NaN: below every number
    uint64_t b = (uint64_t)__double_as_longlong(s);
    return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_score(uint64_t k) {
    if (k <= 1ull) return __longlong_as_double(0x7ff8000000000000LL);
    uint64_t b = (k & 0x8000000000000000ull) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
}

template <typename T>
struct TopkArgs {
    const int32_t* users;
    const T* P; const T* Q; const T* Bu; const T* Bi;
    int32_t n_items;
    int32_t k;
    Hyper<T> h;
    uint64_t* keys;
};

template <typename T, int GS, int V, int KERN>
__global__ __launch_bounds__(kBlock) void k_topk_scores(TopkArgs<T> A) {
    constexpr int R = kWave / GS;
    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS, l = lane % GS;
    const int qy = blockIdx.y;
    const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    const int64_t i0 = wave * kTopkItemsPerWave;
    if (i0 >= A.n_items) return;
    const int k = A.k;
    const int32_t uu = A.users[qy];
    const bool uk = uu >= 0;
    T p[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int f = l + v * GS;
        p[v] = (uk && f < k) ? A.P[(int64_t)uu * k + f] : (T)0;
    }
    const T bu = (uk && KERN != MF_RBF) ? A.Bu[uu] : (T)0;
    const int64_t iend = min((int64_t)A.n_items, i0 + kTopkItemsPerWave);
    uint64_t* keys = A.keys + (int64_t)qy * A.n_items;
    for (int64_t ib = i0; ib < iend; ib += R) {
        const int64_t it = ib + g;
        const bool have = it < iend;
        const T* qr = A.Q + (have ? it : 0) * k;
        T s = (T)0;
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int f = l + v * GS;
            const T qf = (have && f < k) ? qr[f] : (T)0;
            if constexpr (KERN == MF_RBF) {
                const T d = p[v] - qf;
                s = s + d * d;
            } else {
                s = s + p[v] * qf;
            }
        }
        s = group_sum<GS>(s);
        if (have && l == 0) {
            const T bi = (KERN != MF_RBF) ? A.Bi[it] : (T)0;
            T pred;
            if constexpr (KERN == MF_LINEAR) pred = ((A.h.mu + bi) + bu) + s;
            else if constexpr (KERN == MF_SIGMOID)
                pred = A.h.a + A.h.c * ((T)1 / ((T)1 + dexp<T>(-(((A.h.mu + bu) + bi) + s))));
            else pred = A.h.a + A.h.c * dexp<T>((-A.h.gamma) * s);
            keys[it] = order_key((double)pred);
        }
    }
}

// excluded (query, item) pairs: key 0, below every candidate.  One workgroup
// per query walks its CSR list (ids outside [0, n_items) are ignored).
__global__ __launch_bounds__(kBlock) void k_topk_exclude(uint64_t* __restrict__ keys,
                                                         int32_t n_items,
                                                         const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ items) {
    const int qy = blockIdx.x;
    for (int64_t x = ptr[qy] + threadIdx.x; x < ptr[qy + 1]; x += kBlock) {
        const int32_t it = items[x];
        if (it >= 0 && it < n_items) keys[(int64_t)qy * n_items + it] = 0ull;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_topk_select(const uint64_t* __restrict__ all_keys,
                                                        int32_t n_items, int32_t amount,
                                                        int32_t a2, int32_t* out_items,
                                                        T* out_scores) {
    const int qy = blockIdx.x;
    const int tid = threadIdx.x;
    const uint64_t* K = all_keys + (int64_t)qy * n_items;
    __shared__ unsigned hist[256];
    __shared__ uint64_t s_key[kTopkMaxAmount];
    __shared__ int32_t s_idx[kTopkMaxAmount];
    __shared__ int s_cnt, s_rem, s_want, s_base;
    __shared__ uint64_t s_prefix, s_mask;
    __shared__ int wsum[kWavesPerBlock];

    // candidates
    int c = 0;
    for (int i = tid; i < n_items; i += kBlock) c += K[i] != 0ull;
    c = wave_sum(c);
    if ((tid & 63) == 0) wsum[tid / kWave] = c;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) t += wsum[w];
        s_want = t < amount ? t : amount;
        s_rem = s_want;
        s_prefix = 0ull;
        s_mask = 0ull;
        s_cnt = 0;
    }
    __syncthreads();
    const int want = s_want;
    if (want > 0) {
        for (int d = 7; d >= 0; --d) {
            for (int b = tid; b < 256; b += kBlock) hist[b] = 0u;
            __syncthreads();
            const uint64_t pre = s_prefix, msk = s_mask;
            for (int i = tid; i < n_items; i += kBlock) {
                const uint64_t kk = K[i];
                if (kk != 0ull && (kk & msk) == pre) atomicAdd(&hist[(kk >> (8 * d)) & 255u], 1u);
            }
            __syncthreads();
            if (tid == 0) {
                int cum = 0, sel = 0;
                for (int b = 255; b >= 0; --b) {
                    if (cum + (int)hist[b] >= s_rem) { sel = b; break; }
                    cum += (int)hist[b];
                }
                s_rem -= cum;
                s_prefix |= (uint64_t)sel << (8 * d);
                s_mask |= 0xffull << (8 * d);
            }
            __syncthreads();
        }
        const uint64_t thr = s_prefix;
        // every key above the threshold
        for (int i = tid; i < n_items; i += kBlock) {
            const uint64_t kk = K[i];
            if (kk > thr) {
                const int slot = atomicAdd(&s_cnt, 1);
                s_key[slot] = kk;
                s_idx[slot] = i;
            }
        }
        __syncthreads();
        // the s_rem lowest-id items whose key equals the threshold
        if (tid == 0) s_base = s_cnt;
        __syncthreads();
        for (int i0 = 0; i0 < n_items && s_rem > 0; i0 += kBlock) {
            const int i = i0 + tid;
            const bool m = i < n_items && K[i] == thr;
            const unsigned long long bal = __ballot(m);
            const int w = tid / kWave, ln = tid & 63;
            if (ln == 0) wsum[w] = __popcll(bal);
            __syncthreads();
            int before = 0;
            for (int x = 0; x < w; ++x) before += wsum[x];
            before += __popcll(bal & ((1ull << ln) - 1ull));
            if (m && before < s_rem) {
                s_key[s_base + before] = thr;
                s_idx[s_base + before] = i;
            }
            __syncthreads();
            if (tid == 0) {
                int tot = 0;
                for (int x = 0; x < kWavesPerBlock; ++x) tot += wsum[x];
                const int took = tot < s_rem ? tot : s_rem;
                s_base += took;
                s_rem -= took;
            }
            __syncthreads();
        }
    }
    __syncthreads();
    // pad to a2 and bitonic-sort by (key desc, idx asc)
    for (int s = want + tid; s < a2; s += kBlock) { s_key[s] = 0ull; s_idx[s] = INT_MAX; }
    __syncthreads();
    for (int sz = 2; sz <= a2; sz <<= 1) {
        for (int st = sz >> 1; st > 0; st >>= 1) {
            for (int x = tid; x < a2; x += kBlock) {
                const int y = x ^ st;
                if (y > x) {
                    const bool desc = (x & sz) == 0;
                    const uint64_t kx = s_key[x], ky = s_key[y];
                    const int ix = s_idx[x], iy = s_idx[y];
                    // "x before y" in the final order
                    const bool xfirst = kx > ky || (kx == ky && ix < iy);
                    if (desc ? !xfirst : xfirst) {
                        s_key[x] = ky; s_key[y] = kx;
                        s_idx[x] = iy; s_idx[y] = ix;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int s = tid; s < amount; s += kBlock) {
        const bool ok = s < want;
        out_items[(int64_t)qy * amount + s] = ok ? s_idx[s] : -1;
        out_scores[(int64_t)qy * amount + s] =
            ok ? (T)key_score(s_key[s]) : (T)__longlong_as_double(0x7ff8000000000000LL);
    }
}

struct TopkLaunch {
    const int32_t* users; int32_t nq; double mu; const void* bu; const void* bi;
    const void* P; const void* Q; int32_t n_items; int32_t k; double gamma, lo, hi;
    const int64_t* ex_ptr; const int32_t* ex_items; int32_t amount; void* ws; int32_t* out_items; void* out_scores;
    hipStream_t stream;

    template <typename T, int GS, int V, int KERN>
    int run() {
        TopkArgs<T> a;
        a.users = users; a.P = (const T*)P; a.Q = (const T*)Q;
        a.Bu = (const T*)bu; a.Bi = (const T*)bi;
        a.n_items = n_items; a.k = k; a.h = make_hyper<T>(mu, 0.0, 0.0, gamma, lo, hi);
        a.keys = (uint64_t*)ws;
        const int64_t waves = ((int64_t)n_items + kTopkItemsPerWave - 1) / kTopkItemsPerWave;
        const unsigned bx = (unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
        hipLaunchKernelGGL((k_topk_scores<T, GS, V, KERN>), dim3(bx, (unsigned)nq),
                           dim3(kBlock), 0, stream, a);
        if (ex_ptr && ex_items)
            hipLaunchKernelGGL(k_topk_exclude, dim3((unsigned)nq), dim3(kBlock), 0, stream,
                               a.keys, n_items, ex_ptr, ex_items);
        int a2 = 1;
        while (a2 < amount) a2 <<= 1;
        hipLaunchKernelGGL(k_topk_select<T>, dim3((unsigned)nq), dim3(kBlock), 0, stream,
                           (const uint64_t*)ws, n_items, amount, a2, out_items, (T*)out_scores);
        MF_HIP_CHECK(hipGetLastError());
        return MF_OK;
    }
};

}  // namespace mf

#include "mf_dispatch.hpp"

using namespace mf;

extern "C" size_t mf_topk_workspace_bytes(int32_t n_query, int32_t n_items, int32_t amount) {
    (void)amount;
    if (n_query <= 0 || n_items <= 0) return 0;
    return sizeof(uint64_t) * (size_t)n_query * (size_t)n_items;
}

extern "C" int mf_topk(const int32_t* query_users, int32_t n_query, double global_mean,
                       const void* user_biases, const void* item_biases,
                       const void* user_features, const void* item_features, int32_t n_items,
                       int32_t n_factors, int32_t kernel, int32_t dtype, double gamma,
                       double min_rating, double max_rating, const int64_t* exclude_ptr,
                       const int32_t* exclude_items, int32_t amount, void* workspace, int32_t* out_items, void* out_scores,
                       void* stream) {
    if (n_query < 0 || n_items < 0 || amount < 0 || amount > kTopkMaxAmount) {
        set_error("mf_topk: need 0 <= amount <= %d and non-negative sizes", kTopkMaxAmount);
        return MF_ERR_INVALID;
    }
    if (n_query == 0 || amount == 0) return MF_OK;
    if (!workspace || !out_items || !out_scores || !query_users) {
        set_error("mf_topk: NULL buffer");
        return MF_ERR_INVALID;
    }
    if (n_items == 0) {
        // nothing to rank: every slot is padding
        set_error("mf_topk: n_items == 0");
        return MF_ERR_INVALID;
    }
    TopkLaunch L{query_users, n_query, global_mean, user_biases, item_biases, user_features,
                 item_features, n_items, n_factors, gamma, min_rating, max_rating, exclude_ptr,
                 exclude_items, amount, workspace, out_items, out_scores, (hipStream_t)stream};
    return dispatch(dtype, n_factors, kernel, L);
}
