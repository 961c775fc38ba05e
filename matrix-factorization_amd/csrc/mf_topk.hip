// mf_topk.hip -- batched recommend(): score every item for a set of users and
// keep the best `amount` per user (recommender_base.py:214-271 scores all
// candidate items with predict(bound_ratings=False) and sorts descending).
//
// amount <= 64 (recommend's default 10): k_topk_fused + k_topk_merge (below:
// scores never leave the chip).  Larger amounts, or MF_TOPK_TWO_STAGE=1:
// Stage 1 (k_topk_scores): one wave per (user, chunk of items); the user's
//   factor row stays in registers, item rows stream from HBM/L2; each score
//   becomes a 64-bit order-preserving key (1 = NaN); k_topk_exclude then
//   zeroes the keys of the excluded (user, item) pairs (CSR list).
// Stage 2 (k_topk_select): one workgroup per user: 8-pass radix select of
//   the amount-th key (LDS histograms), collect, bitonic sort in LDS by
//   (score desc, item id asc).
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "mf_common.hpp"

namespace mf {

constexpr int kTopkMaxAmount = 2048;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
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

// ---------------------------------------------------------------- fused
// k_topk_fused: the same scores (k_read's arithmetic: lane partials of the
// scalar layout, group_sum<GS>, predict_one) without materialising them.
// Workgroup (split x, user block y) scores items [ibeg, iend) of its split
// against kFusedUsers users whose rows sit in registers; every wave walks
// one item at a time.  A score enters the user's LDS candidate list only if
// it beats the list's current threshold (the amount-th best so far, in the
// order (score desc, item id asc)); excluded items are looked up (binary
// search in the user's sorted CSR list) only for such candidates.  After
// every chunk of items a barrier; lists that grew past A2 + chunk are
// bitonic-sorted and cut to the best A2 (A2 = amount rounded up to a power
// of two), raising the threshold.  At the end each list is sorted and its
// best `amount` go to the split's partial output; k_topk_merge merges the
// splits per user.  Random scores settle the threshold after a few chunks,
// so almost every score costs its reduction and one compare.
constexpr int kFusedUsers = 16;          // users per workgroup (registers)
constexpr int kFusedMaxAmount = 64;
constexpr int kFusedItemsPerWave = 16;   // items per wave between barriers
constexpr int kFusedChunk = kWavesPerBlock * kFusedItemsPerWave;
constexpr int kFusedCap = 256;           // list capacity: A2 + 2 chunks <= 256

struct Cand { uint64_t key; int32_t id; };

// (key desc, id asc): does (ka, ia) come before (kb, ib)?
__device__ __forceinline__ bool cand_before(uint64_t ka, int32_t ia, uint64_t kb, int32_t ib) {
    return ka > kb || (ka == kb && ia < ib);
}

// bitonic sort of n (power of two) candidates in LDS by the whole workgroup
// subset `lanes` (threads t < lanes participate; all threads hit the barriers)
__device__ __forceinline__ void cand_sort(uint64_t* key, int32_t* id, int n, int t, int lanes) {
    for (int sz = 2; sz <= n; sz <<= 1) {
        for (int st = sz >> 1; st > 0; st >>= 1) {
            for (int x = t; x < n && t < lanes; x += lanes) {
                const int y = x ^ st;
                if (y > x) {
                    const bool desc = (x & sz) == 0;
                    const uint64_t kx = key[x], ky = key[y];
                    const int32_t ix = id[x], iy = id[y];
                    const bool xfirst = cand_before(kx, ix, ky, iy);
                    if (desc ? !xfirst : xfirst) {
                        key[x] = ky; key[y] = kx;
                        id[x] = iy; id[y] = ix;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// is `it` in the sorted id range items[lo, hi)?
__device__ __forceinline__ bool in_sorted(const int32_t* items, int64_t lo, int64_t hi, int32_t it) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int32_t v = items[mid];
        if (v == it) return true;
        if (v < it) lo = mid + 1;
        else hi = mid;
    }
    return false;
}
// first position in the sorted items[lo, hi) whose id is >= it
__device__ __forceinline__ int64_t lower_pos(const int32_t* items, int64_t lo, int64_t hi,
                                             int32_t it) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (items[mid] < it) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ bool excluded(const int64_t* ptr, const int32_t* items, int qy,
                                         int32_t it) {
    if (!ptr) return false;
    int64_t lo = ptr[qy], hi = ptr[qy + 1];          // sorted ascending
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int32_t v = items[mid];
        if (v == it) return true;
        if (v < it) lo = mid + 1;
        else hi = mid;
    }
    return false;
}

template <typename T>
struct FusedArgs {
    const int32_t* users; int32_t nq;
    const T* P; const T* Q; const T* Bu; const T* Bi;
    int32_t n_items, k, amount, a2, n_splits;
    Hyper<T> h;
    const int64_t* ex_ptr; const int32_t* ex_items;
    uint64_t* part_key; int32_t* part_id;           // [nq][n_splits][amount]
};

template <typename T, int GS, int V, int KERN>
__global__ __launch_bounds__(kBlock) void k_topk_fused(FusedArgs<T> A) {
    static_assert(GS == kWave || V == 1, "the scalar layout: one item per wave");
    __shared__ uint64_t s_key[kFusedUsers][kFusedCap];
    __shared__ int32_t s_id[kFusedUsers][kFusedCap];
    __shared__ int s_cnt[kFusedUsers];
    __shared__ uint64_t s_tk[kFusedUsers];
    __shared__ int32_t s_ti[kFusedUsers];
    constexpr int R = kWave / GS;                    // items per wave instruction
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    const int g = lane / GS, l = lane % GS;
    const int split = blockIdx.x, q0 = blockIdx.y * kFusedUsers;
    const int k = A.k;
    const int64_t span = ((int64_t)A.n_items + A.n_splits - 1) / A.n_splits;
    const int ibeg = (int)min((int64_t)A.n_items, span * split);
    const int iend = (int)min((int64_t)A.n_items, span * (split + 1));
    if (tid < kFusedUsers) {
        s_cnt[tid] = 0;
        s_tk[tid] = 0ull;                            // below every candidate key (>= 1)
        s_ti[tid] = 0x7fffffff;
    }
    T p[kFusedUsers][V], bu[kFusedUsers];
#pragma unroll
    for (int x = 0; x < kFusedUsers; ++x) {
        const int qy = q0 + x;
        const int32_t uu = qy < A.nq ? A.users[qy] : -1;
        const bool uk = uu >= 0;
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int f = l + v * GS;
            p[x][v] = (uk && f < k) ? A.P[(int64_t)uu * k + f] : (T)0;
        }
        bu[x] = (uk && KERN != MF_RBF) ? A.Bu[uu] : (T)0;
    }
    __syncthreads();
    for (int c0 = ibeg; c0 < iend; c0 += kFusedChunk) {
        // thresholds of this chunk (wave-uniform copies)
        uint64_t tk[kFusedUsers];
        int32_t ti[kFusedUsers];
#pragma unroll
        for (int x = 0; x < kFusedUsers; ++x) { tk[x] = s_tk[x]; ti[x] = s_ti[x]; }
        for (int j = 0; j < kFusedItemsPerWave; j += R) {
            const int it = c0 + wv * kFusedItemsPerWave + j + g;
            const bool have = it < iend;
            const T* qr = A.Q + (int64_t)(have ? it : 0) * k;
            T q[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int f = l + v * GS;
                q[v] = (have && f < k) ? qr[f] : (T)0;
            }
            const T bi = (have && KERN != MF_RBF) ? A.Bi[it] : (T)0;
#pragma unroll
            for (int x = 0; x < kFusedUsers; ++x) {
                T sc = (T)0;
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    if constexpr (KERN == MF_RBF) {
                        const T d = p[x][v] - q[v];
                        sc = sc + d * d;
                    } else {
                        sc = sc + p[x][v] * q[v];
                    }
                }
                sc = group_sum<GS>(sc);
                T pred;                                  // predict_one (mf_rows.hpp)
                if constexpr (KERN == MF_LINEAR) pred = ((A.h.mu + bi) + bu[x]) + sc;
                else if constexpr (KERN == MF_SIGMOID)
                    pred = A.h.a + A.h.c * ((T)1 / ((T)1 + dexp<T>(-(((A.h.mu + bu[x]) + bi) + sc))));
                else pred = A.h.a + A.h.c * dexp<T>((-A.h.gamma) * sc);
                const uint64_t key = order_key((double)pred);
                const int qy = q0 + x;
                if (have && l == 0 && qy < A.nq && cand_before(key, it, tk[x], ti[x]) &&
                    !excluded(A.ex_ptr, A.ex_items, qy, it)) {
                    const int slot = atomicAdd(&s_cnt[x], 1);
                    s_key[x][slot] = key;
                    s_id[x][slot] = it;
                }
            }
        }
        __syncthreads();
        // cut lists that can no longer take a full chunk
#pragma unroll 1
        for (int x = 0; x < kFusedUsers; ++x) {
            const int n = s_cnt[x];
            if (n <= A.a2 + kFusedChunk) continue;       // uniform: s_cnt read after the barrier
            int n2 = 1;
            while (n2 < n) n2 <<= 1;
            for (int y = n + tid; y < n2; y += kBlock) { s_key[x][y] = 0ull; s_id[x][y] = 0x7fffffff; }
            __syncthreads();
            cand_sort(s_key[x], s_id[x], n2, tid, kBlock);
            if (tid == 0) {
                s_cnt[x] = A.a2;
                s_tk[x] = s_key[x][A.amount - 1];        // the amount-th best so far
                s_ti[x] = s_id[x][A.amount - 1];
            }
            __syncthreads();
        }
    }
    // final: sort each list, write its best `amount` (padding: key 0, id -1)
#pragma unroll 1
    for (int x = 0; x < kFusedUsers; ++x) {
        const int qy = q0 + x;
        if (qy >= A.nq) break;                           // uniform
        const int n = s_cnt[x];
        int n2 = 1;
        while (n2 < max(n, A.a2)) n2 <<= 1;
        for (int y = n + tid; y < n2; y += kBlock) { s_key[x][y] = 0ull; s_id[x][y] = 0x7fffffff; }
        __syncthreads();
        cand_sort(s_key[x], s_id[x], n2, tid, kBlock);
        for (int y = tid; y < A.amount; y += kBlock) {
            const int64_t o = ((int64_t)qy * A.n_splits + split) * A.amount + y;
            const bool ok = y < n;
            A.part_key[o] = ok ? s_key[x][y] : 0ull;
            A.part_id[o] = ok ? s_id[x][y] : -1;
        }
        __syncthreads();
    }
}

// merge the n_splits partial lists of one user (a workgroup per user)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_topk_merge(const uint64_t* __restrict__ part_key,
                                                       const int32_t* __restrict__ part_id,
                                                       int32_t n_splits, int32_t amount,
                                                       int32_t* out_items, T* out_scores) {
    __shared__ uint64_t s_key[kFusedCap * 4];
    __shared__ int32_t s_id[kFusedCap * 4];
    const int qy = blockIdx.x, tid = threadIdx.x;
    const int n = n_splits * amount;                     // <= 4 * kFusedCap (launcher)
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int y = tid; y < n2; y += kBlock) {
        const bool ok = y < n;
        const int64_t o = (int64_t)qy * n + y;
        const int32_t id = ok ? part_id[o] : -1;
        s_key[y] = (ok && id >= 0) ? part_key[o] : 0ull;
        s_id[y] = (ok && id >= 0) ? id : 0x7fffffff;
    }
    __syncthreads();
    cand_sort(s_key, s_id, n2, tid, kBlock);
    for (int y = tid; y < amount; y += kBlock) {
        const bool ok = s_key[y] != 0ull;
        out_items[(int64_t)qy * amount + y] = ok ? s_id[y] : -1;
        out_scores[(int64_t)qy * amount + y] =
            ok ? (T)key_score(s_key[y]) : (T)__longlong_as_double(0x7ff8000000000000LL);
    }
}

// splits of the item range for the fused path: enough workgroups to fill the
// chip (~6 per CU), at least 512 items per split, n_splits * amount <= 1024
inline int topk_splits(int32_t nq, int32_t n_items, int32_t amount) {
    const int64_t blocks_q = ((int64_t)nq + kFusedUsers - 1) / kFusedUsers;
    int64_t s = (1536 + blocks_q - 1) / blocks_q;
    s = std::min<int64_t>(s, std::max<int64_t>(1, n_items / 512));
    s = std::min<int64_t>(s, 1024 / std::max(amount, 1));
    return (int)std::max<int64_t>(1, s);
}
inline bool topk_fused(int32_t amount) {
    const char* e = std::getenv("MF_TOPK_TWO_STAGE");
    return amount <= kFusedMaxAmount && !(e && std::atoi(e) == 1);
}

// ---------------------------------------------------------------- MFMA filter
// k_topk_mm (linear kernel, FP32, n_factors a multiple of 4 up to 64): the
// same top-k as k_topk_fused, with the scores of a 64-user x 32-item tile
// computed on MFMA (v_mfma_f32_32x32x2_f32, the K dimension split so that
// lane half h walks columns [h SEG, h SEG + SEG) of the rows it holds).
// Those scores are NOT k_read's bits (another summation order), so they
// only FILTER: a candidate enters the user's LDS list if its approximate
// score s' is at least tau - 2M, tau the amount-th best s' so far and M a
// bound on |s' - s| for this user:
//   |dot_mfma - dot_tree| <= (k + 8) 2^-24 ||p|| max ||q||   (both orders,
//   fma chain and tree of rounded products, within gamma_k sum |p_i q_i|),
//   + the rounding of the three bias additions,
// doubled for safety.  Every item whose exact score could reach the exact
// top `amount` stays in the list; k_topk_mm_merge rescores the survivors
// with k_read's arithmetic (scalar layout, group_sum<GS>) and ranks them by
// (exact score desc, item id asc).  A list whose band outgrows its capacity
// sets *overflow: the results are then not guaranteed and the caller runs
// the exact path (mf_topk).
constexpr int kMmCap = 256;              // list capacity per user and workgroup
constexpr int kMmChunk = kWavesPerBlock * 32;   // items scored between barriers
constexpr int kMmMaxK = 64;
constexpr int kMmMaxSplits = 8;          // item splits (k_topk_mm_merge merges <= 8 bands)

struct MmArgs {
    const int32_t* users; int32_t nq;
    const float* P; const float* Q; const float* Bu; const float* Bi;
    int32_t n_items, k, amount, n_splits;
    float mu;
    const float* stats;                  // [2]: max ||q_i||, max |b_i| (k_topk_mm_stats)
    const int64_t* ex_ptr; const int32_t* ex_items;
    float* part_s; int32_t* part_id;     // [nq][n_splits][kMmCap]
    int32_t* part_n;                     // [nq][n_splits]
    float* marg;                         // [nq]: M per user
    int32_t* overflow;
    int32_t defer;                       // light users skip the exclusion search until the end
    int32_t fill;                        // k_topk_mw: compact a list past this many entries
    const int32_t* probe;                // k_topk_mw: probe items (k_topk_probe), n_probe of them
    int32_t n_probe, probe_group;        // ... one per group of probe_group consecutive ids
    const bf16x8* Qs;                    // k_topk_mw<.., BF>: Q split into bf16 hi + lo (k_topk_split_q)
    int32_t* big;                        // users left to k_topk_mm_merge by k_topk_mm_merge_wave
    int32_t* n_big;                      // ... their count (null big: k_topk_mm_merge takes all)
};

// k_topk_mm_stats: max item-row norm and max |b_i| into stats[0..1], max
// query-user row norm into stats[2].  Each wave reads 64-row chunks; where
// k / 4 is a power of two (k = 4 .. 64) a row is read by L = k / 4 lanes,
// one float4 each, so a wave load covers 64 / L whole rows, all L loads of
// a chunk in flight before the group sums (round 6: one row per lane made
// each load touch 64 lines, and with one atomic per wave on one word the
// kernel took 57 us of the C3 top-k's 1.07 ms).  The norms only bound the
// MFMA filter's error (with a 1e-4 safety factor): any summation order.
__device__ __forceinline__ float row_norm_any(const float* row, int k) {
    float s2 = 0.f;
    for (int f = 0; f < k; ++f) s2 = __builtin_fmaf(row[f], row[f], s2);
    return sqrtf(s2);
}

// the largest row norm of rows[0 .. 64) of a wave's chunk (row r < 0:
// none), L = k / 4 lanes per row: all L loads issued before any sum
template <int L>
__device__ __forceinline__ float chunk_max_norm(const float* base, int k, const int64_t* rowv,
                                                int lane) {
    float4 v[L];
    bool ok[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
        const int64_t row = rowv[j];
        ok[j] = row >= 0;
        v[j] = *reinterpret_cast<const float4*>(base + (ok[j] ? row : 0) * k + 4 * (lane % L));
    }
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < L; ++j) {
        float s2 = v[j].x * v[j].x;
        s2 = __builtin_fmaf(v[j].y, v[j].y, s2);
        s2 = __builtin_fmaf(v[j].z, v[j].z, s2);
        s2 = __builtin_fmaf(v[j].w, v[j].w, s2);
#pragma unroll
        for (int o = 1; o < L; o <<= 1) s2 += __shfl_xor(s2, o, kWave);
        if (ok[j]) m = fmaxf(m, sqrtf(s2));
    }
    return m;
}

template <int L>
__device__ __forceinline__ float chunk_norms(const float* base, int k, int64_t w0, int64_t n,
                                             const int32_t* users, int lane) {
    constexpr int per = kWave / L;
    // users: one id per lane, handed to the lanes that read its row
    const int32_t uid = users && w0 + lane < n ? users[w0 + lane] : -1;
    int64_t rowv[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
        const int r = per * j + lane / L;
        if (users) {
            rowv[j] = __shfl(uid, r, kWave);
        } else {
            rowv[j] = w0 + r < n ? w0 + r : -1;
        }
    }
    return chunk_max_norm<L>(base, k, rowv, lane);
}

// blocks [0, nb_items): item rows, the rest: query users; every wave strides
// over 64-row chunks, one atomic per block and statistic (round 6: one per
// wave on a single word was ~35 of the kernel's 57 us)
__global__ __launch_bounds__(kBlock) void k_topk_mm_stats(const float* __restrict__ Q,
                                                          const float* __restrict__ Bi,
                                                          int32_t n_items, int32_t k,
                                                          float* stats,
                                                          const int32_t* __restrict__ users,
                                                          int32_t nq_users,
                                                          const float* __restrict__ P,
                                                          int32_t nb_items) {
    __shared__ float s_red[2][kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const bool user_part = (int)blockIdx.x >= nb_items;
    const int b = user_part ? (int)blockIdx.x - nb_items : (int)blockIdx.x;
    const int nb = user_part ? (int)gridDim.x - nb_items : nb_items;
    const int64_t n = user_part ? nq_users : n_items;
    const float* base = user_part ? P : Q;
    const int32_t* ids = user_part ? users : nullptr;
    float m0 = 0.f, m1 = 0.f;                      // max norm, max |b_i|
    for (int64_t w0 = ((int64_t)b * kWavesPerBlock + wv) * kWave; w0 < n;
         w0 += (int64_t)nb * kWavesPerBlock * kWave) {
        float m;
        switch (k) {
            case 64: m = chunk_norms<16>(base, k, w0, n, ids, lane); break;
            case 32: m = chunk_norms<8>(base, k, w0, n, ids, lane); break;
            case 16: m = chunk_norms<4>(base, k, w0, n, ids, lane); break;
            case 8: m = chunk_norms<2>(base, k, w0, n, ids, lane); break;
            case 4: m = chunk_norms<1>(base, k, w0, n, ids, lane); break;
            default: {
                m = 0.f;
                const int64_t row = w0 + lane < n ? (ids ? ids[w0 + lane] : w0 + lane) : -1;
                if (row >= 0) m = row_norm_any(base + row * k, k);
            }
        }
        m0 = fmaxf(m0, m);
        if (!user_part && w0 + lane < n) m1 = fmaxf(m1, fabsf(Bi[w0 + lane]));
    }
    for (int o = 32; o > 0; o >>= 1) {
        m0 = fmaxf(m0, __shfl_xor(m0, o, kWave));
        m1 = fmaxf(m1, __shfl_xor(m1, o, kWave));
    }
    if (lane == 0) { s_red[0][wv] = m0; s_red[1][wv] = m1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int x = 1; x < kWavesPerBlock; ++x) {
            m0 = fmaxf(m0, s_red[0][x]);
            m1 = fmaxf(m1, s_red[1][x]);
        }
        // non-negative floats: integer max of the bits
        if (user_part) {
            atomicMax(reinterpret_cast<int*>(stats) + 2, __float_as_int(m0));
        } else {
            atomicMax(reinterpret_cast<int*>(stats), __float_as_int(m0 * 1.0001f));
            atomicMax(reinterpret_cast<int*>(stats) + 1, __float_as_int(m1));
        }
    }
}

// k_topk_probe: the probe items of k_topk_mw -- one per group of G consecutive
// item ids, the group's best by b_i + rho ||q_i|| (rho = half the largest
// query-user norm, stats[2]; ties to the lower id), one wave per group.  Any
// set of items gives a valid admission floor (k_topk_mw); this one is meant
// to hold items that rank high for many users, so that the floor is high.
// Ascending ids (group order), one item per group: excluded ones are found
// by id / G.
__global__ __launch_bounds__(kBlock) void k_topk_probe(const float* __restrict__ Q,
                                                       const float* __restrict__ Bi,
                                                       int32_t n_items, int32_t k, int32_t G,
                                                       int32_t n_probe,
                                                       const float* __restrict__ stats,
                                                       int32_t* __restrict__ probe) {
    const int lane = threadIdx.x & (kWave - 1);
    const int g = blockIdx.x * kWavesPerBlock + (int)threadIdx.x / kWave;
    if (g >= n_probe) return;                            // wave-uniform
    const float rho = 0.5f * stats[2];
    const int64_t lo = (int64_t)g * G, hi = min((int64_t)n_items, lo + G);   // lo < n_items (caller)
    float best = -INFINITY;
    int32_t bid = 0x7fffffff;
    for (int64_t it = lo + lane; it < hi; it += kWave) {
        const float* q = Q + it * k;
        float nn = 0.f;
        for (int f = 0; f < k; f += 4) {
            const float4 v = *reinterpret_cast<const float4*>(q + f);
            nn = __builtin_fmaf(v.x, v.x, nn); nn = __builtin_fmaf(v.y, v.y, nn);
            nn = __builtin_fmaf(v.z, v.z, nn); nn = __builtin_fmaf(v.w, v.w, nn);
        }
        const float key = Bi[it] + rho * sqrtf(nn);
        if (key > best) { best = key; bid = (int32_t)it; }   // ascending: first of equals
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, kWave);
        const int32_t oi = __shfl_xor(bid, o, kWave);
        if (ob > best || (ob == best && oi < bid)) { best = ob; bid = oi; }
    }
    if (lane == 0) probe[g] = bid == 0x7fffffff ? (int32_t)lo : bid;   // (NaN keys: the first)
}

// k_topk_split_q: the item rows as k_topk_mw<.., BF> loads them, in tiles of
// 32 items in the MFMA operand layout.  Element j of lane (c, h)'s fragment
// for column group g is column h seg + 8 g + j (zero past seg or k) of the
// tile's item c, split x = hi + lo + e (hi = bf16(x), lo = bf16(x - hi));
// tile T, group g, part t (0 hi, 1 lo) holds 64 lane-ordered 16-B chunks
// (lane = 32 h + c), so one load instruction of a wave reads 1 KB of whole
// cache lines.  Tiles 0 .. n_tiles-1 are items 32 T + c (zero past n_items),
// the n_ptiles after them the probe items probe[32 T' + c] (zero past
// n_probe).  One thread per (tile, group, lane).
__global__ __launch_bounds__(kBlock) void k_topk_split_q(const float* __restrict__ Q,
                                                         int32_t n_items, int32_t k, int32_t seg,
                                                         int32_t nb, int32_t n_tiles,
                                                         const int32_t* __restrict__ probe,
                                                         int32_t n_probe, int32_t n_ptiles,
                                                         bf16x8* __restrict__ Qs) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (int64_t)(n_tiles + n_ptiles) * nb * 64) return;
    const int64_t T = t / (nb * 64);
    const int rem = (int)(t - T * nb * 64), g = rem / 64, lane = rem % 64;
    const int c = lane & 31, h = lane >> 5;
    int64_t it;
    if (T < n_tiles) {
        it = T * 32 + c;
        if (it >= n_items) it = -1;
    } else {
        const int64_t sl = (T - n_tiles) * 32 + c;
        it = sl < n_probe ? probe[sl] : -1;
    }
    bf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int ci = 8 * g + j, col = h * seg + ci;
        const float x = it >= 0 && ci < seg && col < k ? Q[it * k + col] : 0.f;
        const __bf16 xh = (__bf16)x;
        hi[j] = xh;
        lo[j] = (__bf16)(x - (float)xh);
    }
    bf16x8* o = Qs + ((T * nb + g) * 2) * 64 + lane;
    o[0] = hi;
    o[64] = lo;
}

// (score desc, id asc) bitonic sort of n (power of two) float-keyed entries
__device__ __forceinline__ void mm_sort(float* sc, int32_t* id, int n, int t) {
    for (int sz = 2; sz <= n; sz <<= 1) {
        for (int st = sz >> 1; st > 0; st >>= 1) {
            for (int x = t; x < n; x += kBlock) {
                const int y = x ^ st;
                if (y > x) {
                    const bool desc = (x & sz) == 0;
                    const float kx = sc[x], ky = sc[y];
                    const int32_t ix = id[x], iy = id[y];
                    const bool xfirst = kx > ky || (kx == ky && ix < iy);
                    if (desc ? !xfirst : xfirst) {
                        sc[x] = ky; sc[y] = kx;
                        id[x] = iy; id[y] = ix;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// One wave sorts an N-entry list (N a power of two, 64 <= N <= 256) in LDS
// by (score desc, id asc): bitonic, N / 128 compare-exchange pairs per lane
// and stage (N = 64: lanes 0..31), no workgroup barrier (LDS operations of
// one wave complete in order; the empty asm keeps the compiler from moving a
// lane's accesses across stages, i.e. from forwarding its own stores where
// another lane wrote).
template <int N = kMmCap>
__device__ __forceinline__ void wave_sort(float* sc, int32_t* id, int lane) {
    static_assert(N >= 64 && N <= 256 && (N & (N - 1)) == 0, "64..256, a power of two");
    constexpr int E = N >= 128 ? N / 128 : 1;
    for (int sz = 2; sz <= N; sz <<= 1) {
        for (int st = sz >> 1; st > 0; st >>= 1) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int pi = lane + 64 * e;                 // pair index 0..N/2-1
                if (N >= 128 || pi < N / 2) {
                    const int x = (pi / st) * 2 * st + (pi % st), y = x + st;
                    const bool desc = (x & sz) == 0;
                    const float kx = sc[x], ky = sc[y];
                    const int32_t ix = id[x], iy = id[y];
                    const bool xfirst = kx > ky || (kx == ky && ix < iy);
                    if (desc ? !xfirst : xfirst) {
                        sc[x] = ky; sc[y] = kx;
                        id[x] = iy; id[y] = ix;
                    }
                }
            }
            asm volatile("" ::: "memory");
        }
    }
}

// One wave compacts a user's list: sorted, cut to the band s' >= tau - 2M.
// check: excluded entries are dropped first (binary search in the user's
// sorted exclusion ids that fall in this split's item range, [elo, ehi)),
// and tau is the amount-th best; otherwise (a light user during the sweep:
// at most `extra` excluded ids in the range) tau is the (amount + extra)-th
// best, of which at least `amount` are not excluded.  Returns the band
// size; *adm receives the admission bound.
template <int CAP = kMmCap>
__device__ __forceinline__ int wave_compact(const MmArgs& A, float* sc, int32_t* id, int n,
                                            bool check, int64_t elo, int64_t ehi, int extra,
                                            float mg, int lane, float* adm) {
    if constexpr (CAP == kWave) {
        // one entry per lane: the excluded ids of the range come in 64 at a
        // time (one parallel load instead of a chain of dependent binary-
        // search loads per entry) and every lane compares its id with each
        float v = -INFINITY;
        int32_t it = 0x7fffffff;
        if (lane < n) { v = sc[lane]; it = id[lane]; }
        bool ex = false;
        if (check) {
            for (int64_t b0 = elo; b0 < ehi; b0 += kWave) {          // wave-uniform
                const int64_t j = b0 + lane;
                const int32_t e = j < ehi ? A.ex_items[j] : -1;
                const int ne = (int)min((int64_t)kWave, ehi - b0);
                for (int x = 0; x < ne; ++x) ex |= __builtin_amdgcn_readlane(e, x) == it;
            }
        }
        sc[lane] = ex ? -INFINITY : v;
        id[lane] = ex ? 0x7fffffff : it;
    } else {
        for (int y = lane; y < CAP; y += kWave) {
            float v = -INFINITY;
            int32_t it = 0x7fffffff;
            if (y < n) {
                v = sc[y];
                it = id[y];
                if (check && in_sorted(A.ex_items, elo, ehi, it)) { v = -INFINITY; it = 0x7fffffff; }
            }
            sc[y] = v;
            id[y] = it;
        }
    }
    asm volatile("" ::: "memory");
    wave_sort<CAP>(sc, id, lane);
    const int rank = A.amount + (check ? 0 : extra);     // <= CAP (caller)
    int valid = 0, keep = 0;
    float bound = -INFINITY;
#pragma unroll
    for (int e = 0; e < CAP / kWave; ++e)
        valid += __popcll(__ballot(sc[lane + 64 * e] != -INFINITY));
    if (valid >= rank) bound = sc[rank - 1] - 2.f * mg;
#pragma unroll
    for (int e = 0; e < CAP / kWave; ++e)
        keep += __popcll(__ballot(sc[lane + 64 * e] != -INFINITY && sc[lane + 64 * e] >= bound));
    *adm = bound;
    return keep;
}

// PIPE: the MFMAs of chunk c+1 are issued before chunk c's admission
// epilogue (two accumulator pairs), interleaved with it by sched_group_barrier,
// so the epilogue's VALU work runs in the matrix pipe's shadow.
template <int SEG, bool PIPE = false, int NT = 2>
__global__ __launch_bounds__(kBlock) void k_topk_mm(MmArgs A) {
    constexpr int kU = 32 * NT;          // users per workgroup: NT 32-row MFMA tiles
    using f32x16 = __attribute__((ext_vector_type(16))) float;
    __shared__ float s_sc[kU][kMmCap];
    __shared__ int32_t s_id[kU][kMmCap];
    __shared__ int s_cnt[kU];
    __shared__ float s_adm[kU];    // admission bound tau - 2M (-inf until a full list)
    __shared__ float s_bu[kU];
    __shared__ float s_m[kU];
    __shared__ int64_t s_elo[kU], s_ehi[kU];   // exclusion ids in [ibeg, iend)
    __shared__ int s_need, s_lost;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    const int c = lane & 31, h = lane >> 5;
    const int split = blockIdx.x, q0 = blockIdx.y * kU;
    const int k = A.k;
    const int64_t span = ((int64_t)A.n_items + A.n_splits - 1) / A.n_splits;
    const int ibeg = (int)min((int64_t)A.n_items, span * split);
    const int iend = (int)min((int64_t)A.n_items, span * (split + 1));
    const float qmax = A.stats[0], bimax = A.stats[1];
    const float ck = 2.f * (float)(k + 8) * 0x1p-24f;
    if (tid < kU) {
        const int qy = q0 + tid;
        const int32_t uu = qy < A.nq ? A.users[qy] : -1;
        float pn = 0.f;
        if (uu >= 0)
            for (int f = 0; f < k; ++f) pn = __builtin_fmaf(A.P[(int64_t)uu * k + f],
                                                            A.P[(int64_t)uu * k + f], pn);
        pn = sqrtf(pn) * 1.0001f;
        const float bu = uu >= 0 ? A.Bu[uu] : 0.f;
        // dot-order bound + the bias additions' rounding (scores bounded by
        // |mu| + |b_u| + max|b_i| + ||p|| max||q||), doubled
        const float mg = ck * pn * qmax +
                         0x1p-21f * (fabsf(A.mu) + fabsf(bu) + bimax + pn * qmax);
        s_cnt[tid] = 0;
        s_adm[tid] = -INFINITY;
        s_bu[tid] = bu;
        s_m[tid] = mg;
        if (split == 0 && qy < A.nq) A.marg[qy] = mg;
        int64_t lo = 0, hi = 0;
        if (A.ex_ptr && qy < A.nq) {
            lo = lower_pos(A.ex_items, A.ex_ptr[qy], A.ex_ptr[qy + 1], ibeg);
            hi = lower_pos(A.ex_items, lo, A.ex_ptr[qy + 1], iend);
        }
        s_elo[tid] = lo;
        s_ehi[tid] = hi;
    }
    if (tid == 0) { s_need = 0; s_lost = 0; }
    // A operands: lane (c, h) holds user 32 t + c, columns h SEG .. h SEG + SEG-1
    float a[NT][SEG];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int qy = q0 + 32 * t + c;
        const int32_t uu = qy < A.nq ? A.users[qy] : -1;
        const float* pr = A.P + (int64_t)(uu >= 0 ? uu : 0) * k;
#pragma unroll
        for (int j = 0; j < SEG; j += 4) {
            const int c0 = h * SEG + j;
            const float4 v = *reinterpret_cast<const float4*>(pr + (c0 < k ? c0 : 0));
            const bool ok = uu >= 0 && c0 < k;
            a[t][j + 0] = ok ? v.x : 0.f; a[t][j + 1] = ok ? v.y : 0.f;
            a[t][j + 2] = ok ? v.z : 0.f; a[t][j + 3] = ok ? v.w : 0.f;
        }
    }
    __syncthreads();
    // per-lane copies of the 32 users' b_u and admission bounds (rows of the
    // accumulators: users 32 t + ra(i, h)); the bounds change only at a
    // compaction, after which they are re-read
    float ubu[NT][16], uadm[NT][16];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int m = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
            ubu[t][i] = s_bu[m];
            uadm[t][i] = q0 + m < A.nq ? -INFINITY : INFINITY;   // no query: never admit
        }
    // B operands: raw loads, never consumed here (a select on the loaded
    // values would make the compiler wait for the prefetch right away):
    // items past the range read a valid row and are never admitted, columns
    // past k meet zero A operands
    auto load_b = [&](int it0, float (&b)[SEG], float& bi) __attribute__((always_inline)) {
        const int n = it0 + c;
        const int nn = n < iend ? n : (ibeg < iend ? ibeg : 0);   // empty split: row 0
        const float* qr = A.Q + (int64_t)nn * k;
        bi = A.Bi[nn];                   // first: waiting for it waits for nothing else
#pragma unroll
        for (int j = 0; j < SEG; j += 4) {
            const int c0 = h * SEG + j;
            const float4 v = *reinterpret_cast<const float4*>(qr + (c0 < k ? c0 : 0));
            b[j + 0] = v.x; b[j + 1] = v.y; b[j + 2] = v.z; b[j + 3] = v.w;
        }
    };
    float b[SEG], bi;
    load_b(ibeg + wv * 32, b, bi);
    auto tile = [&](f32x16 (&x)[NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) x[t][i] = 0.f;
#pragma unroll
        for (int s = 0; s < SEG; ++s)
#pragma unroll
            for (int t = 0; t < NT; ++t)
                x[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t][s], b[s], x[t], 0, 0, 0);
    };
    // One chunk: MFMA scores of this wave's 32-item tile into acc[NT],
    // admission of them against the users' bounds.  PIPE: step(c0, X, Y)
    // runs the admission of chunk c (accumulators X, bias bX) while the
    // MFMAs of chunk c+1 go into Y -- unconditionally (past the range they
    // score a clamped valid row that is never admitted), as are the loads of
    // chunk c+2, so MFMAs, loads and compares share one basic block that the
    // sched_group_barriers interleave.
    auto admit = [&](int c0, const f32x16 (&acc)[NT], float bic)
                     __attribute__((always_inline)) -> uint64_t {
        const int it0 = c0 + wv * 32;
        const bool have = it0 + c < iend;
        // epilogue: admission only (exclusions are checked when a list is
        // compacted or written: the rare admitted candidates, in parallel).
        // The compares go into one wave-wide mask first; the per-score
        // branches run only when some lane admits something.
        uint64_t any = 0;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float sp = ((A.mu + bic) + ubu[t][i]) + acc[t][i];
                any |= __builtin_amdgcn_ballot_w64(have && sp >= uadm[t][i]);
            }
        return any;
    };
    auto insert = [&](int c0, const f32x16 (&acc)[NT], float bic)
                      __attribute__((always_inline)) {
        const int it0 = c0 + wv * 32;
        const bool have = it0 + c < iend;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int m = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
                const float sp = ((A.mu + bic) + ubu[t][i]) + acc[t][i];
                if (have && sp >= uadm[t][i]) {
                    const int slot = atomicAdd(&s_cnt[m], 1);
                    if (slot < kMmCap) {
                        s_sc[m][slot] = sp;
                        s_id[m][slot] = it0 + c;
                    } else {
                        s_lost = 1;
                    }
                    if (slot >= kMmCap - kMmChunk) s_need = 1;
                }
            }
        }
    };
    // after a chunk's admission: compact the lists that could not take
    // another chunk (uniform: read after the barrier)
    auto settle = [&]() __attribute__((always_inline)) {
        __syncthreads();
        if (s_need) {
            // each wave compacts users m = wv, wv + 4, ...
            for (int m = wv; m < kU; m += kWavesPerBlock) {
                const int n = min(s_cnt[m], kMmCap);
                if (n <= kMmCap - kMmChunk) continue;    // wave-uniform
                // light users (few excluded ids in this split) skip the
                // search until the end: tau ranks amount + extra entries
                const int extra = (int)(s_ehi[m] - s_elo[m]);
                const bool heavy = !A.defer || A.amount + extra > (kMmCap - kMmChunk) / 2;
                float adm;
                int keep = wave_compact(A, s_sc[m], s_id[m], n, heavy, s_elo[m], s_ehi[m], extra,
                                        s_m[m], lane, &adm);
                if (keep > kMmCap - kMmChunk) {          // the band does not fit
                    if (lane == 0) s_lost = 1;
                    keep = kMmCap - kMmChunk;
                }
                if (lane == 0) {
                    s_cnt[m] = keep;
                    s_adm[m] = adm;
                }
            }
            __syncthreads();
            if (tid == 0) s_need = 0;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int m = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
                    uadm[t][i] = q0 + m < A.nq ? s_adm[m] : INFINITY;
                }
            __syncthreads();
        }
    };
    if constexpr (PIPE) {
        f32x16 xa[NT], xb[NT];
        float ba, bb;
        tile(xa);                                        // chunk 0
        ba = bi;
        load_b(ibeg + kMmChunk + wv * 32, b, bi);        // chunk 1 (clamped past the range)
        auto step = [&](int c0, f32x16 (&x)[NT], float& bx, f32x16 (&y)[NT], float& by)
                        __attribute__((always_inline)) {
            tile(y);                                     // chunk c+1
            by = bi;
            load_b(c0 + 2 * kMmChunk + wv * 32, b, bi);  // chunk c+2
            const uint64_t any = admit(c0, x, bx);
            // one MFMA, then a share of the compares, ... (0x8 MFMA, 0x2 VALU,
            // 0x20 VMEM read): the admission runs while the matrix pipe works
#pragma unroll
            for (int s = 0; s < NT * SEG; ++s) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
            if (any) insert(c0, x, bx);
            settle();
        };
        for (int c0 = ibeg; c0 < iend; c0 += 2 * kMmChunk) {
            step(c0, xa, ba, xb, bb);
            if (c0 + kMmChunk < iend) step(c0 + kMmChunk, xb, bb, xa, ba);
        }
    }
    for (int c0 = ibeg; !PIPE && c0 < iend; c0 += kMmChunk) {
        f32x16 acc[NT];
        tile(acc);
        const float bic = bi;
        if (c0 + kMmChunk < iend) load_b(c0 + kMmChunk + wv * 32, b, bi);   // next tile in flight
        if (admit(c0, acc, bic)) insert(c0, acc, bic);
        settle();
    }
    // final: each wave compacts its users' lists and writes the bands
    for (int m = wv; m < kU; m += kWavesPerBlock) {
        const int qy = q0 + m;
        if (qy >= A.nq) break;                           // wave-uniform
        const int n = min(s_cnt[m], kMmCap);
        float adm;
        int keep = wave_compact(A, s_sc[m], s_id[m], n, true, s_elo[m], s_ehi[m], 0, s_m[m],
                                lane, &adm);
        const int64_t o = ((int64_t)qy * A.n_splits + split) * kMmCap;
        for (int y = lane; y < keep; y += kWave) {
            A.part_s[o + y] = s_sc[m][y];
            A.part_id[o + y] = s_id[m][y];
        }
        if (lane == 0) A.part_n[(int64_t)qy * A.n_splits + split] = keep;
    }
    __syncthreads();
    if (tid == 0 && s_lost) atomicOr(A.overflow, 1);
}

// k_topk_mw (round 3; amount <= kMwMaxAmount): k_topk_mm's filter with the
// users spread over the waves instead of the items.  Each of the four waves
// owns 32 users (one 32-row MFMA tile, A operands in registers) and a
// wave-private LDS list of kMwCap candidates per user; all four walk the
// same 32-item tiles of the split, so a tile's B operands come from L2 once
// per workgroup (128 users) and the other three waves find them in the CU's
// L1.  Nothing is shared between waves after the setup: no workgroup
// barrier per chunk.  The list bookkeeping lives in registers -- lane r < 32
// holds the count and the admission bound of user r of its wave -- so an
// admitted score is written at base + (its rank among the tile's admitted
// lanes of that user), no LDS atomics; a list that might not take another
// tile (count > kMwCap - 32) is compacted in registers (one entry per lane:
// exclusion check against the user's excluded ids of the split, loaded 64 at
// a time; the amount-th best by a rank count; the band kept in lane order).
// Admission rule, margin, exclusions and the (unsorted) bands written per
// (user, split) are k_topk_mm's; k_topk_mm_merge sorts and rescores.
constexpr int kMwCap = kWave;            // one entry per lane in a compaction
constexpr int kMwMaxAmount = 16;         // amount + band must fit kMwCap - 32 after a compaction
constexpr int kMwUsers = 32 * kWavesPerBlock;
constexpr int kMwExCap = 768;            // excluded ids of a wave's users in its split, cached in LDS
constexpr int kMwProbe = 512;            // probe items (k_topk_probe) at most
constexpr int kMwProbeWords = kMwProbe / 64;
static_assert(32 * kMwProbeWords * 8 <= kMwExCap * 4, "probe bits share the exclusion cache");

// v[l] = x (x and l wave-uniform), the other lanes keep v
__device__ __forceinline__ int writelane_i(int x, int l, int v) {
    return (int)(threadIdx.x & (kWave - 1)) == l ? x : v;
}
__device__ __forceinline__ float readlane_f(float v, int j) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
}
__device__ __forceinline__ float writelane_f(float x, int l, float v) {
    return __builtin_bit_cast(float, writelane_i(__builtin_bit_cast(int, x), l,
                                                 __builtin_bit_cast(int, v)));
}

// the r-th largest (r >= 1, with multiplicity) of v over the lanes with m
// set (at least r of them): a binary search on order-preserving keys, 32
// ballots (round 6; was a rank count of every entry against every other,
// one readlane pair per entry)
__device__ __forceinline__ float wave_rth_largest(float v, bool m, int r) {
    const uint32_t b = __float_as_uint(v);
    const uint32_t key = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    uint32_t t = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t c = t | (1u << bit);
        if (__popcll(__builtin_amdgcn_ballot_w64(m && key >= c)) >= r) t = c;
    }
    const uint64_t at = __builtin_amdgcn_ballot_w64(m && key == t);
    return readlane_f(v, (int)__builtin_ctzll(at));
}

template <int SEG, bool PIPE = true, bool BF = false>
__global__ __launch_bounds__(kBlock) void k_topk_mw(MmArgs A) {
    constexpr int CAP = kMwCap;
    constexpr int NB = (SEG + 7) / 8;                    // BF: bf16 MFMAs per term and tile
    using f32x16 = __attribute__((ext_vector_type(16))) float;
    __shared__ float s_sc[kMwUsers][CAP];
    __shared__ int32_t s_id[kMwUsers][CAP];
    __shared__ float s_m[kMwUsers];
    __shared__ int64_t s_elo[kMwUsers], s_ehi[kMwUsers];
    // per wave: its users' excluded ids of the split, packed (after the probe
    // walk); during it, the users' probe-exclusion bits
    __shared__ __align__(16) int32_t s_un[kWavesPerBlock * kMwExCap];
    __shared__ int s_exoff[kMwUsers];                      // offset in the wave's cache, -1: not cached
    __shared__ int s_lost;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    const int c = lane & 31, h = lane >> 5;
    int32_t* const s_exw = s_un + wv * kMwExCap;
    uint64_t* const s_pexw = reinterpret_cast<uint64_t*>(s_exw);
    const int split = blockIdx.x;
    const int m0 = 32 * wv;                              // this wave's users: m0 .. m0 + 31
    const int q0 = blockIdx.y * kMwUsers + m0;
    const int k = A.k;
    // splits start on 32-item tiles (the BF operand tiles, k_topk_split_q)
    const int64_t span = (((int64_t)A.n_items + A.n_splits - 1) / A.n_splits + 31) & ~(int64_t)31;
    const int ibeg = (int)min((int64_t)A.n_items, span * split);
    const int iend = (int)min((int64_t)A.n_items, span * (split + 1));
    const float qmax = A.stats[0], bimax = A.stats[1];
    // |s' - s| <= ck ||p|| max ||q|| (+ the bias additions, below), doubled:
    // f32 MFMA: both orders within gamma_(k+8) sum |p_i q_i|.  BF (3-term
    // bf16 split, p = ph + pl + ep with |ep| <= 2^-14 |p| even for truncating
    // conversions): the dropped terms ph eq + pl ql + ep q within 3 2^-14
    // sum |p_i q_i|, the MFMA's sums of 3k exact products and k_read's tree
    // within (4k + 8) 2^-23 (faithful rounding, either direction)
    const float ck = BF ? 2.02f * (3.f * 0x1p-14f + (float)(4 * k + 8) * 0x1p-23f)
                        : 2.f * (float)(k + 8) * 0x1p-24f;
    if (tid == 0) s_lost = 0;
    float bu_own = 0.f;
    int ex_n = 0;                                        // lane r < 32: excluded ids of user r in the split
    // lane r < 32: count and admission bound of user m0 + r (no query: never admits)
    int lcnt = 0;
    float ladm = q0 + c < A.nq ? -INFINITY : INFINITY;
    float lfloor = -INFINITY;                            // lane r < 32: user r's floor (probe walk)
    bool probing = false;
    if (lane < 32) {
        const int qy = q0 + lane;
        const int32_t uu = qy < A.nq ? A.users[qy] : -1;
        float pn = 0.f;
        if (uu >= 0)
            for (int f = 0; f < k; ++f) pn = __builtin_fmaf(A.P[(int64_t)uu * k + f],
                                                            A.P[(int64_t)uu * k + f], pn);
        pn = sqrtf(pn) * 1.0001f;
        bu_own = uu >= 0 ? A.Bu[uu] : 0.f;
        const float mg = ck * pn * qmax +
                         0x1p-21f * (fabsf(A.mu) + fabsf(bu_own) + bimax + pn * qmax);
        s_m[m0 + lane] = mg;
        if (split == 0 && qy < A.nq) A.marg[qy] = mg;
        int64_t lo = 0, hi = 0;
        if (A.ex_ptr && qy < A.nq) {
            lo = lower_pos(A.ex_items, A.ex_ptr[qy], A.ex_ptr[qy + 1], ibeg);
            hi = lower_pos(A.ex_items, lo, A.ex_ptr[qy + 1], iend);
        }
        s_elo[m0 + lane] = lo;
        s_ehi[m0 + lane] = hi;
        ex_n = (int)(hi - lo);
    }
    // A operands: lane (c, h) holds user q0 + c, columns h SEG .. h SEG + SEG-1
    // (BF: as bf16 hi + lo, element j of MFMA s = column h SEG + 8 s + j)
    float a[SEG];
    bf16x8 ah[NB], al[NB];
    {
        const int qy = q0 + c;
        const int32_t uu = qy < A.nq ? A.users[qy] : -1;
        const float* pr = A.P + (int64_t)(uu >= 0 ? uu : 0) * k;
#pragma unroll
        for (int j = 0; j < SEG; j += 4) {
            const int c0 = h * SEG + j;
            const float4 v = *reinterpret_cast<const float4*>(pr + (c0 < k ? c0 : 0));
            const bool ok = uu >= 0 && c0 < k;
            a[j + 0] = ok ? v.x : 0.f; a[j + 1] = ok ? v.y : 0.f;
            a[j + 2] = ok ? v.z : 0.f; a[j + 3] = ok ? v.w : 0.f;
        }
        if constexpr (BF) {
#pragma unroll
            for (int s2 = 0; s2 < NB; ++s2)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float x = 8 * s2 + j < SEG ? a[8 * s2 + j] : 0.f;
                    const __bf16 xh = (__bf16)x;
                    ah[s2][j] = xh;
                    al[s2][j] = (__bf16)(x - (float)xh);
                }
        }
    }
    // accumulator row i of lane (c, h) is user r(i, h) = (i & 3) + 8 (i >> 2) + 4 h
    float ubu[16], uadm[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = (i & 3) + 8 * (i >> 2) + 4 * h;
        ubu[i] = __shfl(bu_own, r, kWave);
        // probe (MF_TOPK_MM_DEFER=2, timing only: wrong results): admit nothing
        uadm[i] = q0 + r < A.nq && A.defer != 2 ? -INFINITY : INFINITY;
    }
    __syncthreads();                                     // the setup's LDS words
    float b[SEG], bi;
    bf16x8 bh[NB], bl[NB];
    // B operands (and b_i) of item nn: part 0 / 1 = those the first / second
    // half of a tile's MFMAs read (the MFMAs of rows 0..7 / 8..15 in the
    // pipelined loop), 2 = all
    const int n_tiles = (A.n_items + 31) >> 5;
    // BF: tile tb's operands (k_topk_split_q's layout: lane-ordered chunks)
    auto fetch_bf = [&](const bf16x8* tb, int part) __attribute__((always_inline)) {
        constexpr int HB = NB / 2;
#pragma unroll
        for (int s2 = part == 1 ? HB : 0; s2 < (part == 0 ? HB : NB); ++s2) {
            bh[s2] = tb[(2 * s2) * 64 + lane];
            bl[s2] = tb[(2 * s2 + 1) * 64 + lane];
        }
    };
    auto fetch = [&](int nn, int part) __attribute__((always_inline)) {
        if (part != 1) bi = A.Bi[nn];
        if constexpr (BF) {
            // tile of the walk position (it0 = 32 T, nn its lane's item or the
            // clamped one): the caller passes the tile through fetch_tile
        } else {
            const float* qr = A.Q + (int64_t)nn * k;
            constexpr int H4 = (SEG / 2) & ~3;
#pragma unroll
            for (int j = part == 1 ? H4 : 0; j < (part == 0 ? H4 : SEG); j += 4) {
                const int c0 = h * SEG + j;
                const float4 v = *reinterpret_cast<const float4*>(qr + (c0 < k ? c0 : 0));
                b[j + 0] = v.x; b[j + 1] = v.y; b[j + 2] = v.z; b[j + 3] = v.w;
            }
        }
    };
    auto item_of = [&](int it0) __attribute__((always_inline)) -> int {
        const int n = it0 + c;
        return n < iend ? n : (ibeg < iend ? ibeg : 0);  // empty split: row 0
    };
    // the walk's tile at it0 (a multiple of 32: splits start on tiles);
    // past the split's end: its first tile (never admitted, `have`)
    auto tile_ptr = [&](int it0) __attribute__((always_inline)) -> const bf16x8* {
        int T = (it0 < iend ? it0 : ibeg) >> 5;
        T = T < n_tiles ? T : n_tiles - 1;
        return A.Qs + (int64_t)T * NB * 2 * 64;
    };
    auto fetch_tile = [&](int it0, int part) __attribute__((always_inline)) {
        if (part != 1) bi = A.Bi[item_of(it0)];
        fetch_bf(tile_ptr(it0), part);
    };
    auto load_b = [&](int it0) __attribute__((always_inline)) {
        if constexpr (BF) fetch_tile(it0, 2);
        else fetch(item_of(it0), 2);
    };
    // the NM MFMAs of a tile; mfma_m issues the m-th (BF: for each 16 columns
    // lo x hi, hi x lo, hi x hi)
    constexpr int NM = BF ? 3 * NB : SEG;
    auto mfma_m = [&](f32x16& x, int m) __attribute__((always_inline)) {
        if constexpr (BF) {
            const int s2 = m / 3, t = m % 3;
            x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t == 0 ? al[s2] : ah[s2],
                                                        t == 1 ? bl[s2] : bh[s2], x, 0, 0, 0);
        } else {
            x = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m], b[m], x, 0, 0, 0);
        }
    };
    auto tile = [&](f32x16& x) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = 0.f;
#pragma unroll
        for (int m = 0; m < NM; ++m) mfma_m(x, m);
    };
    // the per-row admission ballots of a tile (row i: users r(i, 0) in the
    // low half, r(i, 1) in the high half), kept for insert
    auto admit = [&](int c0, const f32x16& acc, float bic, uint64_t (&bal)[16])
                     __attribute__((always_inline)) -> uint64_t {
        const bool have = c0 + c < iend;
        uint64_t any = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float sp = ((A.mu + bic) + ubu[i]) + acc[i];
            bal[i] = __builtin_amdgcn_ballot_w64(have && sp >= uadm[i]);
            any |= bal[i];
        }
        return any;
    };
    // Compaction of user r's list (r wave-uniform): entries in lanes, excluded
    // ones dropped (check), tau = the rank-th best (rank = amount, or amount +
    // the split's excluded-id count where they were not checked), the band
    // s' >= tau - 2M kept in lane order.  Returns the band's mask and sets
    // the entries' values; the caller writes them where they belong.
    auto compact = [&](int r, bool final_, float& v, int32_t& it, float& bound)
                       __attribute__((always_inline)) -> uint64_t {
        const int m = m0 + r;
        const int n = min(__builtin_amdgcn_readlane(lcnt, r), CAP);
        v = -INFINITY;
        it = 0x7fffffff;
        if (lane < n) { v = s_sc[m][lane]; it = s_id[m][lane]; }
        const int64_t elo = s_elo[m], ehi = s_ehi[m];
        const int extra = (int)(ehi - elo);
        const bool check = !probing && (final_ || !A.defer || A.amount + extra > (CAP - 32) / 2);
        if (check) {
            bool ex = false;
            const int exo = s_exoff[m];
            if (exo >= 0) {                              // cached in LDS
                for (int b0 = 0; b0 < extra; b0 += kWave) {          // wave-uniform
                    const int e = b0 + lane < extra ? s_exw[exo + b0 + lane] : -1;
                    const int ne = min(kWave, extra - b0);
                    for (int x = 0; x < ne; ++x) ex |= __builtin_amdgcn_readlane(e, x) == it;
                }
            } else {
                for (int64_t b0 = elo; b0 < ehi; b0 += kWave) {      // wave-uniform
                    const int64_t j = b0 + lane;
                    const int32_t e = j < ehi ? A.ex_items[j] : -1;
                    const int ne = (int)min((int64_t)kWave, ehi - b0);
                    for (int x = 0; x < ne; ++x) ex |= __builtin_amdgcn_readlane(e, x) == it;
                }
            }
            if (ex) { v = -INFINITY; it = 0x7fffffff; }
        }
        // the rank-th best s' (the entry of rank - 1 in (s' desc, id asc))
        const bool val = v != -INFINITY;
        const int rank = A.amount + (check || probing ? 0 : extra);   // <= CAP - 32 (kMwMaxAmount)
        bound = -INFINITY;
        if (__popcll(__builtin_amdgcn_ballot_w64(val)) >= rank)
            bound = wave_rth_largest(v, val, rank) - 2.f * s_m[m];
        bound = fmaxf(bound, readlane_f(lfloor, r));
        return __builtin_amdgcn_ballot_w64(val && v >= bound);
    };
    auto pos_in = [&](uint64_t mask) __attribute__((always_inline)) -> int {
        return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    };
    // admitted scores of accumulator row i go to their users' lists
    auto insert_row = [&](int i, int c0, const f32x16& acc, float bic, uint64_t bal)
                          __attribute__((always_inline)) {
        const uint32_t below = (1u << c) - 1u;
        const int r0 = (i & 3) + 8 * (i >> 2), r1 = r0 + 4;
        const uint32_t lo = (uint32_t)bal, hi = (uint32_t)(bal >> 32);
        const int base0 = __builtin_amdgcn_readlane(lcnt, r0);
        const int base1 = __builtin_amdgcn_readlane(lcnt, r1);
        const uint32_t half = h ? hi : lo;
        if ((half >> c) & 1) {
            const int pos = (h ? base1 : base0) + __builtin_popcount(half & below);
            const int m = m0 + (h ? r1 : r0);
            if (pos < CAP) {
                s_sc[m][pos] = ((A.mu + bic) + ubu[i]) + acc[i];
                s_id[m][pos] = c0 + c;
            } else {
                s_lost = 1;
            }
        }
        lcnt = writelane_i(base0 + __builtin_popcount(lo), r0, lcnt);
        lcnt = writelane_i(base1 + __builtin_popcount(hi), r1, lcnt);
    };
    auto settle = [&]() __attribute__((always_inline)) {
        // compact the lists that might not take another tile
        uint64_t full = __builtin_amdgcn_ballot_w64(lane < 32 && lcnt > A.fill);
        if (full) {
            asm volatile("" ::: "memory");
            while (full) {
                const int r = __builtin_ctzll(full);          // wave-uniform
                full &= full - 1;
                float v, bound;
                int32_t it;
                const uint64_t keep = compact(r, false, v, it, bound);
                int nk = __popcll(keep);
                const int p = pos_in(keep);
                if ((keep >> lane) & 1) {
                    if (p < CAP - 32) {
                        s_sc[m0 + r][p] = v;
                        s_id[m0 + r][p] = it;
                    }
                }
                if (nk > CAP - 32) {                          // the band does not fit
                    if (lane == 0) s_lost = 1;
                    nk = CAP - 32;
                }
                lcnt = writelane_i(nk, r, lcnt);
                ladm = __builtin_bit_cast(float, writelane_i(__builtin_bit_cast(int, bound), r,
                                                            __builtin_bit_cast(int, ladm)));
                asm volatile("" ::: "memory");
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int r0 = (i & 3) + 8 * (i >> 2);
                const float a0 = readlane_f(ladm, r0), a1 = readlane_f(ladm, r0 + 4);
                uadm[i] = h ? a1 : a0;
            }
        }
    };
    auto insert = [&](int c0, const f32x16& acc, float bic, const uint64_t (&bal)[16])
                      __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (bal[i]) insert_row(i, c0, acc, bic, bal[i]);       // wave-uniform
        settle();
    };
    // Probe walk (A.n_probe > 0): the probe items (k_topk_probe) first, the
    // users' excluded ones masked out.  The amount-th best s' of a user's list
    // minus 2M is a floor under every later admission bound of the user: its
    // `amount` probe items at or above tau have exact scores >= tau - M, so
    // an item of the exact top `amount` has s >= tau - M, s' >= tau - 2M.  The
    // lists are emptied afterwards (each probe item is scored again in its
    // own split).  C3 model, a NumPy model of the admission rule: ~167
    // admissions per user and split without it, ~3 with 512 probe items.
    if (A.n_probe > 0) {
        const int np = A.n_probe, G = A.probe_group;
        // bit g of user r: probe item g is one of r's excluded items (an item
        // e can only be probe item e / G)
        for (int x = lane; x < 32 * kMwProbeWords; x += kWave) s_pexw[x] = 0ull;
        asm volatile("" ::: "memory");
        if (A.ex_ptr && q0 < A.nq) {
            const int64_t elo = A.ex_ptr[q0], ehi = A.ex_ptr[min(q0 + 32, A.nq)];
            constexpr int U = 4;                         // loads in flight per lane
            for (int64_t b0 = elo; b0 < ehi; b0 += U * kWave) {        // wave-uniform
                int32_t e[U], pg[U];
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const int64_t t = b0 + j * kWave + lane;
                    e[j] = t < ehi ? A.ex_items[t] : -1;
                }
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const int g = e[j] >= 0 && e[j] < A.n_items ? e[j] / G : np;
                    pg[j] = g < np ? A.probe[g] : -2;
                }
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    if (pg[j] == e[j]) {                 // rare: whose exclusion is it?
                        const int64_t t = b0 + j * kWave + lane;
                        int r = 0;
                        while (r + 1 < 32 && q0 + r + 1 < A.nq && A.ex_ptr[q0 + r + 1] <= t) ++r;
                        const int g = e[j] / G;
                        atomicOr(reinterpret_cast<unsigned long long*>(
                                     &s_pexw[r * kMwProbeWords + (g >> 6)]),
                                 1ull << (g & 63));
                    }
                }
            }
        }
        asm volatile("" ::: "memory");
        probing = true;
        auto load_p = [&](int t0) __attribute__((always_inline)) {
            const int sl = t0 + c;
            if constexpr (BF) {       // the probe tiles follow the item tiles
                bi = A.Bi[A.probe[sl < np ? sl : np - 1]];
                fetch_bf(A.Qs + (int64_t)(n_tiles + (t0 >> 5)) * NB * 2 * 64, 2);
            } else {
                fetch(A.probe[sl < np ? sl : np - 1], 2);
            }
        };
        load_p(0);
        for (int t0 = 0; t0 < np; t0 += 32) {
            f32x16 acc;
            tile(acc);
            const float bic = bi;
            if (t0 + 32 < np) load_p(t0 + 32);
            const int sl = t0 + c;
            const bool have = sl < np;
            const uint64_t* pw = s_pexw + (have ? sl >> 6 : 0);
            uint64_t bal[16], any = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int r = (i & 3) + 8 * (i >> 2) + 4 * h;
                const bool ex = (pw[r * kMwProbeWords] >> (sl & 63)) & 1ull;
                const float sp = ((A.mu + bic) + ubu[i]) + acc[i];
                bal[i] = __builtin_amdgcn_ballot_w64(have && !ex && sp >= uadm[i]);
                any |= bal[i];
            }
            if (any) insert(t0, acc, bic, bal);
        }
        asm volatile("" ::: "memory");
        for (int r = 0; r < 32; ++r) {
            if (q0 + r >= A.nq) break;                   // wave-uniform
            float v, bound;
            int32_t it;
            (void)compact(r, false, v, it, bound);
            lfloor = writelane_f(bound, r, lfloor);
        }
        probing = false;
        lcnt = 0;
        ladm = q0 + c < A.nq ? lfloor : INFINITY;
        if (A.defer != 2) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int r0 = (i & 3) + 8 * (i >> 2);
                const float a0 = readlane_f(ladm, r0), a1 = readlane_f(ladm, r0 + 4);
                uadm[i] = h ? a1 : a0;
            }
        }
        asm volatile("" ::: "memory");
    }
    // The excluded ids of this wave's users in the split, packed into the
    // wave's LDS area (users in order while they fit; the rest search HBM):
    // a compaction then checks its list without a global-memory round trip.
    {
        int incl = ex_n;                                 // inclusive scan over lanes 0..31
        for (int o = 1; o < 32; o <<= 1) {
            const int t = __shfl_up(incl, o, kWave);
            if (c >= o) incl += t;
        }
        const int off = incl - ex_n;
        const bool fits = incl <= kMwExCap;
        if (lane < 32) s_exoff[m0 + lane] = fits ? off : -1;
        const uint64_t fm = __builtin_amdgcn_ballot_w64(lane < 32 && fits);
        const int nfit = __popcll(fm);                   // users 0 .. nfit-1 are cached
        const int ntot = nfit > 0 ? __builtin_amdgcn_readlane(incl, nfit - 1) : 0;
        asm volatile("" ::: "memory");
        // all loads in flight first, then the LDS stores
        constexpr int kSteps = kMwExCap / kWave;
        int32_t val[kSteps];
#pragma unroll
        for (int j = 0; j < kSteps; ++j) {
            const int t = lane + kWave * j;
            val[j] = 0;
            if (t < ntot) {
                int u = 0;                               // last user whose range starts at or before t
                for (int r = 1; r < nfit; ++r) u += __builtin_amdgcn_readlane(off, r) <= t ? 1 : 0;
                val[j] = A.ex_items[s_elo[m0 + u] + (t - s_exoff[m0 + u])];
            }
        }
#pragma unroll
        for (int j = 0; j < kSteps; ++j)
            if (lane + kWave * j < ntot) s_exw[lane + kWave * j] = val[j];
    }
    asm volatile("" ::: "memory");
    if constexpr (PIPE && BF) {
        // Two operand sets (round 6): tile c+2 loads into the set tile c
        // used, right after the first MFMA of tile c+1 -- a whole tile of
        // MFMAs and admission work ahead of its use.  (With one set, the
        // second half of tile c+2's operands could only load once tile
        // c+1's last MFMA had read that half, i.e. at the step's end, and
        // the next step waited for it.)
        bf16x8 sh[2][NB], sl[2][NB];
        float sb[2];
        auto fetch_set = [&](int it0, int S) __attribute__((always_inline)) {
            sb[S] = A.Bi[item_of(it0)];
            const bf16x8* tb = tile_ptr(it0);
#pragma unroll
            for (int s2 = 0; s2 < NB; ++s2) {
                sh[S][s2] = tb[(2 * s2) * 64 + lane];
                sl[S][s2] = tb[(2 * s2 + 1) * 64 + lane];
            }
        };
        auto mfma_s = [&](f32x16& x, int m, int S) __attribute__((always_inline)) {
            const int s2 = m / 3, t = m % 3;
            x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t == 0 ? al[s2] : ah[s2],
                                                        t == 1 ? sl[S][s2] : sh[S][s2], x, 0, 0, 0);
        };
        f32x16 xa, xb;
        fetch_set(ibeg, 0);
        fetch_set(ibeg + 32, 1);
#pragma unroll
        for (int i = 0; i < 16; ++i) xa[i] = 0.f;
#pragma unroll
        for (int m = 0; m < NM; ++m) mfma_s(xa, m, 0);
        // x: tile c0 (its operands were set 1 - S), y: tile c0 + 32 from set S
        auto step2 = [&](int c0, f32x16& x, f32x16& y, int S) __attribute__((always_inline)) {
            const float bx = sb[1 - S];
            const float mb = A.mu + bx;
#pragma unroll
            for (int i = 0; i < 16; ++i) y[i] = 0.f;
            const bool have = c0 + c < iend;
            // the admission test of tile c0 as in `step` below (sign bits of
            // sp - adm ANDed over the rows; the exact per-row test decides)
            uint32_t neg = 0xffffffffu;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
#pragma unroll
                for (int m = i * NM / 16; m < (i + 1) * NM / 16; ++m) mfma_s(y, m, S);
                if (i == 1) fetch_set(c0 + 64, 1 - S);
                const float sp = (mb + ubu[i]) + x[i];
                neg &= __builtin_bit_cast(uint32_t, sp - uadm[i]);
            }
            if (__builtin_amdgcn_ballot_w64(have && !(neg >> 31))) {     // wave-uniform
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float sp = (mb + ubu[i]) + x[i];
                    const uint64_t bal = __builtin_amdgcn_ballot_w64(have && sp >= uadm[i]);
                    if (bal) insert_row(i, c0, x, bx, bal);
                }
            }
            settle();
        };
        for (int c0 = ibeg; c0 < iend; c0 += 64) {
            step2(c0, xa, xb, 1);
            if (c0 + 32 < iend) step2(c0 + 32, xb, xa, 0);
        }
    } else if constexpr (PIPE) {
        load_b(ibeg);
        // Tile c+1's MFMAs interleaved with tile c's admission, row by row:
        // the 16 accumulator rows of tile c are compared and inserted
        // between the SEG / 16 MFMAs of each slice of tile c+1, so the list
        // work runs while the matrix pipe executes (an MFMA chain leaves the
        // wave free to issue other instructions between its links).  B
        // operands of tile c+2 are loaded in two halves, each as soon as the
        // MFMAs of tile c+1 have read that half.
        f32x16 xa, xb;
        float ba, bb;
        tile(xa);
        ba = bi;
        load_b(ibeg + 32);
        // (the first part: the operands the MFMAs of rows 0..7 have read --
        // f32: whole float4 groups among the first SEG / 2 columns; BF: the
        // first NB / 2 column groups, whose 3 NB / 2 MFMAs come first)
        auto load_half = [&](int it0, int part) __attribute__((always_inline)) {
            if constexpr (BF) fetch_tile(it0, part);
            else fetch(item_of(it0), part);
        };
        auto step = [&](int c0, f32x16& x, float& bx, f32x16& y, float& by)
                        __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 16; ++i) y[i] = 0.f;
            by = bi;
            const bool have = c0 + c < iend;
            // admission test of tile c's rows between the MFMAs, one branch
            // per tile (a tile admits anything rarely once the floor is set:
            // the per-row ballot and branch were most of the loop's issue).
            // Branch-free: the sign bits of sp - adm ANDed over the rows
            // (sp >= adm <=> sp - adm >= +0 for finite sp, adm = +-inf
            // included); a NaN only sends the tile to the exact per-row
            // test below, which decides.
            const float mb = A.mu + bx;
            uint32_t neg = 0xffffffffu;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
#pragma unroll
                for (int m = i * NM / 16; m < (i + 1) * NM / 16; ++m) mfma_m(y, m);
                if (i == 7) load_half(c0 + 64, 0);       // tile c+2, columns of the first half
                const float sp = (mb + ubu[i]) + x[i];
                neg &= __builtin_bit_cast(uint32_t, sp - uadm[i]);
            }
            const bool anyl = have && !(neg >> 31);
            if (__builtin_amdgcn_ballot_w64(anyl)) {     // wave-uniform
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float sp = ((A.mu + bx) + ubu[i]) + x[i];
                    const uint64_t bal = __builtin_amdgcn_ballot_w64(have && sp >= uadm[i]);
                    if (bal) insert_row(i, c0, x, bx, bal);
                }
            }
            load_half(c0 + 64, 1);
            settle();
        };
        for (int c0 = ibeg; c0 < iend; c0 += 64) {
            step(c0, xa, ba, xb, bb);
            if (c0 + 32 < iend) step(c0 + 32, xb, bb, xa, ba);
        }
    } else {
        load_b(ibeg);
        for (int c0 = ibeg; c0 < iend; c0 += 32) {
            f32x16 acc;
            tile(acc);
            const float bic = bi;
            if (c0 + 32 < iend) load_b(c0 + 32);
            uint64_t bal[16];
            if (admit(c0, acc, bic, bal)) insert(c0, acc, bic, bal);
        }
    }
    // final: every list checked against the exclusions and cut to its band,
    // written (unsorted) as this split's band of the user
    asm volatile("" ::: "memory");
    for (int r = 0; r < 32; ++r) {
        const int qy = q0 + r;
        if (qy >= A.nq) break;                           // wave-uniform
        float v, bound;
        int32_t it;
        const uint64_t keep = compact(r, true, v, it, bound);
        const int64_t o = ((int64_t)qy * A.n_splits + split) * kMmCap;
        if ((keep >> lane) & 1) {
            const int p = pos_in(keep);
            A.part_s[o + p] = v;
            A.part_id[o + p] = it;
        }
        if (lane == 0) A.part_n[(int64_t)qy * A.n_splits + split] = __popcll(keep);
    }
    __syncthreads();
    if (tid == 0 && s_lost) atomicOr(A.overflow, 1);
}

// per user: merge the splits' bands, keep s' >= (amount-th best s') - 2M,
// rescore those with k_read's arithmetic, rank by (score desc, id asc) --
// the order keys and the sort of k_topk_merge, so the output is its output
template <int GS>
__global__ __launch_bounds__(kBlock) void k_topk_mm_merge(MmArgs A, int32_t* out_items,
                                                          float* out_scores) {
    __shared__ float s_sc[kMmMaxSplits * kMmCap];
    __shared__ int32_t s_id[kMmMaxSplits * kMmCap];
    __shared__ uint64_t s_key[kMmMaxSplits * kMmCap];
    __shared__ int s_off[kMmMaxSplits + 1], s_keep;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1), wv = tid / kWave;
    const int ns = A.n_splits;                       // <= kMmMaxSplits (topk_mm_splits)
    // the users k_topk_mm_merge_wave listed (bands past 64 entries), or all
    const int n_users = A.big ? *A.n_big : A.nq;
    for (int xq = blockIdx.x; xq < n_users; xq += gridDim.x) {
    const int qy = A.big ? A.big[xq] : xq;
    if (tid == 0) {
        int n = 0;
        for (int x = 0; x < ns; ++x) { s_off[x] = n; n += A.part_n[(int64_t)qy * ns + x]; }
        s_off[ns] = n;
    }
    __syncthreads();
    const int n = s_off[ns];
    int n2 = 1;
    while (n2 < max(n, 1)) n2 <<= 1;
    for (int y = tid; y < n2; y += kBlock) {
        float sc = -INFINITY;
        int32_t id = 0x7fffffff;
        if (y < n) {
            int x = 0;
            while (y >= s_off[x + 1]) ++x;
            const int64_t o = ((int64_t)qy * ns + x) * kMmCap + (y - s_off[x]);
            sc = A.part_s[o];
            id = A.part_id[o];
        }
        s_sc[y] = sc;
        s_id[y] = id;
    }
    __syncthreads();
    mm_sort(s_sc, s_id, n2, tid);
    if (tid == 0) {
        int keep = n;
        if (n >= A.amount) {
            const float adm = s_sc[A.amount - 1] - 2.f * A.marg[qy];
            keep = A.amount;
            while (keep < n && s_sc[keep] >= adm) ++keep;
        }
        s_keep = keep;
    }
    __syncthreads();
    const int keep = s_keep;
    // exact rescoring: one candidate per group of GS lanes (scalar layout,
    // lane partial 0 + p_f q_f, group_sum<GS>, predict_one's additions)
    const int32_t uu = A.users[qy];
    const float bu = uu >= 0 ? A.Bu[uu] : 0.f;
    const int k = A.k;
    const int g = lane / GS, l = lane % GS;
    constexpr int R = kWave / GS;
    const float pl = (uu >= 0 && l < k) ? A.P[(int64_t)uu * k + l] : 0.f;
    for (int y0 = wv * R; y0 < keep; y0 += kWavesPerBlock * R) {
        const int y = y0 + g;
        const bool have = y < keep;
        const int32_t it = have ? s_id[y] : 0;
        const float ql = (have && l < k) ? A.Q[(int64_t)it * k + l] : 0.f;
        const float sc = group_sum<GS>(0.f + pl * ql);
        const float pred = ((A.mu + (have ? A.Bi[it] : 0.f)) + bu) + sc;
        if (have && l == 0) s_key[y] = order_key((double)pred);
    }
    __syncthreads();
    int k2 = 1;
    while (k2 < max(keep, 1)) k2 <<= 1;
    for (int y = keep + tid; y < k2; y += kBlock) { s_key[y] = 0ull; s_id[y] = 0x7fffffff; }
    __syncthreads();
    cand_sort(s_key, s_id, k2, tid, kBlock);
    for (int y = tid; y < A.amount; y += kBlock) {
        const bool ok = y < keep && s_key[y] != 0ull;
        out_items[(int64_t)qy * A.amount + y] = ok ? s_id[y] : -1;
        out_scores[(int64_t)qy * A.amount + y] =
            ok ? (float)key_score(s_key[y]) : __int_as_float(0x7fc00000);
    }
    __syncthreads();                                 // the LDS lists are reused
    }
}

// k_topk_mm_merge for the users whose bands hold at most 64 entries over
// all splits (C3, top-10: ~18): one wave per user, entries one per lane, no
// workgroup barrier (round 6; the workgroup-per-user form's two bitonic
// sorts with a barrier per stage took 90 us of the C3 top-k's 1.07 ms).
// Same keep rule (s' >= the amount-th best s' - 2M), the same rescoring
// arithmetic and the same (key desc, id asc) order, so the same output;
// users with more entries are listed for k_topk_mm_merge (A.big).
template <int GS>
__global__ __launch_bounds__(kBlock) void k_topk_mm_merge_wave(MmArgs A, int32_t* out_items,
                                                               float* out_scores) {
    __shared__ int32_t s_kid[kWavesPerBlock][kWave];
    __shared__ uint64_t s_kkey[kWavesPerBlock][kWave];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int qy = blockIdx.x * kWavesPerBlock + wv;
    if (qy >= A.nq) return;                              // wave-uniform
    const int ns = A.n_splits;
    // offsets of the splits' bands (inclusive scan over lanes < ns)
    const int cnt = lane < ns ? A.part_n[(int64_t)qy * ns + lane] : 0;
    int incl = cnt;
    for (int o = 1; o < kMmMaxSplits; o <<= 1) {
        const int t = __shfl_up(incl, o, kWave);
        if (lane >= o) incl += t;
    }
    const int n = __builtin_amdgcn_readlane(incl, kMmMaxSplits - 1);
    if (n > kWave) {                                     // k_topk_mm_merge's user
        if (lane == 0) A.big[atomicAdd(A.n_big, 1)] = qy;
        return;
    }
    float sc = -INFINITY;
    int32_t id = 0x7fffffff;
    const bool valid = lane < n;
    int x = 0, base = 0;                                 // split of entry `lane`, its start
    for (int t = 0; t < ns; ++t) {                       // wave-uniform
        const int end = __builtin_amdgcn_readlane(incl, t);
        if (lane >= end) { x = t + 1; base = end; }
    }
    if (valid) {
        const int64_t o = ((int64_t)qy * ns + x) * kMmCap + (lane - base);
        sc = A.part_s[o];
        id = A.part_id[o];
    }
    uint64_t keep = __builtin_amdgcn_ballot_w64(valid);
    if (n >= A.amount) {
        // the amount-th best s' (the sorted list's entry amount - 1)
        const float adm = wave_rth_largest(sc, valid, A.amount) - 2.f * A.marg[qy];
        keep = __builtin_amdgcn_ballot_w64(valid && sc >= adm);
    }
    const int K = __popcll(keep);
    const int pos = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(keep >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)keep, 0u));
    if ((keep >> lane) & 1) s_kid[wv][pos] = id;
    asm volatile("" ::: "memory");
    // exact rescoring, R candidates per pass (k_topk_mm_merge's arithmetic)
    const int32_t uu = A.users[qy];
    const float bu = uu >= 0 ? A.Bu[uu] : 0.f;
    const int k = A.k;
    const int g = lane / GS, l = lane % GS;
    constexpr int R = kWave / GS;
    const float pl = (uu >= 0 && l < k) ? A.P[(int64_t)uu * k + l] : 0.f;
    constexpr int U = 4;                                 // candidates' loads in flight
    for (int y0 = 0; y0 < K; y0 += U * R) {              // wave-uniform
        float ql[U], bq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int y = y0 + u * R + g;
            const bool have = y < K;
            const int32_t it = have ? s_kid[wv][y] : 0;
            ql[u] = (have && l < k) ? A.Q[(int64_t)it * k + l] : 0.f;
            bq[u] = have ? A.Bi[it] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int y = y0 + u * R + g;
            const float s2 = group_sum<GS>(0.f + pl * ql[u]);
            const float pred = ((A.mu + bq[u]) + bu) + s2;
            if (y < K && l == 0) s_kkey[wv][y] = order_key((double)pred);
        }
    }
    asm volatile("" ::: "memory");
    // (key desc, id asc) rank among the K kept, the first `amount` written
    uint64_t key = 0;
    int32_t kid = 0x7fffffff;
    if (lane < K) { key = s_kkey[wv][lane]; kid = s_kid[wv][lane]; }
    int rk = 0;
    for (int j = 0; j < K; ++j) {
        const uint64_t kj = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(key >> 32), j) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, j);
        const int32_t ij = __builtin_amdgcn_readlane(kid, j);
        rk += cand_before(kj, ij, key, kid) ? 1 : 0;
    }
    const int64_t ob = (int64_t)qy * A.amount;
    if (lane < K && rk < A.amount) {
        out_items[ob + rk] = kid;
        out_scores[ob + rk] = (float)key_score(key);
    }
    for (int y = K + lane; y < A.amount; y += kWave) {
        out_items[ob + y] = -1;
        out_scores[ob + y] = __int_as_float(0x7fc00000);
    }
}

// 32-user MFMA tiles per wave of k_topk_mm: 1 (the default: 32 users, 64 KB
// of lists, 251 VGPRs, two workgroups per CU, so one workgroup's MFMAs run
// beside the other's admission, barriers and compaction) or 2 (64 users,
// 128 KB, one workgroup per CU; the round-2 form).  C3, 10K users: 3.55 vs
// 5.52 ms (gpurun_out r02s14).
inline int topk_mm_nt() {
    if (const char* e = std::getenv("MF_TOPK_MM_NT")) {          // probes
        const int v = std::atoi(e);
        if (v == 1 || v == 2) return v;
    }
    return 1;
}

inline int topk_mm_splits(int32_t nq, int32_t n_items) {
    if (const char* e = std::getenv("MF_TOPK_MM_SPLITS")) {      // probes
        const int v = std::atoi(e);
        if (v >= 1 && v <= kMmMaxSplits) return v;
    }
    const int nt = topk_mm_nt();
    const int64_t blocks_q = ((int64_t)nq + 32 * nt - 1) / (32 * nt);
    // ~1.9 rounds of the resident workgroups (one per CU at nt = 2; C3, 10K
    // users: 3 splits, 5.3 ms; 1 / 2 / 4 splits 5.5 / 6.9 / 6.5 ms, gpurun_out r02z)
    int64_t s = (480 * (3 - nt) + blocks_q / 2) / blocks_q;
    s = std::min<int64_t>(s, std::max<int64_t>(1, n_items / 2048));
    s = std::min<int64_t>(s, 4);                            // merge: 4 x kMmCap entries
    return (int)std::max<int64_t>(1, s);
}

// the wave-private form (k_topk_mw) for small amounts; MF_TOPK_MW=0 keeps
// k_topk_mm (probes, A/B)
inline bool topk_use_mw(int32_t amount) {
    if (amount > kMwMaxAmount) return false;
    const char* e = std::getenv("MF_TOPK_MW");
    return !(e && std::atoi(e) == 0);
}

// k_topk_mw: 128 users per workgroup, two workgroups per CU; item splits so
// that the grid is about one round of the resident workgroups (C3, 10K
// users: 79 user blocks x 6 splits = 474)
inline int topk_mw_splits(int32_t nq, int32_t n_items) {
    if (const char* e = std::getenv("MF_TOPK_MM_SPLITS")) {      // probes
        const int v = std::atoi(e);
        if (v >= 1 && v <= kMmMaxSplits) return v;
    }
    const int64_t blocks_q = ((int64_t)nq + kMwUsers - 1) / kMwUsers;
    int64_t s = (512 + blocks_q / 2) / blocks_q;
    s = std::min<int64_t>(s, std::max<int64_t>(1, n_items / 2048));
    s = std::min<int64_t>(s, kMmMaxSplits);
    return (int)std::max<int64_t>(1, s);
}

struct TopkLaunch {
    const int32_t* users; int32_t nq; double mu; const void* bu; const void* bi;
    const void* P; const void* Q; int32_t n_items; int32_t k; double gamma, lo, hi;
    const int64_t* ex_ptr; const int32_t* ex_items; int32_t amount; void* ws; int32_t* out_items; void* out_scores;
    hipStream_t stream;

    template <typename T, int GS, int V, int KERN>
    int run() {
        if (topk_fused(amount)) {
            FusedArgs<T> f;
            f.users = users; f.nq = nq; f.P = (const T*)P; f.Q = (const T*)Q;
            f.Bu = (const T*)bu; f.Bi = (const T*)bi; f.n_items = n_items; f.k = k;
            f.amount = amount;
            int a2 = 1;
            while (a2 < amount) a2 <<= 1;
            f.a2 = a2;
            f.n_splits = topk_splits(nq, n_items, amount);
            f.h = make_hyper<T>(mu, 0.0, 0.0, gamma, lo, hi);
            f.ex_ptr = ex_items ? ex_ptr : nullptr; f.ex_items = ex_items;
            const size_t np = (size_t)nq * f.n_splits * amount;
            f.part_key = (uint64_t*)ws;
            f.part_id = (int32_t*)((uint64_t*)ws + np);
            const unsigned by = (unsigned)((nq + kFusedUsers - 1) / kFusedUsers);
            hipLaunchKernelGGL((k_topk_fused<T, GS, V, KERN>), dim3((unsigned)f.n_splits, by),
                               dim3(kBlock), 0, stream, f);
            hipLaunchKernelGGL(k_topk_merge<T>, dim3((unsigned)nq), dim3(kBlock), 0, stream,
                               (const uint64_t*)f.part_key, (const int32_t*)f.part_id, f.n_splits,
                               amount, out_items, (T*)out_scores);
            MF_HIP_CHECK(hipGetLastError());
            return MF_OK;
        }
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

void touch_topk(hipStream_t s) { hipLaunchKernelGGL(k_touch<6>, dim3(1), dim3(64), 0, s); }

}  // namespace mf

#include "mf_dispatch.hpp"

using namespace mf;

extern "C" size_t mf_topk_workspace_bytes(int32_t n_query, int32_t n_items, int32_t amount) {
    if (n_query <= 0 || n_items <= 0) return 0;
    if (topk_fused(amount))       // partial lists: n_query x splits x amount (key + id)
        return (sizeof(uint64_t) + sizeof(int32_t)) * (size_t)n_query *
               (size_t)topk_splits(n_query, n_items, amount) * (size_t)std::max(amount, 1);
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

// ---------------------------------------------------------------- MFMA filter ABI
static int mm_seg(int k) { return ((k / 2 + 3) / 4) * 4; }
// bytes per item of k_topk_split_q's rows at the largest k (2 halves x hi / lo x NB groups)
constexpr size_t kMwSplitRowBytes = 2 * 2 * ((kMmMaxK / 2 + 7) / 8) * sizeof(bf16x8);

extern "C" int32_t mf_topk_mm_supported(int32_t n_factors, int32_t kernel, int32_t dtype,
                                        int32_t amount) {
    return (dtype == MF_F32 && kernel == MF_LINEAR && n_factors >= 4 && n_factors <= kMmMaxK &&
            n_factors % 4 == 0 && amount >= 1 && amount <= kFusedMaxAmount) ? 1 : 0;
}

extern "C" size_t mf_topk_mm_workspace_bytes(int32_t n_query, int32_t n_items) {
    if (n_query <= 0 || n_items <= 0) return 0;
    // room for either kernel's bands (the launch picks by amount)
    const size_t ns = (size_t)std::max(topk_mm_splits(n_query, n_items),
                                       topk_mw_splits(n_query, n_items));
    return 16 + 4 * (size_t)n_query + 4 * (size_t)n_query * ns +
           8 * (size_t)n_query * ns * kMmCap + 4 * (size_t)kMwProbe + 4 * (size_t)n_query + 16 +
           kMwSplitRowBytes * (32 * (((size_t)n_items + 31) / 32) + kMwProbe);
}

// k_topk_mw's operands: bf16 hi + lo parts on the bf16 MFMA (BF, 5.3x fewer
// matrix cycles than the f32 MFMA per tile) -- MF_TOPK_BF16=0: f32 (probes)
inline bool topk_mw_bf16() {
    const char* e = std::getenv("MF_TOPK_BF16");
    return !(e && std::atoi(e) == 0);
}

// k_topk_mw's probe items: one per group of >= 128 item ids, at most kMwProbe
// (C3, 100K items: 511 groups of 196; the caller trims the count so that no
// group is empty).  MF_TOPK_PROBE=0: none (probes, A/B).
inline int topk_mw_probes(int32_t n_items) {
    if (const char* e = std::getenv("MF_TOPK_PROBE"))
        if (std::atoi(e) == 0) return 0;
    return std::min<int32_t>(kMwProbe, n_items / 128);
}

extern "C" int mf_topk_mm(const int32_t* query_users, int32_t n_query, double global_mean,
                          const void* user_biases, const void* item_biases,
                          const void* user_features, const void* item_features, int32_t n_items,
                          int32_t n_factors, int32_t kernel, int32_t dtype,
                          const int64_t* exclude_ptr, const int32_t* exclude_items,
                          int32_t amount, void* workspace, int32_t* out_items, void* out_scores,
                          int32_t* overflow, void* stream) {
    if (!mf_topk_mm_supported(n_factors, kernel, dtype, amount)) {
        set_error("mf_topk_mm: linear kernel, float32, n_factors a multiple of 4 in [4, %d], "
                  "1 <= amount <= %d only (use mf_topk)", kMmMaxK, kFusedMaxAmount);
        return MF_ERR_INVALID;
    }
    if (n_query < 0 || n_items <= 0) {
        set_error("mf_topk_mm: n_query >= 0 and n_items > 0 required");
        return MF_ERR_INVALID;
    }
    if (n_query == 0) return MF_OK;
    if (!workspace || !out_items || !out_scores || !query_users || !overflow ||
        !user_features || !item_features || !user_biases || !item_biases) {
        set_error("mf_topk_mm: NULL buffer");
        return MF_ERR_INVALID;
    }
    hipStream_t st = (hipStream_t)stream;
    MmArgs a;
    a.users = query_users; a.nq = n_query;
    a.P = (const float*)user_features; a.Q = (const float*)item_features;
    a.Bu = (const float*)user_biases; a.Bi = (const float*)item_biases;
    a.n_items = n_items; a.k = n_factors; a.amount = amount;
    const bool mw = topk_use_mw(amount);
    a.n_splits = mw ? topk_mw_splits(n_query, n_items) : topk_mm_splits(n_query, n_items);
    a.mu = (float)global_mean;
    a.ex_ptr = exclude_items ? exclude_ptr : nullptr; a.ex_items = exclude_items;
    char* w = (char*)workspace;
    float* stats = (float*)w;
    a.stats = stats;
    a.marg = (float*)(w + 16);
    a.part_n = (int32_t*)(a.marg + n_query);
    a.part_s = (float*)(a.part_n + (size_t)n_query * a.n_splits);
    a.part_id = (int32_t*)(a.part_s + (size_t)n_query * a.n_splits * kMmCap);
    a.overflow = overflow;
    a.probe = (int32_t*)(a.part_id + (size_t)n_query * a.n_splits * kMmCap);
    a.big = const_cast<int32_t*>(a.probe) + kMwProbe;
    a.n_big = reinterpret_cast<int32_t*>(stats) + 3;    // zeroed with the statistics
    {
        const uintptr_t qs = reinterpret_cast<uintptr_t>(a.big + n_query);
        a.Qs = reinterpret_cast<const bf16x8*>((qs + 15) & ~(uintptr_t)15);
    }
    const char* pe = std::getenv("MF_TOPK_MM_PIPE");
    const bool pipe = pe ? std::atoi(pe) != 0 : true;
    const bool bf = mw && pipe && topk_mw_bf16();
    a.n_probe = mw ? topk_mw_probes(n_items) : 0;
    a.probe_group = a.n_probe > 0 ? (n_items + a.n_probe - 1) / a.n_probe : 0;
    // every group non-empty (C3: 512 groups of 196 ids would leave the last
    // one past n_items; 511 are used)
    if (a.n_probe > 0) a.n_probe = (n_items + a.probe_group - 1) / a.probe_group;
    {
        const char* e = std::getenv("MF_TOPK_MM_DEFER");             // probes
        a.defer = e ? std::atoi(e) : 0;
        // k_topk_mw: compact a list once it holds more than `fill` entries
        // (<= kMwCap - 32: room for a whole tile).  Probes: MF_TOPK_MW_FILL.
        const char* f = std::getenv("MF_TOPK_MW_FILL");
        const int fv = f ? std::atoi(f) : kMwCap - 32;
        a.fill = std::max(amount + 1, std::min(fv, kMwCap - 32));
    }
    MF_HIP_CHECK(hipMemsetAsync(stats, 0, 16, st));
    const int32_t nb_si = (int32_t)std::min<int64_t>(512, ((int64_t)n_items + kBlock - 1) / kBlock);
    const int32_t nb_su = a.n_probe > 0 ? (int32_t)std::min<int64_t>(64, ((int64_t)n_query + kBlock - 1) / kBlock) : 0;
    hipLaunchKernelGGL(k_topk_mm_stats, dim3((unsigned)(nb_si + nb_su)), dim3(kBlock), 0, st, a.Q,
                       a.Bi, n_items, n_factors, stats, query_users, n_query, a.P, nb_si);
    if (a.n_probe > 0)
        hipLaunchKernelGGL(k_topk_probe,
                           dim3((unsigned)((a.n_probe + kWavesPerBlock - 1) / kWavesPerBlock)),
                           dim3(kBlock), 0, st, a.Q, a.Bi, n_items, n_factors, a.probe_group,
                           a.n_probe, (const float*)stats, const_cast<int32_t*>(a.probe));
    if (bf) {
        const int seg = mm_seg(n_factors), nb = (seg + 7) / 8;
        const int n_tiles = (n_items + 31) / 32, n_ptiles = (a.n_probe + 31) / 32;
        const int64_t nt = (int64_t)(n_tiles + n_ptiles) * nb * 64;
        hipLaunchKernelGGL(k_topk_split_q, dim3((unsigned)((nt + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, st, a.Q, n_items, n_factors, seg, nb, n_tiles,
                           a.probe, a.n_probe, n_ptiles, const_cast<bf16x8*>(a.Qs));
    }
    const int nt = topk_mm_nt();
    const dim3 grid((unsigned)a.n_splits, (unsigned)((n_query + 32 * nt - 1) / (32 * nt)));
    const dim3 grid_mw((unsigned)a.n_splits, (unsigned)((n_query + kMwUsers - 1) / kMwUsers));
#define MF_MM_LAUNCH(S)                                                                        \
    if (mw) {                                                                                 \
        if (pipe && bf) hipLaunchKernelGGL((k_topk_mw<S, true, true>), grid_mw, dim3(kBlock), 0, st, a); \
        else if (pipe) hipLaunchKernelGGL((k_topk_mw<S, true>), grid_mw, dim3(kBlock), 0, st, a); \
        else hipLaunchKernelGGL((k_topk_mw<S, false>), grid_mw, dim3(kBlock), 0, st, a);      \
    } else if (nt == 1) {                                                                            \
        if (pipe) hipLaunchKernelGGL((k_topk_mm<S, true, 1>), grid, dim3(kBlock), 0, st, a);  \
        else hipLaunchKernelGGL((k_topk_mm<S, false, 1>), grid, dim3(kBlock), 0, st, a);      \
    } else {                                                                                  \
        if (pipe) hipLaunchKernelGGL((k_topk_mm<S, true, 2>), grid, dim3(kBlock), 0, st, a);  \
        else hipLaunchKernelGGL((k_topk_mm<S, false, 2>), grid, dim3(kBlock), 0, st, a);      \
    }
    switch (mm_seg(n_factors)) {
        case 4: MF_MM_LAUNCH(4); break;
        case 8: MF_MM_LAUNCH(8); break;
        case 12: MF_MM_LAUNCH(12); break;
        case 16: MF_MM_LAUNCH(16); break;
        case 20: MF_MM_LAUNCH(20); break;
        case 24: MF_MM_LAUNCH(24); break;
        case 28: MF_MM_LAUNCH(28); break;
        default: MF_MM_LAUNCH(32); break;
    }
#undef MF_MM_LAUNCH
    // the users with <= 64 band entries one wave each, then the others one
    // workgroup each (MF_TOPK_MERGE_WAVE=0: all by workgroups, probes)
    const char* mwv = std::getenv("MF_TOPK_MERGE_WAVE");
    const bool wave_merge = !(mwv && mwv[0] == '0');
    if (!wave_merge) a.big = nullptr;
    const dim3 grid_mrg((unsigned)((n_query + kWavesPerBlock - 1) / kWavesPerBlock));
    // the listed users (usually none) by a grid of resident workgroups
    const dim3 grid_big((unsigned)(wave_merge ? std::min<int32_t>(n_query, 512) : n_query));
#define MF_MERGE_LAUNCH(GS)                                                                      \
    if (wave_merge)                                                                           \
        hipLaunchKernelGGL(k_topk_mm_merge_wave<GS>, grid_mrg, dim3(kBlock), 0, st, a, out_items, \
                           (float*)out_scores);                                               \
    hipLaunchKernelGGL(k_topk_mm_merge<GS>, grid_big, dim3(kBlock), 0, st, a, out_items,        \
                       (float*)out_scores);
    switch (kpad_of(n_factors)) {
        case 16: MF_MERGE_LAUNCH(16); break;
        case 32: MF_MERGE_LAUNCH(32); break;
        default: MF_MERGE_LAUNCH(64); break;
    }
#undef MF_MERGE_LAUNCH
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}
