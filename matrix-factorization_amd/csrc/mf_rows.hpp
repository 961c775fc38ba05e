// mf_rows.hpp -- the two hot kernels of the KernelMF path and their launchers:
//   k_sgd_batch  one conflict-free batch of SGD updates (kernels.py:108-327
//                applied to every rating of the batch)
//   k_sse_stream training sum of squared errors (_calculate_rmse,
//                kernel_matrix_factorization.py:240-317)
//
// Row layout.  A factor row of k values is moved by a
// GROUP of GS lanes; each lane moves W consecutive values per access (W = 4
// for float, 2 for double when k allows: one 16-B global_load_dwordx4 per
// lane), V accesses per lane.  GS <= 16 for W > 1, so a group is (part of) a
// DPP row and the dot product reduces with 0..4 DPP adds; R = 64 / GS
// ratings share one wave instruction.  W = 1 keeps 16/32/64-lane groups for
// k that is not a multiple of W.
//
// Included by mf_rows_f32.hip / mf_rows_f64.hip (one dtype each).
#pragma once

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "mf_common.hpp"

namespace mf {

// ------------------------------------------------------------ memory ops
// User rows, user biases and triples stream through once per batch: load and
// store them non-temporally so they do not evict item rows from L2.
template <bool NT, typename X>
__device__ __forceinline__ X ld(const X* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, typename X>
__device__ __forceinline__ void st(X* p, X v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// User-row access policy POL of k_sgd_batch: 0 plain, 1 non-temporal
// global ops, >= 2 buffer ops with explicit gfx950 cache-policy bits
// (aux: sc0 = 1, nt = 2, sc1 = 16) -- table kPolAux, for the L2-residency
// experiments of tools/sweep_sgd.py.
struct PolAux { int ld, st; };
constexpr PolAux kPolAux[8] = {{0, 0}, {0, 0}, {0, 0}, {2, 16}, {16, 16}, {17, 17}, {19, 19}, {2, 2}};
constexpr int kBufDword3 = 0x00020000;     // raw buffer, gfx9 family

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint64_t bytes) {
    const uint32_t nr = bytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)nr, kBufDword3);
}
template <int AUX, typename X>
__device__ __forceinline__ X buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    if constexpr (sizeof(X) == 16)
        return __builtin_bit_cast(X, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX));
    else if constexpr (sizeof(X) == 8)
        return __builtin_bit_cast(X, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, AUX));
    else
        return __builtin_bit_cast(X, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, AUX));
}
// a * b + c with a, b < 2^24 (b wave-uniform) as ONE full-rate
// v_mad_u32_u24: the compiler turns (uint32_t)a * b + c into a quarter-rate
// v_mul_lo_u32 / v_mad_u64_u32 when b is a run-time value
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t o;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(o) : "v"(a), "s"(b), "v"(c));
    return o;
}

template <int AUX, typename X>
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t off, X v) {
    using U4 = __attribute__((ext_vector_type(4))) unsigned;
    using U2 = __attribute__((ext_vector_type(2))) unsigned;
    if constexpr (sizeof(X) == 16)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U4, v), r, (int)off, 0, AUX);
    else if constexpr (sizeof(X) == 8)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U2, v), r, (int)off, 0, AUX);
    else
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, AUX);
}

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
    int32_t* claim;         // nullable: 8 per-slice tile counters of this launch
    uint64_t p_bytes;       // bytes of P (buffer-policy range; < 4 GiB when POL >= 2)
    Hyper<T> h;
};

template <typename T>
struct ReadArgs {
    const int32_t* u;
    const int32_t* i;
    const T* r;
    const T* P;
    const T* Q;
    const T* Bu;
    const T* Bi;
    int64_t n;
    int32_t k;
    int32_t bound;
    T* out;
    double* partials;
    Hyper<T> h;
    // byte sizes of P, Q, Bu, Bi (buffer-load ranges of k_sse_owned; < 4 GiB)
    uint64_t p_bytes, q_bytes, bu_bytes, bi_bytes;
};

// buffer offset past every resource of the read passes: loads return zero
constexpr uint32_t kBufDropRd = 0xFFFFFFF0u;

// Work split of the read-only passes: `n` slices of the rating array (the
// item-range slices of mf_sched_slices), slice x walked by the workgroups
// b with b % n == x.  Placement only changes speed.
constexpr int kMaxSlices = 128;
struct SliceTab {
    int64_t off[kMaxSlices + 1];
    int32_t n;
};

// The slice a wave walks and its index among the slice's waves.  n <= 8 (or
// not a multiple of 8): slice b % n.  n = 8 P, P > 1: the grid is cut into P
// consecutive parts in dispatch order and part p deals slice (b % 8) + 8 p to
// block b's XCD, so at any time an XCD's L2 serves about one 1/(8 P) item
// range instead of P of them side by side (the user rows are then read P
// times per XCD instead of once).
struct SliceWave {
    int x;
    int64_t wv, nw;
};
__device__ __forceinline__ SliceWave slice_wave(const SliceTab& SL) {
    const int64_t bps = gridDim.x / SL.n;
    SliceWave s;
    int64_t j;
    if (SL.n > 8 && SL.n % 8 == 0) {
        const int64_t per = gridDim.x / (SL.n / 8);      // = 8 bps blocks per part
        const int64_t ph = blockIdx.x / per, r = blockIdx.x % per;
        s.x = (int)(r % 8 + 8 * ph);
        j = r / 8;
    } else {
        s.x = blockIdx.x % SL.n;
        j = blockIdx.x / SL.n;
    }
    s.nw = bps * kWavesPerBlock;
    s.wv = j * kWavesPerBlock + threadIdx.x / kWave;
    return s;
}

// kernels.py:21-105.  `s` = group-reduced dot product (linear/sigmoid) or
// squared distance (rbf).
template <typename T, int KERN>
__device__ __forceinline__ T predict_one(T s, T bu, T bi, const Hyper<T> h) {
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

// rating-slot broadcast: wave-uniform source -> v_readlane, else ds_bpermute
template <int GS>
__device__ __forceinline__ int take_i(int v, int src) {
    if constexpr (GS == kWave) return rl_i32(v, src);
    else return bcast_i32(v, src);
}
template <int GS, typename T>
__device__ __forceinline__ T take_f(T v, int src) {
    if constexpr (GS == kWave) return rl_f(v, src);
    else return bcast_f(v, src);
}

// Rating slots per wave: ~16 ratings and <= 32 row registers per operand.
template <int R, int V, int W>
struct SlotsFor {
    static constexpr int a = 16 / R > 0 ? 16 / R : 1;
    static constexpr int b = 32 / (V * W) > 0 ? 32 / (V * W) : 1;
    static constexpr int c = a < b ? a : b;
    static constexpr int S = c > 8 ? 8 : c;
};

// Gather the rows of S rating slots: all loads issued before any use;
// indices clamped so no load sits behind a branch; vector slots past the
// row end are zeroed afterwards.
template <typename T, int W, int GS, int V, int S, int POL>
__device__ __forceinline__ void gather_rows(const T* base, const int (&id)[S], int k, int kv, int l,
                                            typename VecOf<T, W>::type (&out)[S][V],
                                            uint64_t bytes = 0) {
    using VT = typename VecOf<T, W>::type;
    [[maybe_unused]] __amdgpu_buffer_rsrc_t rs;
    if constexpr (POL >= 2) rs = buf_rsrc(base, bytes);
#pragma unroll
    for (int x = 0; x < S; ++x) {
        const VT* row = reinterpret_cast<const VT*>(base + (int64_t)id[x] * k);
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int vi = v * GS + l;
            const int vc = vi < kv ? vi : kv - 1;
            if constexpr (POL >= 2)
                out[x][v] = buf_ld<kPolAux[POL].ld, VT>(
                    rs, (uint32_t)(((uint32_t)id[x] * (uint32_t)k + (uint32_t)(vc * W)) * sizeof(T)));
            else
                out[x][v] = ld<POL == 1>(row + vc);
        }
    }
#pragma unroll
    for (int x = 0; x < S; ++x)
#pragma unroll
        for (int v = 0; v < V; ++v)
            if (v * GS + l >= kv) out[x][v] = (VT)(T)0;
}

// FUSED: the FP32 SGD form (fused multiply-adds, see sgd_error); the read
// paths (predict, SSE, top-k) keep the unfused form they are pinned to.
template <typename T, int W, int V, int KERN, bool FUSED = false>
__device__ __forceinline__ T lane_partial(const typename VecOf<T, W>::type (&p)[V],
                                          const typename VecOf<T, W>::type (&q)[V]) {
    T s = (T)0;
#pragma unroll
    for (int v = 0; v < V; ++v) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            T a, b;
            if constexpr (W == 1) { a = p[v]; b = q[v]; }
            else { a = p[v][w]; b = q[v][w]; }
            if constexpr (FUSED && std::is_same<T, float>::value) {   // FP32 SGD: fused
                if constexpr (KERN == MF_RBF) {
                    const T d = a - b;
                    s = __builtin_fmaf(d, d, s);
                } else {
                    s = __builtin_fmaf(a, b, s);
                }
            } else if constexpr (KERN == MF_RBF) {
                const T d = a - b;
                s = s + d * d;
            } else {
                s = s + a * b;
            }
        }
    }
    return s;
}

// lane_partial of one vector without the leading 0 + (the same value up to
// the sign of a zero sum): the training-SSE form
template <typename T, int W, int KERN>
__device__ __forceinline__ T lane_partial_first(const typename VecOf<T, W>::type (&p)[1],
                                                const typename VecOf<T, W>::type (&q)[1]) {
    T s = (T)0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        T a, b;
        if constexpr (W == 1) { a = p[0]; b = q[0]; }
        else { a = p[0][w]; b = q[0][w]; }
        T t;
        if constexpr (KERN == MF_RBF) { const T d = a - b; t = d * d; }
        else t = a * b;
        s = w == 0 ? t : s + t;
    }
    return s;
}

// Per-rating SGD arithmetic shared by k_sgd_batch and k_sgd_strata (same
// expression order as the reference, FP contraction off).  `s` = group-reduced
// dot product / squared distance; returns the error e and the kernel's
// derivative factor d (1 for linear).
//
// FP32 (the reference computes in FP64, so the FP32 path is already an
// approximation held to the RMSE tolerance): exp as v_exp_f32 of x log2(e),
// the sigmoid's reciprocal as v_rcp_f32, and fused multiply-adds in the
// row updates -- the C2 step is VALU-issue bound and these are ~40 of its
// ~120 VALU instructions.  FP64 keeps the reference's expression order
// unfused (-ffp-contract=off).
__device__ __forceinline__ float fast_exp(float x) {
    return __builtin_amdgcn_exp2f(x * 1.44269504088896341f);
}

template <typename T, int KERN>
__device__ __forceinline__ void sgd_error(T s, T bu, T bi, T r, const Hyper<T> h, T& e, T& d) {
    d = (T)1;
    if constexpr (std::is_same<T, float>::value && KERN == MF_SIGMOID) {
        const float lin = ((h.mu + bu) + bi) + s;
        const float ex = fast_exp(-lin);
        const float sg = __builtin_amdgcn_rcpf(1.0f + ex);
        e = __builtin_fmaf(h.c, sg, h.a) - r;
        d = (sg * sg) * ex;
        return;
    } else if constexpr (std::is_same<T, float>::value && KERN == MF_RBF) {
        const float E = fast_exp((-h.gamma) * s);
        e = __builtin_fmaf(h.c, E, h.a) - r;
        d = (2.0f * E) * h.gamma;
        return;
    }
    if constexpr (KERN == MF_LINEAR) {
        const T pred = ((h.mu + bi) + bu) + s;                   // kernels.py:148-153
        e = pred - r;                                            // :156
    } else if constexpr (KERN == MF_SIGMOID) {
        const T lin = ((h.mu + bu) + bi) + s;                    // kernels.py:226-228
        const T ex = dexp<T>(-lin);
        const T sg = (T)1 / ((T)1 + ex);                         // :229
        const T pred = h.a + h.c * sg;                           // :230
        e = pred - r;                                            // :233
        d = (sg * sg) * ex;                                      // :236 (no c factor)
    } else {
        const T E = dexp<T>((-h.gamma) * s);                     // kernels.py:302-303
        const T pred = h.a + h.c * E;                            // :304
        e = pred - r;                                            // :307
        d = ((T)2 * E) * h.gamma;                                // :310 (no c factor)
    }
}

// kernels.py:159-163 (linear) / :239-245 (sigmoid); rbf has no biases
template <typename T, int KERN>
__device__ __forceinline__ T sgd_bias(T b, T e, T d, const Hyper<T> h) {
    if constexpr (std::is_same<T, float>::value) {
        const float g = KERN == MF_LINEAR ? __builtin_fmaf(h.reg, b, e)
                                          : __builtin_fmaf(e, d, h.reg * b);
        return __builtin_fmaf(-h.lr, g, b);
    }
    if constexpr (KERN == MF_LINEAR) return b - h.lr * (e + h.reg * b);
    else return b - h.lr * (e * d + h.reg * b);
}

// kernels.py:166-178 / :248-260 / :313-325
template <typename T, int KERN, typename VT>
__device__ __forceinline__ void sgd_rows(VT pf, VT qf, T e, T d, const Hyper<T> h, VT& np, VT& nq) {
    if constexpr (std::is_same<T, float>::value) {
        // packed FP32 FMAs (v_pk_fma_f32 on float2 halves)
        const float ed = KERN == MF_LINEAR ? e : e * d;
        const VT nl = (VT)(-h.lr), rg = (VT)h.reg, ev = (VT)ed;
        if constexpr (KERN == MF_RBF) {
            const VT df = qf - pf;
            np = __builtin_elementwise_fma(nl, __builtin_elementwise_fma(ev, df, rg * pf), pf);
            nq = __builtin_elementwise_fma(nl, __builtin_elementwise_fma(-ev, df, rg * qf), qf);
        } else {
            np = __builtin_elementwise_fma(nl, __builtin_elementwise_fma(ev, qf, rg * pf), pf);
            nq = __builtin_elementwise_fma(nl, __builtin_elementwise_fma(ev, pf, rg * qf), qf);
        }
        return;
    }
    if constexpr (KERN == MF_LINEAR) {
        np = pf - h.lr * (e * qf + h.reg * pf);
        nq = qf - h.lr * (e * pf + h.reg * qf);
    } else if constexpr (KERN == MF_SIGMOID) {
        np = pf - h.lr * (e * (qf * d) + h.reg * pf);
        nq = qf - h.lr * (e * (pf * d) + h.reg * qf);
    } else {
        np = pf - h.lr * (e * (d * (qf - pf)) + h.reg * pf);
        nq = qf - h.lr * (e * (d * (pf - qf)) + h.reg * qf);
    }
}

// ----------------------------------------------------- tile placement
// A batch is item-sorted, so tile t of T covers item slice ~ t*8/T.  Static:
// blocks b and b+8 share an XCD (observed round-robin dealing), so the
// bijective swizzle gives every XCD a contiguous tile range -- but the XCD
// that receives block 0 changes from launch to launch.  Claiming: the block
// reads the XCD it actually runs on and takes the next tile of that XCD's
// slice from a per-launch counter (stealing from the other slices when its
// own is exhausted), so each XCD keeps revisiting the same slice of Q across
// launches.  Every tile is claimed exactly once whatever the placement:
// T blocks make T successful claims.
__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 7u;
}

__device__ __forceinline__ int64_t claim_tile(int32_t* ctr, int64_t nt) {
    __shared__ int64_t s_tile;
    if (threadIdx.x == 0) {
        const unsigned xcc = xcc_id();
        int64_t tile = -1;
        for (unsigned k = 0; k < 8 && tile < 0; ++k) {
            const unsigned x = (xcc + k) & 7u;
            const int64_t lo = nt * x / 8, hi = nt * (x + 1) / 8;
            if (hi <= lo) continue;
            const int t = atomicAdd(ctr + x, 1);
            if (t < hi - lo) tile = lo + t;
        }
        s_tile = tile;
    }
    __syncthreads();
    return s_tile;
}

// ------------------------------------------------------------- SGD batch
// Wave w applies ratings [w*RPW, (w+1)*RPW) of the batch (RPW = S*R):
//   1. lane j loads triple j and gathers b_u / b_i of rating j;
//   2. all rows of all slots are loaded;
//   3. per slot: dot product (DPP), update, predicated stores.
// No two ratings of a batch share a row, so no slot reads another's write.
template <typename T, int W, int GS, int V, int KERN, int S, int POL>
__global__ __launch_bounds__(kBlock) void k_sgd_batch(SgdArgs<T> A) {
    using VT = typename VecOf<T, W>::type;
    constexpr int R = kWave / GS;
    constexpr int RPW = S * R;
    static_assert(RPW <= kWave, "one lane per rating for the triple loads");

    constexpr bool NT = POL != 0;
    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS;
    const int l = lane % GS;
    const int64_t blk = A.claim ? claim_tile(A.claim, gridDim.x)
                      : A.swizzle ? xcd_swizzle(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t w0 = (blk * kWavesPerBlock + threadIdx.x / kWave) * RPW;
    if (w0 >= A.n) return;
    const int nw = (int)min((int64_t)RPW, A.n - w0);
    const int k = A.k;
    const int kv = k / W;
    const Hyper<T> h = A.h;

    int tu, ti;
    T tr, tbu = (T)0, tbi = (T)0;
    {
        const int64_t pos = A.off + w0 + (lane < nw ? lane : 0);
        const int64_t j = A.order ? (int64_t)A.order[pos] : pos;
        tu = ld<NT>(A.u + j);
        ti = ld<NT>(A.i + j);
        tr = ld<NT>(A.r + j);
        if constexpr (KERN != MF_RBF) {
            tbu = ld<NT>(A.Bu + tu);
            tbi = A.Bi[ti];
        }
    }

    int uu[S], ii[S];
    bool have[S];
    T rr[S];
#pragma unroll
    for (int x = 0; x < S; ++x) {
        const int idx = x * R + g;
        have[x] = idx < nw;
        const int src = have[x] ? idx : 0;
        uu[x] = take_i<GS>(tu, src);
        ii[x] = take_i<GS>(ti, src);
        rr[x] = take_f<GS>(tr, src);
    }
    VT p[S][V], q[S][V];
    if (kv > 0) {
        gather_rows<T, W, GS, V, S, POL>(A.P, uu, k, kv, l, p, A.p_bytes);
        gather_rows<T, W, GS, V, S, 0>(A.Q, ii, k, kv, l, q);
    } else {
#pragma unroll
        for (int x = 0; x < S; ++x)
#pragma unroll
            for (int v = 0; v < V; ++v) p[x][v] = q[x][v] = (VT)(T)0;
    }
    T bu[S], bi[S];
#pragma unroll
    for (int x = 0; x < S; ++x) {             // overlaps the row loads in flight
        const int src = have[x] ? x * R + g : 0;
        bu[x] = KERN != MF_RBF ? take_f<GS>(tbu, src) : (T)0;
        bi[x] = KERN != MF_RBF ? take_f<GS>(tbi, src) : (T)0;
    }

#pragma unroll
    for (int x = 0; x < S; ++x) {
        const T s = group_sum<GS>(lane_partial<T, W, V, KERN, true>(p[x], q[x]));
        T e, d;
        sgd_error<T, KERN>(s, bu[x], bi[x], rr[x], h, e, d);
        const bool lead = have[x] && l == 0;
        if constexpr (KERN != MF_RBF) {
            if (A.upd_user && lead) st<NT>(A.Bu + uu[x], sgd_bias<T, KERN>(bu[x], e, d, h));
            if (A.upd_item && lead) A.Bi[ii[x]] = sgd_bias<T, KERN>(bi[x], e, d, h);
        }
        VT* pw = reinterpret_cast<VT*>(A.P + (int64_t)uu[x] * k);
        VT* qw = reinterpret_cast<VT*>(A.Q + (int64_t)ii[x] * k);
        [[maybe_unused]] __amdgpu_buffer_rsrc_t prs;
        if constexpr (POL >= 2) prs = buf_rsrc(A.P, A.p_bytes);
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int vi = v * GS + l;
            if (!(have[x] && vi < kv)) continue;
            VT np, nq;
            sgd_rows<T, KERN>(p[x][v], q[x][v], e, d, h, np, nq);
            if constexpr (POL >= 2) {
                if (A.upd_user)
                    buf_st<kPolAux[POL].st>(
                        prs, (uint32_t)(((uint32_t)uu[x] * (uint32_t)k + (uint32_t)(vi * W)) * sizeof(T)),
                        np);
            } else {
                if (A.upd_user) st<NT>(pw + vi, np);
            }
            if (A.upd_item) qw[vi] = nq;
        }
    }
}

// -------------------------------------------------------- training SSE
// Each wave owns a contiguous run of its slice; triples arrive 64 at a time
// (lane j <-> rating j) and the next chunk's triples are in flight while the
// current chunk is consumed S*R ratings per step.  In mf_sched_slices order
// consecutive ratings share the user's P row and a slice's Q rows stay in one
// XCD's L2.
template <typename T, int W, int GS, int V, int KERN, int S>
__global__ __launch_bounds__(kBlock) void k_sse_stream(ReadArgs<T> A, SliceTab SL) {
    using VT = typename VecOf<T, W>::type;
    constexpr int R = kWave / GS;
    constexpr int STEP = S * R;
    static_assert(kWave % STEP == 0, "chunk of 64 ratings = whole steps");
    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS;
    const int l = lane % GS;
    const int k = A.k;
    const int kv = k / W;
    const Hyper<T> h = A.h;
    const SliceWave sw = slice_wave(SL);
    const int x_slice = sw.x;
    const int64_t nw_slice = sw.nw;
    const int64_t wv = sw.wv;
    const int64_t s0 = SL.off[x_slice], len = SL.off[x_slice + 1] - s0;
    const int64_t b0 = s0 + len * wv / nw_slice;
    const int64_t b1 = s0 + len * (wv + 1) / nw_slice;
    double acc = 0.0;
    if (b0 < b1) {
        auto fetch = [&](int64_t c0, int& u, int& i, T& r) {
            const int64_t j = min(c0 + lane, b1 - 1);
            u = A.u[j]; i = A.i[j]; r = A.r[j];
        };
        int nu_, ni_;
        T nr_;
        fetch(b0, nu_, ni_, nr_);
        for (int64_t c0 = b0; c0 < b1; c0 += kWave) {
            const int tu = nu_, ti = ni_;
            const T tr = nr_;
            T tbu = (T)0, tbi = (T)0;
            if constexpr (KERN != MF_RBF) { tbu = A.Bu[tu]; tbi = A.Bi[ti]; }
            const int nw = (int)min((int64_t)kWave, b1 - c0);
            if (c0 + kWave < b1) fetch(c0 + kWave, nu_, ni_, nr_);   // prefetch
            for (int t = 0; t < nw; t += STEP) {
                int uu[S], ii[S];
                bool have[S];
                T rr[S], bu[S], bi[S];
                VT p[S][V], q[S][V];
#pragma unroll
                for (int x = 0; x < S; ++x) {
                    const int idx = t + x * R + g;
                    have[x] = idx < nw;
                    const int src = have[x] ? idx : t;
                    uu[x] = take_i<GS>(tu, src);
                    ii[x] = take_i<GS>(ti, src);
                    rr[x] = take_f<GS>(tr, src);
                }
                if (kv > 0) {
                    gather_rows<T, W, GS, V, S, 0>(A.P, uu, k, kv, l, p);
                    gather_rows<T, W, GS, V, S, 0>(A.Q, ii, k, kv, l, q);
                } else {
#pragma unroll
                    for (int x = 0; x < S; ++x)
#pragma unroll
                        for (int v = 0; v < V; ++v) p[x][v] = q[x][v] = (VT)(T)0;
                }
#pragma unroll
                for (int x = 0; x < S; ++x) {
                    const int src = have[x] ? t + x * R + g : t;
                    bu[x] = take_f<GS>(tbu, src);
                    bi[x] = take_f<GS>(tbi, src);
                }
#pragma unroll
                for (int x = 0; x < S; ++x) {
                    const T sm = group_sum<GS>(lane_partial<T, W, V, KERN>(p[x], q[x]));
                    const T err = rr[x] - predict_one<T, KERN>(sm, bu[x], bi[x], h);   // :313
                    if (have[x] && l == 0) acc += (double)err * (double)err;
                }
            }
        }
    }
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

// Training SSE with user rows OWNED by lane groups (same result as
// k_sse_stream up to the order of the FP64 accumulation).  The wave's share
// of its slice is cut into R contiguous runs, one per group of GS lanes; in
// mf_sched_slices order a run is user-major (a user has ~nnz/(n_users *
// slices) consecutive ratings in a slice), so a group loads a user's P row
// and bias once per run of that user and only the item row per rating: the
// vector-memory instructions per rating drop from two row loads to one plus
// the rare user change.  Each group walks its run S ratings per step; the
// triples come in chunks of GS per group (lane l of group g holds rating
// r0 + c + l), prefetched one chunk ahead.
template <typename T, int W, int GS, int V, int KERN, int S>
__global__ __launch_bounds__(kBlock) void k_sse_owned(ReadArgs<T> A, SliceTab SL) {
    using VT = typename VecOf<T, W>::type;
    constexpr int R = kWave / GS;
    static_assert(GS % S == 0, "a chunk of GS ratings is whole steps");
    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS;
    const int l = lane % GS;
    const int k = A.k;
    const int kv = k / W;
    const Hyper<T> h = A.h;
    const SliceWave sw = slice_wave(SL);
    const int x_slice = sw.x;
    const int64_t nw_slice = sw.nw;
    const int64_t wv = sw.wv;
    const int64_t s0 = SL.off[x_slice], len = SL.off[x_slice + 1] - s0;
    const int64_t b0 = s0 + len * wv / nw_slice;
    const int64_t b1 = s0 + len * (wv + 1) / nw_slice;
    double acc = 0.0;
    if (b0 < b1) {
        const int64_t wl = b1 - b0;
        const int64_t r0 = b0 + wl * g / R, r1 = b0 + wl * (g + 1) / R;   // this group's run
        const int64_t maxrun = (wl + R - 1) / R;                          // wave-uniform trips
        const int64_t last = r1 > r0 ? r1 - 1 : b0;
        const __amdgpu_buffer_rsrc_t rp = buf_rsrc(A.P, A.p_bytes), rq = buf_rsrc(A.Q, A.q_bytes);
        const __amdgpu_buffer_rsrc_t rbu = buf_rsrc(A.Bu, A.bu_bytes), rbi = buf_rsrc(A.Bi, A.bi_bytes);
        auto fetch = [&](int64_t c, int& u, int& i, T& r) {
            const int64_t j = min(r0 + c + l, last);
            u = A.u[j]; i = A.i[j]; r = A.r[j];
        };
        int nu_, ni_;
        T nr_;
        fetch(0, nu_, ni_, nr_);
        int pu = -1;                       // user whose row is held in pp / pbu
        VT pp[V];
        T pbu = (T)0;
#pragma unroll
        for (int v = 0; v < V; ++v) pp[v] = (VT)(T)0;
        for (int64_t c = 0; c < maxrun; c += GS) {
            const int tu = nu_, ti = ni_;
            const T tr = nr_;
            if (c + GS < maxrun) fetch(c + GS, nu_, ni_, nr_);          // prefetch
#pragma unroll 1
            for (int t = 0; t < GS; t += S) {
                int uu[S], ii[S];
                T rr[S];
                bool hv[S], need[S];
#pragma unroll
                for (int x = 0; x < S; ++x) {
                    const int src = g * GS + t + x;
                    uu[x] = take_i<GS>(tu, src);
                    ii[x] = take_i<GS>(ti, src);
                    rr[x] = take_f<GS>(tr, src);
                    hv[x] = r0 + c + t + x < r1;
                }
#pragma unroll
                for (int x = 0; x < S; ++x) need[x] = uu[x] != (x == 0 ? pu : uu[x - 1]);
                // Branch-free loads: item rows for every rating, user rows as
                // buffer loads whose offset is out of range (returns 0, no
                // memory access) where the run stays on the same user.
                VT q[S][V], p[S][V];
                T bi[S], bu[S];
#pragma unroll
                for (int x = 0; x < S; ++x) {
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        const int vi = v * GS + l;
                        const int vc = vi < kv ? vi : kv - 1;
                        q[x][v] = buf_ld<0, VT>(rq, (uint32_t)(((uint32_t)ii[x] * (uint32_t)k +
                                                               (uint32_t)(vc * W)) * sizeof(T)));
                        const uint32_t po = need[x] ? (uint32_t)(((uint32_t)uu[x] * (uint32_t)k +
                                                                   (uint32_t)(vc * W)) * sizeof(T))
                                                    : 0xFFFFFFF0u;
                        // skipped by the whole wave when no group changes user
                        if (__builtin_amdgcn_ballot_w64(need[x]) != 0)
                            p[x][v] = buf_ld<0, VT>(rp, po);
                        else
                            p[x][v] = (VT)(T)0;
                    }
                    if constexpr (KERN != MF_RBF) {
                        bi[x] = buf_ld<0, T>(rbi, (uint32_t)ii[x] * (uint32_t)sizeof(T));
                        bu[x] = buf_ld<0, T>(rbu, need[x] ? (uint32_t)uu[x] * (uint32_t)sizeof(T)
                                                          : 0xFFFFFFF0u);
                    } else {
                        bi[x] = bu[x] = (T)0;
                    }
                }
                // the user row of each rating: loaded, or carried from the
                // previous rating of the run
#pragma unroll
                for (int x = 0; x < S; ++x) {
#pragma unroll
                    for (int v = 0; v < V; ++v) p[x][v] = need[x] ? p[x][v] : (x == 0 ? pp[v] : p[x - 1][v]);
                    bu[x] = need[x] ? bu[x] : (x == 0 ? pbu : bu[x - 1]);
                }
#pragma unroll
                for (int x = 0; x < S; ++x) {
                    T part = (T)0;
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        VT pv[1] = {p[x][v]}, qv[1] = {q[x][v]};
                        const T pt = lane_partial<T, W, 1, KERN>(pv, qv);
                        part += v * GS + l < kv ? pt : (T)0;
                    }
                    const T sm = group_sum<GS>(part);
                    const T err = rr[x] - predict_one<T, KERN>(sm, bu[x], bi[x], h);   // :313
                    if (hv[x] && l == 0) acc += (double)err * (double)err;
                }
#pragma unroll
                for (int v = 0; v < V; ++v) pp[v] = p[S - 1][v];
                pbu = bu[S - 1];
                pu = uu[S - 1];
            }
        }
    }
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

// Training SSE, k_sse_owned's walk with fewer VALU instructions per rating
// (the pass is VALU-issue bound: 10.4 VALU wave-instructions per rating at
// C3, PMC r02h, about 1.7 of its 2.3 ms).  Same ratings per wave, same owned
// user rows, same per-rating arithmetic and the same FP64 sum, bit for bit:
//  * row offsets as one v_mad_u32_u24 where every id < 2^24 (U24) instead of
//    the quarter-rate v_mul_lo_u32 + shift;
//  * the user row and user bias are loaded only inside the wave-uniform
//    "some group changes user" branch; no zero-fill of skipped slots (their
//    registers are never selected), one carried row instead of S copies;
//  * the dot product starts from the first product (0 + x = x up to the
//    sign of zero, which err^2 does not see); rows without a tail (k ==
//    GS V W) skip the per-vector masks;
//  * live ratings counted in int32 per step; the FP64 square-add of FP32
//    errors as one v_fma_f64 (err^2 is exact in FP64, so fma == mul + add)
//    of an error zeroed on idle slots and on non-lead lanes.
// The walk of k_sse_lean over one wave's share [b0, b1) of the evaluation
// order; returns the lane's part of the FP64 SSE (non-lead lanes: 0).
// BC (bias per chunk): the item and user biases of a chunk's GS ratings are
// loaded ONE per lane when the chunk starts (lane l holds rating c + l's) and
// handed to each rating's step by the same lane broadcast as its rating --
// instead of one wave-wide load per rating and step (S + the user-change
// loads per step: FP32 rank 64 issued as many bias loads as row loads,
// 16 + 16 per step), which cost the texture path (TA) an instruction each
// for 8 or 4 bytes.  Same values, same arithmetic, bit for bit.
template <typename T, int W, int GS, int V, int KERN, int S, bool U24, bool BC = true>
__device__ __forceinline__ double sse_lean_range(const ReadArgs<T>& A, int64_t b0, int64_t b1) {
    using VT = typename VecOf<T, W>::type;
    constexpr int R = kWave / GS;
    static_assert(GS % S == 0, "a chunk of GS ratings is whole steps");
    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS;
    const int l = lane % GS;
    const int k = A.k;
    const int kv = k / W;
    const Hyper<T> h = A.h;
    double acc = 0.0;
    if (b0 < b1) {
        const int64_t wl = b1 - b0;
        const int64_t r0 = b0 + wl * g / R, r1 = b0 + wl * (g + 1) / R;   // this group's run
        const int64_t maxrun = (wl + R - 1) / R;                          // wave-uniform trips
        const int64_t last = r1 > r0 ? r1 - 1 : b0;
        const int nrun = (int)(r1 - r0);                                  // < 2^31: one wave's share
        const __amdgpu_buffer_rsrc_t rp = buf_rsrc(A.P, A.p_bytes), rq = buf_rsrc(A.Q, A.q_bytes);
        const __amdgpu_buffer_rsrc_t rbu = buf_rsrc(A.Bu, A.bu_bytes), rbi = buf_rsrc(A.Bi, A.bi_bytes);
        const uint32_t kb = (uint32_t)k * (uint32_t)sizeof(T);
        auto row_off = [&](int id, int vc) __attribute__((always_inline)) -> uint32_t {
            const uint32_t col = (uint32_t)(vc * W) * (uint32_t)sizeof(T);
            if constexpr (U24) {
                // one full-rate instruction; written out because the compiler
                // turns __umul24 + col into a quarter-rate v_mad_u64_u32 where
                // it can bound col
                uint32_t o;
                asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(o) : "v"(id), "s"(kb), "v"(col));
                return o;
            } else {
                return (uint32_t)id * kb + col;
            }
        };
        const bool lead = l == 0;
        auto fetch = [&](int64_t c, int& u, int& i, T& r) __attribute__((always_inline)) {
            const int64_t j = min(r0 + c + l, last);
            u = A.u[j]; i = A.i[j]; r = A.r[j];
        };
        auto sweep = [&](auto full) __attribute__((always_inline)) {
            constexpr bool FULL = decltype(full)::value;
            int nu_, ni_;
            T nr_;
            fetch(0, nu_, ni_, nr_);
            int pu = -1;                   // user whose row is carried in pc / buc
            VT pc[V];
            T buc = (T)0;
#pragma unroll
            for (int v = 0; v < V; ++v) pc[v] = (VT)(T)0;
            for (int64_t c = 0; c < maxrun; c += GS) {
                const int tu = nu_, ti = ni_;
                const T tr = nr_;
                // BC: the chunk's biases, one per lane (issued before the
                // prefetch: the counter waits for them do not wait for it)
                [[maybe_unused]] T tbi = (T)0, tbu = (T)0;
                if constexpr (BC && KERN != MF_RBF) {
                    tbi = buf_ld<0, T>(rbi, (uint32_t)ti * (uint32_t)sizeof(T));
                    tbu = buf_ld<0, T>(rbu, (uint32_t)tu * (uint32_t)sizeof(T));
                }
                if (c + GS < maxrun) fetch(c + GS, nu_, ni_, nr_);      // prefetch
#pragma unroll 1
                for (int t = 0; t < GS; t += S) {
                    const int live = nrun - (int)c - t;                 // slots x < live hold a rating
                    int uu[S], ii[S];
                    T rr[S];
                    bool need[S];
#pragma unroll
                    for (int x = 0; x < S; ++x) {
                        const int src = g * GS + t + x;
                        uu[x] = take_i<GS>(tu, src);
                        ii[x] = take_i<GS>(ti, src);
                        rr[x] = take_f<GS>(tr, src);
                    }
#pragma unroll
                    for (int x = 0; x < S; ++x) need[x] = uu[x] != (x == 0 ? pu : uu[x - 1]);
                    VT q[S][V], pl[S][V];
                    T bi[S], bul[S];
#pragma unroll
                    for (int x = 0; x < S; ++x) {
#pragma unroll
                        for (int v = 0; v < V; ++v) {
                            const int vi = v * GS + l;
                            const int vc = FULL || vi < kv ? vi : kv - 1;
                            q[x][v] = buf_ld<0, VT>(rq, row_off(ii[x], vc));
                        }
                        if constexpr (KERN != MF_RBF) {
                            if constexpr (BC)
                                bi[x] = take_f<GS>(tbi, g * GS + t + x);
                            else
                                bi[x] = buf_ld<0, T>(rbi, (uint32_t)ii[x] * (uint32_t)sizeof(T));
                        }
                        // wave-uniform: skipped unless some group changes user
                        // here; a lane that keeps its user reads out of range
                        if (__builtin_amdgcn_ballot_w64(need[x]) != 0) {
#pragma unroll
                            for (int v = 0; v < V; ++v) {
                                const int vi = v * GS + l;
                                const int vc = FULL || vi < kv ? vi : kv - 1;
                                pl[x][v] = buf_ld<0, VT>(rp, need[x] ? row_off(uu[x], vc) : kBufDropRd);
                            }
                            if constexpr (KERN != MF_RBF && !BC)
                                bul[x] = buf_ld<0, T>(rbu, need[x] ? (uint32_t)uu[x] * (uint32_t)sizeof(T)
                                                                   : kBufDropRd);
                        }
                        if constexpr (KERN != MF_RBF && BC) bul[x] = take_f<GS>(tbu, g * GS + t + x);
                    }
#pragma unroll
                    for (int x = 0; x < S; ++x) {
                        // the user row of this rating: loaded, or carried
#pragma unroll
                        for (int v = 0; v < V; ++v) pc[v] = need[x] ? pl[x][v] : pc[v];
                        if constexpr (KERN != MF_RBF) buc = need[x] ? bul[x] : buc;
                        T part = (T)0;
#pragma unroll
                        for (int v = 0; v < V; ++v) {
                            VT pv[1] = {pc[v]}, qv[1] = {q[x][v]};
                            const T pt = lane_partial_first<T, W, KERN>(pv, qv);
                            const T ptm = FULL || v * GS + l < kv ? pt : (T)0;
                            part = v == 0 ? ptm : part + ptm;
                        }
                        const T sm = group_sum<GS>(part);
                        const T err = rr[x] - predict_one<T, KERN>(sm, buc, KERN != MF_RBF ? bi[x] : (T)0, h);
                        const bool on = (x < live) & lead;     // one select, no branch
                        const T e = on ? err : (T)0;
                        if constexpr (std::is_same<T, float>::value)
                            acc = __builtin_fma((double)e, (double)e, acc);     // e^2 exact in FP64
                        else
                            acc += (double)e * (double)e;
                    }
                    pu = uu[S - 1];
                }
            }
        };
        if (kv == GS * V) sweep(std::true_type{});
        else sweep(std::false_type{});
    }
    return acc;
}

__device__ __forceinline__ void sse_block_partial(double acc, double* partials) {
    acc = wave_sum(acc);
    __shared__ double red[kWavesPerBlock];
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) t += red[w];
        partials[blockIdx.x] = t;
    }
}

template <typename T, int W, int GS, int V, int KERN, int S, bool U24, bool BC = true>
__global__ __launch_bounds__(kBlock) void k_sse_lean(ReadArgs<T> A, SliceTab SL) {
    const SliceWave sw = slice_wave(SL);
    const int64_t s0 = SL.off[sw.x], len = SL.off[sw.x + 1] - s0;
    const int64_t b0 = s0 + len * sw.wv / sw.nw;
    const int64_t b1 = s0 + len * (sw.wv + 1) / sw.nw;
    sse_block_partial(sse_lean_range<T, W, GS, V, KERN, S, U24, BC>(A, b0, b1), A.partials);
}

// Training SSE over TILES walked in phases by a resident grid (the FP64
// pass; DESIGN.md section 5, "FP64 RMSE pass").  The evaluation order is
// cut into n = 8 P tiles (mf_sched_tiles: user chunk c x item slice s,
// tile c * S + s, users ascending inside a tile); phase ph = tile / 8 and
// block b walks, phase after phase, its share of tile 8 ph + (b mod 8).
// With one block per resident slot every block of an XCD (b mod 8 under
// the observed round-robin placement -- speed only) is in about the same
// phase at the same time, so the XCD's L2 serves one item slice (and one
// user chunk's rows) instead of the several a dispatch-ordered grid has in
// flight.  Same ratings per wave-share, same per-rating arithmetic and the
// same FP64 sum per lane as k_sse_lean.
template <typename T, int W, int GS, int V, int KERN, int S, bool U24>
__global__ __launch_bounds__(kBlock) void k_sse_phased(ReadArgs<T> A, SliceTab SL) {
    const int64_t per_x = gridDim.x / 8;                        // blocks per XCD
    const int64_t nw = per_x * kWavesPerBlock;
    const int64_t wv = (int64_t)(blockIdx.x / 8) * kWavesPerBlock + threadIdx.x / kWave;
    const int xb = (int)(blockIdx.x % 8);
    double acc = 0.0;
    for (int ph = 0; ph < SL.n / 8; ++ph) {
        const int x = 8 * ph + xb;
        const int64_t s0 = SL.off[x], len = SL.off[x + 1] - s0;
        acc += sse_lean_range<T, W, GS, V, KERN, S, U24>(A, s0 + len * wv / nw,
                                                          s0 + len * (wv + 1) / nw);
    }
    sse_block_partial(acc, A.partials);
}


// Training SSE, software-pipelined form of k_sse_owned (same ratings, same
// owned user rows, same per-rating arithmetic).  A group's run is cut into
// chunks of GS ratings (the triples of a chunk arrive in the group's GS
// lanes) and a chunk into Q = GS / S pieces of S ratings; the loads of piece
// j+1 are in flight while piece j is reduced (two register sets A / B used
// alternately, so no in-flight register is ever copied).  Every load is
// issued unconditionally -- the user row of a rating whose user the run
// already holds is a buffer load past the resource (kBufRowDrop: dropped, no
// memory access) -- so the compiler's waits count exactly the other set's
// loads.
constexpr uint32_t kBufRowDrop = 0xFFFFFFF0u;

template <typename T, int W, int GS, int V, int KERN, int S>
__global__ __launch_bounds__(kBlock) void k_sse_pipe(ReadArgs<T> A, SliceTab SL) {
    using VT = typename VecOf<T, W>::type;
    constexpr int R = kWave / GS;
    constexpr int Q = GS / S;
    static_assert(GS % S == 0 && Q % 2 == 0, "a chunk is an even number of pieces");
    const int lane = threadIdx.x & (kWave - 1);
    const int g = lane / GS;
    const int l = lane % GS;
    const int k = A.k;
    const int kv = k / W;
    const Hyper<T> h = A.h;
    const SliceWave sw = slice_wave(SL);
    const int x_slice = sw.x;
    const int64_t nw_slice = sw.nw;
    const int64_t wv = sw.wv;
    const int64_t s0 = SL.off[x_slice], len = SL.off[x_slice + 1] - s0;
    const int64_t b0 = s0 + len * wv / nw_slice;
    const int64_t b1 = s0 + len * (wv + 1) / nw_slice;
    double acc = 0.0;
    if (b0 < b1) {
        const int64_t wl = b1 - b0;
        const int64_t r0 = b0 + wl * g / R, r1 = b0 + wl * (g + 1) / R;   // this group's run
        const int64_t maxrun = (wl + R - 1) / R;                          // wave-uniform trips
        const int64_t last = r1 > r0 ? r1 - 1 : b0;
        const __amdgpu_buffer_rsrc_t rp = buf_rsrc(A.P, A.p_bytes), rq = buf_rsrc(A.Q, A.q_bytes);
        const __amdgpu_buffer_rsrc_t rbu = buf_rsrc(A.Bu, A.bu_bytes), rbi = buf_rsrc(A.Bi, A.bi_bytes);
        struct Tri { int u, i; T r; };
        struct Piece {
            int uu[S];
            bool hv[S], need[S];
            T rr[S], bi[S], bu[S];
            VT q[S][V], p[S][V];
        };
        auto fetch = [&](int64_t c, Tri& t) __attribute__((always_inline)) {
            const int64_t j = min(r0 + c + l, last);
            t.u = A.u[j]; t.i = A.i[j]; t.r = A.r[j];
        };
        int lastu = -1;                    // user of the last rating issued by this group
        // issue the loads of piece `pc` of the chunk at run offset c (triples tr)
        auto issue = [&](const Tri& tr, int64_t c, int pc, Piece& o) __attribute__((always_inline)) {
            int ii[S];
#pragma unroll
            for (int x = 0; x < S; ++x) {
                const int src = g * GS + pc * S + x;
                o.uu[x] = take_i<GS>(tr.u, src);
                ii[x] = take_i<GS>(tr.i, src);
                o.rr[x] = take_f<GS>(tr.r, src);
                o.hv[x] = r0 + c + pc * S + x < r1;
            }
#pragma unroll
            for (int x = 0; x < S; ++x) o.need[x] = o.uu[x] != (x == 0 ? lastu : o.uu[x - 1]);
            lastu = o.uu[S - 1];
#pragma unroll
            for (int x = 0; x < S; ++x) {
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const int vi = v * GS + l;
                    const int vc = vi < kv ? vi : kv - 1;
                    o.q[x][v] = buf_ld<0, VT>(rq, (uint32_t)(((uint32_t)ii[x] * (uint32_t)k +
                                                             (uint32_t)(vc * W)) * sizeof(T)));
                    o.p[x][v] = buf_ld<0, VT>(
                        rp, o.need[x] ? (uint32_t)(((uint32_t)o.uu[x] * (uint32_t)k +
                                                    (uint32_t)(vc * W)) * sizeof(T))
                                      : kBufRowDrop);
                }
                if constexpr (KERN != MF_RBF) {
                    o.bi[x] = buf_ld<0, T>(rbi, (uint32_t)ii[x] * (uint32_t)sizeof(T));
                    o.bu[x] = buf_ld<0, T>(rbu, o.need[x] ? (uint32_t)o.uu[x] * (uint32_t)sizeof(T)
                                                          : kBufRowDrop);
                } else {
                    o.bi[x] = o.bu[x] = (T)0;
                }
            }
        };
        VT pp[V];                          // row / bias of the run's current user
        T pbu = (T)0;
#pragma unroll
        for (int v = 0; v < V; ++v) pp[v] = (VT)(T)0;
        auto consume = [&](Piece& o) __attribute__((always_inline)) {
#pragma unroll
            for (int x = 0; x < S; ++x) {
#pragma unroll
                for (int v = 0; v < V; ++v)
                    o.p[x][v] = o.need[x] ? o.p[x][v] : (x == 0 ? pp[v] : o.p[x - 1][v]);
                o.bu[x] = o.need[x] ? o.bu[x] : (x == 0 ? pbu : o.bu[x - 1]);
            }
#pragma unroll
            for (int x = 0; x < S; ++x) {
                T part = (T)0;
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    VT pv[1] = {o.p[x][v]}, qv[1] = {o.q[x][v]};
                    const T pt = lane_partial<T, W, 1, KERN>(pv, qv);
                    part += v * GS + l < kv ? pt : (T)0;
                }
                const T sm = group_sum<GS>(part);
                const T err = o.rr[x] - predict_one<T, KERN>(sm, o.bu[x], o.bi[x], h);   // :313
                if (o.hv[x] && l == 0) acc += (double)err * (double)err;
            }
#pragma unroll
            for (int v = 0; v < V; ++v) pp[v] = o.p[S - 1][v];
            pbu = o.bu[S - 1];
        };
        Tri tc, tn;
        Piece pa, pb;
        fetch(0, tc);
        issue(tc, 0, 0, pa);
        for (int64_t c = 0; c < maxrun; c += GS) {
            fetch(c + GS, tn);             // the next chunk's triples
#pragma unroll
            for (int j = 0; j < Q; j += 2) {
                issue(tc, c, j + 1, pb);
                consume(pa);
                if (j + 2 < Q) issue(tc, c, j + 2, pa);
                else issue(tn, c + GS, 0, pa);     // past the run: clamped, hv false
                consume(pb);
            }
            tc = tn;
        }
    }
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

__global__ void k_sum_partials(const double* part, int n, double* out);

constexpr int kSseMaxBlocks = 8192;

// ------------------------------------------------ (dtype, k) -> row layout
// Calls F.template run<W, GS, V, KERN>() for dtype T.
template <typename T, typename F>
int dispatch_rows(int k, int kernel, F&& f) {
    constexpr int WV = 16 / (int)sizeof(T);           // values per 16-B access
    if (k < 0 || k > kMaxFactors) {
        set_error("n_factors=%d outside [0, %d]", k, kMaxFactors);
        return MF_ERR_INVALID;
    }
    if (kernel < MF_LINEAR || kernel > MF_RBF) {
        set_error("unknown kernel code %d", kernel);
        return MF_ERR_INVALID;
    }
#define MF_K3(W, GS, V)                                                         \
    {                                                                           \
        if (kernel == MF_LINEAR) return f.template run<W, GS, V, MF_LINEAR>();  \
        if (kernel == MF_SIGMOID) return f.template run<W, GS, V, MF_SIGMOID>();\
        return f.template run<W, GS, V, MF_RBF>();                              \
    }
    if (k > 0 && k % WV == 0 && k / WV <= 256) {
        int kvp = 1;
        while (kvp < k / WV) kvp <<= 1;
        switch (kvp) {
            case 1: MF_K3(WV, 1, 1)
            case 2: MF_K3(WV, 2, 1)
            case 4: MF_K3(WV, 4, 1)
            case 8: MF_K3(WV, 8, 1)
            case 16: MF_K3(WV, 16, 1)
            case 32: MF_K3(WV, 16, 2)
            case 64: MF_K3(WV, 16, 4)
            case 128: MF_K3(WV, 16, 8)
            case 256: MF_K3(WV, 16, 16)
            default: break;
        }
    } else {
        switch (kpad_of(k)) {
            case 16: MF_K3(1, 16, 1)
            case 32: MF_K3(1, 32, 1)
            case 64: MF_K3(1, 64, 1)
            case 128: MF_K3(1, 64, 2)
            case 256: MF_K3(1, 64, 4)
            case 512: MF_K3(1, 64, 8)
            case 1024: MF_K3(1, 64, 16)
            default: break;
        }
    }
#undef MF_K3
    set_error("internal: no row layout for n_factors=%d", k);
    return MF_ERR_INVALID;
}

// ----------------------------------------------------------- launchers
struct SgdParams {
    const int32_t* u; const int32_t* i; const void* r; const int32_t* order;
    const int64_t* offs; const int32_t* seq; int32_t nl;     // nl = launches
    double mu; void* bu; void* bi; void* P; void* Q; int32_t k; int32_t kernel;
    double gamma, lr, reg, lo, hi; int32_t uu, ui, flags;
    hipStream_t stream; double* kernel_ms;
    int32_t* claim;         // nullable: nl x 8 tile counters (zeroed here)
    int64_t n_users;
};

struct SseParams {
    const int32_t* u; const int32_t* i; const void* r; int64_t n;
    double mu; const void* bu; const void* bi; const void* P; const void* Q;
    int32_t n_users, n_items;
    int32_t k; int32_t kernel; double gamma, lo, hi;
    double* partials; double* sse_out; hipStream_t stream; SliceTab S;
    int32_t max_blocks;      // > 0: at most this many workgroups (mf_sse_capped)
};

template <typename T>
struct SgdRun {
    const SgdParams& p;

    // flags bits 8..11: experimental slot count for the rank-64 FP32 layout
    // flags bits 8..11: experimental slot count, bits 12..15: experimental
    // user-row policy (kPolAux), both for the rank-64 FP32 linear layout only
    template <int W, int GS, int V, int KERN>
    int run() {
        constexpr int SD = SlotsFor<kWave / GS, V, W>::S;
        const bool nt = (p.flags & MF_FLAG_NT_USER) != 0;
        if constexpr (std::is_same<T, float>::value && W == 4 && GS == 16 && V == 1) {
            switch ((p.flags >> 8) & 0xf) {
                case 1: return nt ? go<W, GS, V, KERN, 2, 1>() : go<W, GS, V, KERN, 2, 0>();
                case 2: return nt ? go<W, GS, V, KERN, 8, 1>() : go<W, GS, V, KERN, 8, 0>();
                case 3: return nt ? go<W, GS, V, KERN, 1, 1>() : go<W, GS, V, KERN, 1, 0>();
                default: break;
            }
            if constexpr (KERN == MF_LINEAR) {
                const int pol = (p.flags >> 12) & 0xf;
                if (pol >= 2 && (uint64_t)p.n_users * (uint64_t)p.k * sizeof(T) > 0xFFFFFFFFull) {
                    set_error("user-row policy %d needs P < 4 GiB", pol);
                    return MF_ERR_INVALID;
                }
                switch (pol) {
                    case 2: return go<W, GS, V, KERN, SD, 2>();
                    case 3: return go<W, GS, V, KERN, SD, 3>();
                    case 4: return go<W, GS, V, KERN, SD, 4>();
                    case 5: return go<W, GS, V, KERN, SD, 5>();
                    case 6: return go<W, GS, V, KERN, SD, 6>();
                    case 7: return go<W, GS, V, KERN, SD, 7>();
                    default: break;
                }
            }
        }
        return nt ? go<W, GS, V, KERN, SD, 1>() : go<W, GS, V, KERN, SD, 0>();
    }

    template <int W, int GS, int V, int KERN, int S, int POL>
    int go() {
        constexpr int RPW = S * (kWave / GS);
        SgdArgs<T> a;
        a.u = p.u; a.i = p.i; a.r = static_cast<const T*>(p.r); a.order = p.order;
        a.P = static_cast<T*>(p.P); a.Q = static_cast<T*>(p.Q);
        a.Bu = static_cast<T*>(p.bu); a.Bi = static_cast<T*>(p.bi);
        a.k = p.k; a.upd_user = p.uu; a.upd_item = p.ui;
        a.swizzle = (p.flags & MF_FLAG_XCD_SWIZZLE) ? 1 : 0;
        a.claim = nullptr;
        a.p_bytes = (uint64_t)p.n_users * (uint64_t)p.k * sizeof(T);
        a.h = make_hyper<T>(p.mu, p.lr, p.reg, p.gamma, p.lo, p.hi);
        if (p.claim) MF_HIP_CHECK(hipMemsetAsync(p.claim, 0, sizeof(int32_t) * 8 * (size_t)p.nl,
                                                 p.stream));
        // optional timing: hipEvents around every `stride`-th launch
        const int stride = std::max(1, (p.flags >> 16) & 0xff);
        std::vector<hipEvent_t> ev;
        if (p.kernel_ms) {
            ev.resize(2 * (size_t)((p.nl + stride - 1) / stride));
            for (auto& e : ev) MF_HIP_CHECK(hipEventCreate(&e));
        }
        int rc = MF_OK;
        int32_t timed = 0;
        for (int32_t s = 0; s < p.nl; ++s) {
            const int32_t b = p.seq ? p.seq[s] : s;
            a.off = p.offs[b];
            a.n = p.offs[b + 1] - p.offs[b];
            if (a.n <= 0) continue;
            const int64_t waves = (a.n + RPW - 1) / RPW;
            const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
            if (p.claim) a.claim = p.claim + 8 * (int64_t)s;
            const bool tm = p.kernel_ms && (s % stride == 0);
            if (tm) {
                hipError_t e = hipEventRecord(ev[2 * (s / stride)], p.stream);
                if (e != hipSuccess) { rc = hip_fail(e, "hipEventRecord"); break; }
            }
            hipLaunchKernelGGL((k_sgd_batch<T, W, GS, V, KERN, S, POL>), grid, dim3(kBlock), 0,
                               p.stream, a);
            if (tm) {
                hipError_t e = hipEventRecord(ev[2 * (s / stride) + 1], p.stream);
                if (e != hipSuccess) { rc = hip_fail(e, "hipEventRecord"); break; }
                ++timed;
            }
        }
        hipError_t le = hipGetLastError();
        if (rc == MF_OK && le != hipSuccess) rc = hip_fail(le, "k_sgd_batch launch");
        if (p.kernel_ms) {
            double tot = 0.0;
            if (rc == MF_OK) {
                hipError_t e = hipStreamSynchronize(p.stream);
                if (e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize");
            }
            for (int32_t s = 0; rc == MF_OK && s < p.nl; s += stride) {
                const int32_t b = p.seq ? p.seq[s] : s;
                if (p.offs[b + 1] - p.offs[b] <= 0) continue;
                float ms = 0.f;
                hipError_t e = hipEventElapsedTime(&ms, ev[2 * (s / stride)],
                                                   ev[2 * (s / stride) + 1]);
                if (e != hipSuccess) { rc = hip_fail(e, "hipEventElapsedTime"); break; }
                tot += ms;
            }
            for (auto& e : ev) (void)hipEventDestroy(e);
            if (rc == MF_OK) { p.kernel_ms[0] = tot; p.kernel_ms[1] = (double)timed; }
        }
        return rc;
    }
};

template <typename T>
struct SseRun {
    const SseParams& p;

    template <int W, int GS, int V, int KERN>
    int run() {
        constexpr int S = SlotsFor<kWave / GS, V, W>::S;
        ReadArgs<T> a;
        a.u = p.u; a.i = p.i; a.r = static_cast<const T*>(p.r);
        a.P = static_cast<const T*>(p.P); a.Q = static_cast<const T*>(p.Q);
        a.Bu = static_cast<const T*>(p.bu); a.Bi = static_cast<const T*>(p.bi);
        a.n = p.n; a.k = p.k; a.bound = 0; a.out = nullptr; a.partials = p.partials;
        a.h = make_hyper<T>(p.mu, 0.0, 0.0, p.gamma, p.lo, p.hi);
        // Up to eight workgroups per resident slot, each an equal share of
        // its slice, but at least ~6K ratings per wave: the shorter shares
        // even out the per-wave rate differences on large inputs (C3, rank
        // 64: 2.45 ms with one share per resident slot, 2.26 / 2.25 / 2.24 ms
        // with 2048 / 4096 / 8192 workgroups; tools/sse_probe.py), while on
        // small ones (C2, the N=8 shard) more workgroups only add tail
        // (0.094 -> 0.105 ms, 0.276 -> 0.286 ms at 8 per slot).
        // MF_SSE_BLOCKS overrides (probes).
        a.p_bytes = (uint64_t)p.n_users * p.k * sizeof(T);
        a.q_bytes = (uint64_t)p.n_items * p.k * sizeof(T);
        a.bu_bytes = (uint64_t)p.n_users * sizeof(T);
        a.bi_bytes = (uint64_t)p.n_items * sizeof(T);
        // k_sse_owned (default); MF_SSE_VARIANT=1 selects k_sse_stream (probes,
        // tools/sse_probe.py) and so does a P or Q too large for a buffer
        // resource.  Measured at C3 (rank 64, FP32): 2.49 vs 2.66 ms; the
        // owned kernel without the wave-uniform skip of user-row loads took
        // 2.72 ms, with non-temporal user streams 2.69 ms.
        // k_sse_lean (default; the ids-below-2^24 form where they are) and,
        // as probes (MF_SSE_VARIANT): 6 = k_sse_owned, the round-2 default.
        const char* ev = std::getenv("MF_SSE_VARIANT");
        int var = ev && std::atoi(ev) == 1 ? 1 : 0;
        if (a.p_bytes >= (1ull << 32) - 64 || a.q_bytes >= (1ull << 32) - 64) var = 1;  // buffer range
        const bool u24 = p.n_users < (1 << 24) && p.n_items < (1 << 24);
        auto kfn = var == 1 ? k_sse_stream<T, W, GS, V, KERN, S>
                 : u24      ? k_sse_lean<T, W, GS, V, KERN, S, true>
                            : k_sse_lean<T, W, GS, V, KERN, S, false>;
        if (var == 0 && ev && std::atoi(ev) == 6) { var = 6; kfn = k_sse_owned<T, W, GS, V, KERN, S>; }
        // probe: 12 = the round-5 k_sse_lean (a bias load per rating and step)
        if (var == 0 && u24 && ev && std::atoi(ev) == 12) {
            var = 12;
            kfn = k_sse_lean<T, W, GS, V, KERN, S, true, false>;
            if constexpr (GS == 16 && V == 1 && std::is_same<T, float>::value)
                kfn = k_sse_lean<T, W, GS, V, KERN, 16, true, false>;
        }
        // FP32 rows of one vector per lane (rank 64): a whole chunk of 16
        // ratings per group per step (C3: 2.45 vs 2.52 ms with S = 4, 2.46
        // with 8; tools/sse_probe.py).  Probes: 2 = 8 per step, 3 = SlotsFor.
        if constexpr (GS == 16 && V == 1 && std::is_same<T, float>::value) {
            if (var == 0) kfn = u24 ? k_sse_lean<T, W, GS, V, KERN, 16, true>
                                    : k_sse_lean<T, W, GS, V, KERN, 16, false>;
            if (var == 6) kfn = k_sse_owned<T, W, GS, V, KERN, 16>;
            if (var == 0 && u24 && ev && std::atoi(ev) == 8) { var = 8; kfn = k_sse_lean<T, W, GS, V, KERN, 8, true>; }
            if (var == 0 && u24 && ev && std::atoi(ev) == 9) { var = 9; kfn = k_sse_lean<T, W, GS, V, KERN, 4, true>; }
            if (var == 0 && ev && std::atoi(ev) == 2) { var = 2; kfn = k_sse_owned<T, W, GS, V, KERN, 8>; }
            if (var == 0 && ev && std::atoi(ev) == 3) { var = 3; kfn = k_sse_owned<T, W, GS, V, KERN, S>; }
            if (var == 0 && ev && std::atoi(ev) == 4) { var = 4; kfn = k_sse_pipe<T, W, GS, V, KERN, 8>; }
            if (var == 0 && ev && std::atoi(ev) == 5) { var = 5; kfn = k_sse_pipe<T, W, GS, V, KERN, 4>; }
        }
        // tiles walked in phases by a resident grid (mf_sched_tiles order:
        // n > 8, a multiple of 8); MF_SSE_PHASED=0 walks them as a
        // dispatch-ordered grid (slice_wave) instead
        const char* ep = std::getenv("MF_SSE_PHASED");
        const bool phased = var == 0 && p.S.n > 8 && p.S.n % 8 == 0 && !(ep && ep[0] == '0');
        if (phased) {
            var = u24 ? 10 : 11;
            kfn = u24 ? k_sse_phased<T, W, GS, V, KERN, S, true>
                      : k_sse_phased<T, W, GS, V, KERN, S, false>;
            if constexpr (GS == 16 && V == 1 && std::is_same<T, float>::value)
                kfn = u24 ? k_sse_phased<T, W, GS, V, KERN, 16, true>
                          : k_sse_phased<T, W, GS, V, KERN, 16, false>;
        }
        if (var == 0 && !u24) var = 7;                    // its own occupancy entry
        static int resident_tab[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // per instantiation and variant
        int& resident = resident_tab[var];
        if (resident == 0) {
            const LaunchTrace lt;
            int dev = 0, cus = 0, per_cu = 0;
            if (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) ==
                    hipSuccess &&
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kBlock, 0) ==
                    hipSuccess && cus > 0 && per_cu > 0)
                resident = cus * per_cu;
            else
                resident = kSseMaxBlocks;
            lt.mark("sse occupancy");
        }
        constexpr int64_t kSseRatingsPerWave = 6144;
        const int64_t by_size = p.n / (kSseRatingsPerWave * kWavesPerBlock);
        int blocks = (int)std::min<int64_t>(
            std::max<int64_t>(resident, std::min<int64_t>(by_size, 8 * (int64_t)resident)),
            kSseMaxBlocks);
        // phased: one block per resident slot (all of an XCD's blocks move
        // through the phases together)
        if (phased) blocks = std::min(resident, kSseMaxBlocks);
        if (const char* e = std::getenv("MF_SSE_BLOCKS")) {
            const int v = std::atoi(e);
            if (v > 0) blocks = std::min(v, kSseMaxBlocks);
        }
        if (p.max_blocks > 0) blocks = std::min(blocks, p.max_blocks);
        if (phased) {
            blocks = std::max(8, (blocks / 8) * 8);      // a multiple of 8
        } else {
            blocks = std::max(p.S.n, (blocks / p.S.n) * p.S.n);
        }
        const LaunchTrace lt2;
        hipLaunchKernelGGL(kfn, dim3(blocks), dim3(kBlock), 0, p.stream, a, p.S);
        hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(kBlock), 0, p.stream,
                           (const double*)p.partials, blocks, p.sse_out);
        lt2.mark("sse launches");
        MF_HIP_CHECK(hipGetLastError());
        return MF_OK;
    }
};

// defined in mf_rows_f32.hip / mf_rows_f64.hip
int sgd_launch_f32(const SgdParams& p);
int sgd_launch_f64(const SgdParams& p);
int sse_launch_f32(const SseParams& p);
int sse_launch_f64(const SseParams& p);

}  // namespace mf
