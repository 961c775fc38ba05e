// mf_strata.hpp -- the stratified SGD sweep ("strata").
//
// Users are cut into B contiguous ranges and items into B contiguous ranges;
// block (ub, ib) holds the ratings of user range ub x item range ib.  Stratum
// s is the B blocks (ub = (w + s) mod B, ib = w), w = 0..B-1: they share no
// user and no item, so one launch applies a whole stratum with workgroup w on
// block w.  The workgroup stages its item slab Q[ib] (+ b_i) and the user-bias
// slice b_u[ub] in LDS, sweeps the block's colours (conflict-free inside the
// block, mf_sched_strata) with a workgroup barrier between colours -- user
// rows P[u] gathered from / written to HBM, item rows read and written in LDS
// -- and writes the slab back.  The epoch = the B strata in a caller-chosen
// order; inside a block the colours run from a per-(seed, block) rotation.
// Every such order is a sequential order of the ratings, so the result is
// exactly the sequential sweep of that serialised order (kernels.py:108-327
// per rating, kernel_matrix_factorization.py:371-425 per epoch).
//
// Per update the HBM traffic is the user row read + write (2 * 4k B at FP32)
// and the triple; the item slab (2 * n_items * 4k B per stratum) and the
// bias slices amortise over the block's ratings.
#pragma once

#include "mf_rows.hpp"

namespace mf {

constexpr int kStrataWaves = 16;                    // 1024-thread workgroups
constexpr int kStrataThreads = kStrataWaves * kWave;
constexpr int kLdsLimit = 160 * 1024;               // gfx950 LDS per CU

template <typename T>
struct StrataArgs {
    const int32_t* u;
    const int32_t* i;
    const T* r;
    T* P;
    T* Q;
    T* Bu;
    T* Bi;
    const int32_t* ubnd;     // B + 1 user-range bounds
    const int32_t* ibnd;     // B + 1 item-range bounds
    const int64_t* boff;     // B*B + 1: block (s, w) at s*B + w
    const int32_t* cstart;   // B*B + 1: first colour offset of each block
    const int32_t* coff;     // colour offsets, relative to the block start
    int32_t B;
    int32_t s;
    uint32_t seed;
    int32_t k;
    int32_t upd_user;
    int32_t upd_item;
    Hyper<T> h;
};

// first colour of block `blk` in this epoch (mirrored by engine.strata_rotation)
__host__ __device__ inline uint32_t strata_mix(uint32_t seed, uint32_t blk) {
    uint32_t x = seed ^ (blk * 0x9E3779B9u);
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}

template <typename T>
__host__ __device__ inline size_t strata_lds_bytes(int max_items, int max_users, int k) {
    return sizeof(T) * ((size_t)max_items * (size_t)k + (size_t)max_items + (size_t)max_users);
}

template <typename T, int W, int GS, int V, int KERN, int S>
__global__ __launch_bounds__(kStrataThreads) void k_sgd_strata(StrataArgs<T> A) {
    using VT = typename VecOf<T, W>::type;
    constexpr int R = kWave / GS;
    constexpr int RPW = S * R;
    constexpr int PASS = kStrataWaves * RPW;
    static_assert(RPW <= kWave, "one lane per rating for the triple loads");
    extern __shared__ __align__(16) unsigned char smem[];

    const int B = A.B;
    const int w = blockIdx.x;
    const int ub = (w + A.s) % B;
    const int64_t blk = (int64_t)A.s * B + w;
    const int ilo = A.ibnd[w], nqi = A.ibnd[w + 1] - ilo;
    const int ulo = A.ubnd[ub], nus = A.ubnd[ub + 1] - ulo;
    const int k = A.k;
    const int kv = k / W;
    const Hyper<T> h = A.h;
    T* Qs = reinterpret_cast<T*>(smem);
    T* Bis = Qs + (size_t)nqi * k;
    T* Bus = Bis + nqi;

    // ---- stage the item slab and the bias slices (contiguous, coalesced)
    {
        const VT* src = reinterpret_cast<const VT*>(A.Q + (int64_t)ilo * k);
        VT* dst = reinterpret_cast<VT*>(Qs);
        const int nv = nqi * kv;
#pragma unroll 4
        for (int t = threadIdx.x; t < nv; t += kStrataThreads) dst[t] = src[t];
        if constexpr (KERN != MF_RBF) {
            for (int t = threadIdx.x; t < nqi; t += kStrataThreads) Bis[t] = A.Bi[ilo + t];
            for (int t = threadIdx.x; t < nus; t += kStrataThreads) Bus[t] = A.Bu[ulo + t];
        }
    }
    __syncthreads();

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int g = lane / GS;
    const int l = lane % GS;
    const int c0 = A.cstart[blk];
    const int nc = A.cstart[blk + 1] - c0 - 1;
    const int64_t base = A.boff[blk];
    int c = nc > 0 ? (int)(strata_mix(A.seed, (uint32_t)blk) % (uint32_t)nc) : 0;

    for (int cc = 0; cc < nc; ++cc) {
        const int64_t ca = base + A.coff[c0 + c], cb = base + A.coff[c0 + c + 1];
        for (int64_t p0 = ca + (int64_t)wv * RPW; p0 < cb; p0 += PASS) {
            const int nw = (int)min((int64_t)RPW, cb - p0);
            int tu, ti;
            T tr, tbu = (T)0, tbi = (T)0;
            {
                const int64_t j = p0 + (lane < nw ? lane : 0);
                tu = ld<true>(A.u + j);
                ti = ld<true>(A.i + j);
                tr = ld<true>(A.r + j);
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
                ii[x] = take_i<GS>(ti, src) - ilo;           // slab row
                rr[x] = take_f<GS>(tr, src);
            }
            VT p[S][V], q[S][V];
            if (kv > 0) {
                gather_rows<T, W, GS, V, S, 1>(A.P, uu, k, kv, l, p);
#pragma unroll
                for (int x = 0; x < S; ++x) {
                    const VT* row = reinterpret_cast<const VT*>(Qs + (size_t)ii[x] * k);
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        const int vi = v * GS + l;
                        q[x][v] = vi < kv ? row[vi] : (VT)(T)0;
                    }
                }
            } else {
#pragma unroll
                for (int x = 0; x < S; ++x)
#pragma unroll
                    for (int v = 0; v < V; ++v) p[x][v] = q[x][v] = (VT)(T)0;
            }
            if constexpr (KERN != MF_RBF) {
                tbu = Bus[tu - ulo];
                tbi = Bis[ti - ilo];
            }
            T bu[S], bi[S];
#pragma unroll
            for (int x = 0; x < S; ++x) {
                const int src = have[x] ? x * R + g : 0;
                bu[x] = KERN != MF_RBF ? take_f<GS>(tbu, src) : (T)0;
                bi[x] = KERN != MF_RBF ? take_f<GS>(tbi, src) : (T)0;
            }
#pragma unroll
            for (int x = 0; x < S; ++x) {
                const T sm = group_sum<GS>(lane_partial<T, W, V, KERN>(p[x], q[x]));
                T e, d;
                sgd_error<T, KERN>(sm, bu[x], bi[x], rr[x], h, e, d);
                const bool lead = have[x] && l == 0;
                if constexpr (KERN != MF_RBF) {
                    if (A.upd_user && lead) Bus[uu[x] - ulo] = sgd_bias<T, KERN>(bu[x], e, d, h);
                    if (A.upd_item && lead) Bis[ii[x]] = sgd_bias<T, KERN>(bi[x], e, d, h);
                }
                VT* pw = reinterpret_cast<VT*>(A.P + (int64_t)uu[x] * k);
                VT* qw = reinterpret_cast<VT*>(Qs + (size_t)ii[x] * k);
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const int vi = v * GS + l;
                    if (!(have[x] && vi < kv)) continue;
                    VT np, nq;
                    sgd_rows<T, KERN>(p[x][v], q[x][v], e, d, h, np, nq);
                    if (A.upd_user) st<true>(pw + vi, np);
                    if (A.upd_item) qw[vi] = nq;
                }
            }
        }
        if (++c == nc) c = 0;
        // The next colour may touch a user row written in this one: the
        // workgroup barrier orders the (same-CU) global stores before the
        // next loads, and the LDS slab writes before the next LDS reads.
        __syncthreads();
    }
    if (nc == 0) __syncthreads();

    // ---- write the slab and the bias slices back
    if (A.upd_item) {
        VT* dst = reinterpret_cast<VT*>(A.Q + (int64_t)ilo * k);
        const VT* src = reinterpret_cast<const VT*>(Qs);
        const int nv = nqi * kv;
#pragma unroll 4
        for (int t = threadIdx.x; t < nv; t += kStrataThreads) dst[t] = src[t];
        if constexpr (KERN != MF_RBF)
            for (int t = threadIdx.x; t < nqi; t += kStrataThreads) A.Bi[ilo + t] = Bis[t];
    }
    if constexpr (KERN != MF_RBF) {
        if (A.upd_user)
            for (int t = threadIdx.x; t < nus; t += kStrataThreads) A.Bu[ulo + t] = Bus[t];
    }
}

struct StrataParams {
    const int32_t* u; const int32_t* i; const void* r;
    const int32_t* ubnd; const int32_t* ibnd; const int64_t* boff;
    const int32_t* cstart; const int32_t* coff;
    int32_t B; int32_t max_items; int32_t max_users;
    const int32_t* seq; int32_t n_seq; uint32_t seed;
    double mu; void* bu; void* bi; void* P; void* Q; int32_t k; int32_t kernel;
    double gamma, lr, reg, lo, hi; int32_t uu, ui, flags;
    hipStream_t stream; double* kernel_ms;
};

template <typename T>
struct StrataRun {
    const StrataParams& p;

    template <int W, int GS, int V, int KERN>
    int run() {
        // two rating slots per wave: 16 waves x 8 ratings = one 128-rating
        // pass per colour at rank 64 (colours hold ~m/D ratings)
        constexpr int SD = (kWave / GS) >= 8 ? 1 : 2;
        return go<W, GS, V, KERN, SD>();
    }

    template <int W, int GS, int V, int KERN, int S>
    int go() {
        const size_t lds = strata_lds_bytes<T>(p.max_items, p.max_users, p.k);
        if (lds > (size_t)kLdsLimit) {
            set_error("strata block needs %zu B of LDS (> %d): use more blocks", lds, kLdsLimit);
            return MF_ERR_INVALID;
        }
        auto kfn = k_sgd_strata<T, W, GS, V, KERN, S>;
        MF_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        StrataArgs<T> a;
        a.u = p.u; a.i = p.i; a.r = static_cast<const T*>(p.r);
        a.P = static_cast<T*>(p.P); a.Q = static_cast<T*>(p.Q);
        a.Bu = static_cast<T*>(p.bu); a.Bi = static_cast<T*>(p.bi);
        a.ubnd = p.ubnd; a.ibnd = p.ibnd; a.boff = p.boff; a.cstart = p.cstart; a.coff = p.coff;
        a.B = p.B; a.seed = p.seed; a.k = p.k; a.upd_user = p.uu; a.upd_item = p.ui;
        a.h = make_hyper<T>(p.mu, p.lr, p.reg, p.gamma, p.lo, p.hi);
        hipEvent_t ev[2] = {nullptr, nullptr};
        if (p.kernel_ms) {
            MF_HIP_CHECK(hipEventCreate(&ev[0]));
            MF_HIP_CHECK(hipEventCreate(&ev[1]));
            MF_HIP_CHECK(hipEventRecord(ev[0], p.stream));
        }
        for (int32_t t = 0; t < p.n_seq; ++t) {
            a.s = p.seq[t];
            hipLaunchKernelGGL(kfn, dim3((unsigned)p.B), dim3(kStrataThreads), lds, p.stream, a);
        }
        hipError_t le = hipGetLastError();
        int rc = le == hipSuccess ? MF_OK : hip_fail(le, "k_sgd_strata launch");
        if (p.kernel_ms) {
            if (rc == MF_OK) {
                hipError_t e = hipEventRecord(ev[1], p.stream);
                if (e == hipSuccess) e = hipEventSynchronize(ev[1]);
                float ms = 0.f;
                if (e == hipSuccess) e = hipEventElapsedTime(&ms, ev[0], ev[1]);
                if (e != hipSuccess) rc = hip_fail(e, "strata timing");
                p.kernel_ms[0] = ms;
                p.kernel_ms[1] = (double)p.n_seq;
            }
            (void)hipEventDestroy(ev[0]);
            (void)hipEventDestroy(ev[1]);
        }
        return rc;
    }
};

// defined in mf_rows_f32.hip / mf_rows_f64.hip
int strata_launch_f32(const StrataParams& p);
int strata_launch_f64(const StrataParams& p);

}  // namespace mf
