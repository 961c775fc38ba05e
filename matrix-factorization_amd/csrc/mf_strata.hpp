// mf_strata.hpp -- the stratified SGD sweep ("strata").
//
// Users are cut into C*B contiguous ranges (C user-range classes, 1 by
// default) and items into B contiguous ranges; block (ub, ib) holds the
// ratings of user range ub x item range ib.  Stratum s (s < C*B) is the B
// blocks (ub = (s + C*w) mod C*B, ib = w), w = 0..B-1: they share no user and
// no item, so one launch applies a whole stratum with workgroup w on block w.
// Stratum s only touches the user ranges of class s mod C, so with C > 1 the
// persistent kernel cycles through the classes and every user-range hand-off
// has C - 1 whole blocks of slack (see k_sgd_strata_epoch).  The workgroup stages its item slab Q[ib] (+ b_i) and the user-bias
// slice b_u[ub] in LDS and walks the block's plan (mf_strata_sched.cpp): a
// D x NS grid, one step per row, one rating SLOT per lane group.  Every user
// of the block is owned by one slot, so a user row is only ever read and
// written by the same lanes, in program order; a step holds each item at most
// once, so the item rows in LDS need one LDS-only barrier per step.  The steps
// run from a per-(seed, block) rotation.  Every such order is a sequential
// order of the ratings, so the result is exactly the sequential sweep of that
// serialised order (kernels.py:108-327 per rating,
// kernel_matrix_factorization.py:371-425 per epoch).
//
// Software pipeline (per lane group, no global-memory barrier anywhere):
//   step t   loads the triples of step t+2 and gathers the user rows of step
//            t+1, then applies step t from registers (its rows arrived during
//            step t-1) and the LDS slab.
// A user row prefetched for step t+1 was read before step t's stores; when
// the slot's user is the same in both steps the row just computed is
// forwarded instead (the only read-after-write the prefetch can miss: older
// stores precede the load in the same lanes' program order).
//
// Per update the HBM traffic is the user row read + write (2 * 4k B at FP32)
// and the triple; the item slab (2 * n_items * 4k B per stratum) and the
// bias slices amortise over the block's ratings.
#pragma once

#include <type_traits>

#include "mf_rows.hpp"

namespace mf {

constexpr int kStrataWaves = 16;                    // 1024-thread workgroups
constexpr int kStrataThreads = kStrataWaves * kWave;
constexpr int kLdsLimit = 160 * 1024;               // gfx950 LDS per CU
// buffer offset past any resource this file builds (P < kBufDrop bytes): a
// store there is dropped by the range check, a load returns zero
constexpr uint32_t kBufDrop = 0xFFFFFFF0u;

// rating slots per lane group of one wave-instruction (16 waves x RPW slots):
// two while a lane's share of a row is small (<= 32 B of floats, 16 B of
// doubles), else one -- 1024-lane workgroups leave 128 registers per lane
// for the two pipeline stages
template <typename T, int W, int GS, int V>
constexpr int strata_group_slots() {
    constexpr int bytes = W * V * (int)sizeof(T);
    return ((kWave / GS) < 8 && bytes <= (sizeof(T) == 4 ? 32 : 16)) ? 2 : 1;
}
template <typename T, int W, int GS, int V, int NW = kStrataWaves>
constexpr int strata_slots() {
    return NW * strata_group_slots<T, W, GS, V>() * (kWave / GS);
}

template <typename T>
struct StrataArgs {
    const int32_t* u;        // plan order, NS per step; u < 0 = idle slot
    const int32_t* i;
    const T* r;
    T* P;
    T* Q;
    T* Bu;
    T* Bi;
    const int32_t* ubnd;     // B + 1 user-range bounds
    const int32_t* ibnd;     // B + 1 item-range bounds
    const int64_t* bstep;    // B*B + 1 step offsets: block (s, w) at s*B + w
    int32_t B;
    int32_t s;
    int32_t cls;             // user-range classes C (C*B user ranges)
    uint32_t seed;
    int32_t k;
    int32_t upd_user;
    int32_t upd_item;
    uint64_t p_bytes;        // bytes of P (write-through buffer stores: < 4 GiB)
    uint64_t bu_bytes;       // bytes of Bu (sc1 buffer loads of the bias slice)
    uint32_t tri_bytes;      // bytes of each triple array (WT: buffer loads; < 4 GiB)
    T* Dq;                   // nullable: delta-out mode (persistent kernel): the epoch
    T* Dbi;                  //   leaves Q / Bi untouched and writes Dq = Q' - Q, Dbi
    Hyper<T> h;
    int64_t* probe;          // nullable: persistent-kernel phase stamps (mf_strata_set_probe)
    int32_t* xtab;           // nullable: MF_FLAG_L2_HANDOFF -- per workgroup ((base+1) << 4) | XCC id
    int32_t early;           // persistent, C > 1: poll the next position's user range during
                             // the current block (0: MF_FLAG_NO_EARLY_POLL)
};

// first step of block `blk` in this epoch (mirrored by engine.strata_mix)
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

// Orders the LDS accesses of the workgroup only: global loads and stores in
// flight are not waited for (the pipeline keeps them in flight across steps).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// The steps of block `blk` (user range from ulo, item range from ilo): the
// software-pipelined sweep described at the top of this file.  Qs / Bis / Bus
// are the LDS images of the item slab, its biases and the user-bias slice.
// WT: user rows are loaded and stored with sc1 buffer ops (write-through
// stores, L1-bypassing loads), the hand-off form of the persistent kernel: no
// L2 write-back fence on the producer, no L1 invalidate on the consumer.
// BUS_IN: the block stages its user-bias slice itself (handed-off bytes, sc1
// loads), issued behind the pipeline prologue's loads so the two global-load
// latencies at the start of a block overlap (nus: users in the range).
// DEPTH: user rows gathered DEPTH steps ahead (1: rows of t+1 and triples of
// t+2 in flight while step t applies; 2: rows of t+1 and t+2, triples of t+3
// and t+4 -- for blocks of few steps, where each step otherwise waits one
// load latency).
// hook(): called once the prologue's loads are issued and consumed, before
// the first step (vmcnt counts in issue order: a load issued ahead of the
// prologue would hold up its waits).
struct StrataNoHook {
    __device__ __forceinline__ void operator()() const {}
};
template <typename T, int W, int GS, int V, int KERN, int S, bool WT = false, bool BUS_IN = false,
          int DEPTH = 1, int NW = kStrataWaves, typename Hook = StrataNoHook>
__device__ __forceinline__ void strata_block(const StrataArgs<T>& A, int64_t blk, int ulo, int ilo,
                                             T* Qs, T* Bis, T* Bus, const Hyper<T> h,
                                             int nus = 0, bool keep_l2 = false,
                                             const Hook& hook = Hook{}) {
    using VT = typename VecOf<T, W>::type;
    constexpr int R = kWave / GS;
    constexpr int RPW = S * R;
    constexpr int NS = NW * RPW;
    constexpr int TH = NW * kWave;                  // threads of the workgroup
    const int k = A.k;
    const int kv = k / W;
    [[maybe_unused]] __amdgpu_buffer_rsrc_t prs;
    if constexpr (WT) prs = buf_rsrc(A.P, A.p_bytes);
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int g = lane / GS;
    const int l = lane % GS;
    const int64_t st0 = A.bstep[blk];
    const int nst = (int)(A.bstep[blk + 1] - st0);
    const int rot = nst > 0 ? (int)(strata_mix(A.seed, (uint32_t)blk) % (uint32_t)nst) : 0;
    // position of this lane's slot in step 0 of the block
    const int64_t lpos = st0 * NS + wv * RPW + (lane < RPW ? lane : 0);
    auto pos_of = [&](int t) __attribute__((always_inline)) -> int64_t {
        int c = rot + t;
        if (c >= nst) c -= nst;
        return lpos + (int64_t)c * NS;
    };
    // WT (the persistent kernel; its launcher guarantees n_users < 2^24 and
    // the triple arrays and P below 4 GiB): row and triple offsets as 32-bit
    // values from full-rate 24-bit multiply-adds, triples by buffer loads --
    // no quarter-rate 32 / 64-bit multiplies and no 64-bit address math per
    // step (the step is VALU-issue bound where HBM is not the limit)
    [[maybe_unused]] const uint32_t kb = (uint32_t)k * (uint32_t)sizeof(T);
    [[maybe_unused]] __amdgpu_buffer_rsrc_t tru, tri, trr;
    [[maybe_unused]] uint32_t lpos_b = 0;
    if constexpr (WT) {
        tru = buf_rsrc(A.u, A.tri_bytes);
        tri = buf_rsrc(A.i, A.tri_bytes);
        trr = buf_rsrc(A.r, (uint64_t)A.tri_bytes / sizeof(int32_t) * sizeof(T));
        lpos_b = (uint32_t)lpos;
    }
    auto qrow = [&](int i) __attribute__((always_inline)) -> VT* {
        if constexpr (WT)
            return reinterpret_cast<VT*>(reinterpret_cast<char*>(Qs) + mad_u24((uint32_t)i, kb, 0u));
        else
            return reinterpret_cast<VT*>(Qs + (size_t)i * k);
    };

    // Pipeline state, two copies used alternately (the loop is unrolled by
    // two so no register holding an in-flight load is ever copied):
    //   Tri   the triple of this lane's slot for one step
    //   Rows  the broadcast ids, rating and gathered user rows of one step
    struct Tri { int u, i; T r; };
    struct Rows { int u[S], i[S]; bool have[S]; T r[S]; VT p[S][V]; };
    // Every load is issued unconditionally (past the last step: a re-read of
    // the last step, never applied): a load behind a branch would make the
    // compiler drain the whole memory counter where its result is used.
    auto load_tri = [&](int t, Tri& o) __attribute__((always_inline)) {
        if constexpr (WT) {
            int tt = t < nst ? t : nst - 1;
            int c = rot + tt;
            if (c >= nst) c -= nst;
            const uint32_t j = lpos_b + (uint32_t)c * (uint32_t)NS;     // < 2^30
            o.u = buf_ld<2, int>(tru, j * 4u);                          // nt
            o.i = buf_ld<2, int>(tri, j * 4u);
            o.r = buf_ld<2, T>(trr, j * (uint32_t)sizeof(T));
        } else {
            const int64_t j = pos_of(t < nst ? t : nst - 1);
            o.u = ld<true>(A.u + j); o.i = ld<true>(A.i + j); o.r = ld<true>(A.r + j);
        }
    };
    // slot x of lane group g <- triple lane x*R + g; idle slots point at a
    // valid row (first user of the range, slab row 0) and never store.  Row
    // tails past k are masked where the rows are used, not here: a register
    // write would wait for the load in flight.
    auto unpack_gather = [&](const Tri& tr, Rows& o, auto full) __attribute__((always_inline)) {
        constexpr bool FULL = decltype(full)::value;
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const int src = x * R + g;
            const int uv = take_i<GS>(tr.u, src);
            const int iv = take_i<GS>(tr.i, src);
            o.have[x] = uv >= 0;
            o.u[x] = o.have[x] ? uv : ulo;
            o.i[x] = o.have[x] ? iv - ilo : 0;
            o.r[x] = take_f<GS>(tr.r, src);
        }
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const VT* row = reinterpret_cast<const VT*>(A.P + (int64_t)o.u[x] * k);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int vi = v * GS + l;
                const int vc = FULL || vi < kv ? vi : kv - 1;           // kv >= 1
                if constexpr (WT)   // sc1: L2-served, never a stale L1 line
                    o.p[x][v] = buf_ld<16, VT>(
                        prs, mad_u24((uint32_t)o.u[x], kb, (uint32_t)(vc * W * (int)sizeof(T))));
                else
                    o.p[x][v] = ld<true>(row + vc);
            }
        }
    };
    int uprev[S];
    VT pprev[S][V];
#pragma unroll
    for (int x = 0; x < S; ++x) uprev[x] = -1;

    // step t: triples of t+2 -> trX, rows of t+1 (from trY) -> rwY, apply rwX.
    // full: std::true_type when the lane groups cover the row exactly
    // (k == GS V W): no tail masks.
    auto step = [&](int t, Tri& trX, Tri& trY, Rows& rwX, Rows& rwY, auto full)
                    __attribute__((always_inline)) {
        constexpr bool FULL = decltype(full)::value;
        load_tri(t + 2, trX);
        unpack_gather(trY, rwY, full);
        VT p[S][V], q[S][V];
        T bu[S], bi[S];
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const bool fwd = uprev[x] == rwX.u[x];
            const VT* row = qrow(rwX.i[x]);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int vi = v * GS + l;
                const bool in = FULL || vi < kv;
                // selects, no branch: the prefetched row is consumed on every
                // path, so the compiler can wait for exactly that load
                const VT qv = row[in ? vi : kv - 1];
                p[x][v] = in ? (fwd ? pprev[x][v] : rwX.p[x][v]) : (VT)(T)0;
                q[x][v] = in ? qv : (VT)(T)0;
            }
            if constexpr (KERN != MF_RBF) {
                bu[x] = Bus[rwX.u[x] - ulo];
                bi[x] = Bis[rwX.i[x]];
            } else {
                bu[x] = bi[x] = (T)0;
            }
        }
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const T sm = group_sum<GS>(lane_partial<T, W, V, KERN, true>(p[x], q[x]));
            T e, d;
            sgd_error<T, KERN>(sm, bu[x], bi[x], rwX.r[x], h, e, d);
            const bool lead = rwX.have[x] && l == 0;
            if constexpr (KERN != MF_RBF) {
                if (A.upd_user && lead) Bus[rwX.u[x] - ulo] = sgd_bias<T, KERN>(bu[x], e, d, h);
                if (A.upd_item && lead) Bis[rwX.i[x]] = sgd_bias<T, KERN>(bi[x], e, d, h);
            }
            VT* pw = reinterpret_cast<VT*>(A.P + (int64_t)rwX.u[x] * k);
            VT* qw = qrow(rwX.i[x]);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int vi = v * GS + l;
                VT np, nq;
                sgd_rows<T, KERN>(p[x][v], q[x][v], e, d, h, np, nq);
                pprev[x][v] = np;
                const bool ok = rwX.have[x] && (FULL || vi < kv);
                if constexpr (WT) {
                    // unconditional store; a masked lane's offset is out of
                    // range and the store is dropped -- one store per lane and
                    // step on every path keeps the vmcnt waits exact
                    const uint32_t off = (ok && A.upd_user)
                        ? mad_u24((uint32_t)rwX.u[x], kb, (uint32_t)(vi * W * (int)sizeof(T)))
                        : kBufDrop;
                    // keep_l2 (wave-uniform): the successor shares this XCD's
                    // L2 -- a plain store keeps the line there (sc1 drops it)
                    if (keep_l2) buf_st<0>(prs, off, np);
                    else buf_st<16>(prs, off, np);
                } else {
                    if (ok && A.upd_user) st<true>(pw + vi, np);
                }
                if (ok && A.upd_item) qw[vi] = nq;
            }
            uprev[x] = (rwX.have[x] && A.upd_user) ? rwX.u[x] : -1;
        }
        lds_barrier();
    };

    // DEPTH 2: the rows applied at step t were gathered at the start of step
    // t-2, before the stores of steps t-2 and t-1: forward from either.
    [[maybe_unused]] int uprev2[S];
    [[maybe_unused]] VT pprev2[S][V];
#pragma unroll
    for (int x = 0; x < S; ++x) uprev2[x] = -1;
    // step t (DEPTH 2): rows of t+2 from Tc, triples of t+4 -> Tn, apply Ra
    auto step2 = [&](int t, Tri& Tc, Tri& Tn, Rows& Ra, Rows& Rc, auto full)
                     __attribute__((always_inline)) {
        constexpr bool FULL = decltype(full)::value;
        unpack_gather(Tc, Rc, full);
        load_tri(t + 4, Tn);
        VT p[S][V], q[S][V];
        T bu[S], bi[S];
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const bool f1 = uprev[x] == Ra.u[x];
            const bool f2 = !f1 && uprev2[x] == Ra.u[x];
            const VT* row = qrow(Ra.i[x]);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int vi = v * GS + l;
                const bool in = FULL || vi < kv;
                const VT qv = row[in ? vi : kv - 1];
                p[x][v] = in ? (f1 ? pprev[x][v] : (f2 ? pprev2[x][v] : Ra.p[x][v])) : (VT)(T)0;
                q[x][v] = in ? qv : (VT)(T)0;
            }
            if constexpr (KERN != MF_RBF) {
                bu[x] = Bus[Ra.u[x] - ulo];
                bi[x] = Bis[Ra.i[x]];
            } else {
                bu[x] = bi[x] = (T)0;
            }
        }
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const T sm = group_sum<GS>(lane_partial<T, W, V, KERN, true>(p[x], q[x]));
            T e, d;
            sgd_error<T, KERN>(sm, bu[x], bi[x], Ra.r[x], h, e, d);
            const bool lead = Ra.have[x] && l == 0;
            if constexpr (KERN != MF_RBF) {
                if (A.upd_user && lead) Bus[Ra.u[x] - ulo] = sgd_bias<T, KERN>(bu[x], e, d, h);
                if (A.upd_item && lead) Bis[Ra.i[x]] = sgd_bias<T, KERN>(bi[x], e, d, h);
            }
            VT* pw = reinterpret_cast<VT*>(A.P + (int64_t)Ra.u[x] * k);
            VT* qw = qrow(Ra.i[x]);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int vi = v * GS + l;
                VT np, nq;
                sgd_rows<T, KERN>(p[x][v], q[x][v], e, d, h, np, nq);
                pprev2[x][v] = pprev[x][v];
                pprev[x][v] = np;
                const bool ok = Ra.have[x] && (FULL || vi < kv);
                if constexpr (WT) {
                    const uint32_t off = (ok && A.upd_user)
                        ? mad_u24((uint32_t)Ra.u[x], kb, (uint32_t)(vi * W * (int)sizeof(T)))
                        : kBufDrop;
                    if (keep_l2) buf_st<0>(prs, off, np);
                    else buf_st<16>(prs, off, np);
                } else {
                    if (ok && A.upd_user) st<true>(pw + vi, np);
                }
                if (ok && A.upd_item) qw[vi] = nq;
            }
            uprev2[x] = uprev[x];
            uprev[x] = (Ra.have[x] && A.upd_user) ? Ra.u[x] : -1;
        }
        lds_barrier();
    };

    Tri ta, tb;
    Rows ra, rb;
    [[maybe_unused]] Tri tc;
    [[maybe_unused]] Rows rc;
    if (nst > 0) {
        if constexpr (DEPTH == 2) {
            load_tri(0, ta);
            load_tri(1, tb);
            load_tri(2, tc);
            unpack_gather(ta, ra, std::false_type{});
            load_tri(3, ta);
            unpack_gather(tb, rb, std::false_type{});
        } else {
            load_tri(0, ta);
            load_tri(1, tb);
            unpack_gather(ta, ra, std::false_type{});
        }
    }
    if constexpr (BUS_IN && KERN != MF_RBF) {
        // all loads issued before the first LDS write waits for them.  sc1
        // BUFFER loads, not relaxed atomic loads: the same L2-served access,
        // but an atomic load here makes the compiler drain every memory
        // operation (s_waitcnt vmcnt(0)) at the top of the step loop below,
        // i.e. the row prefetch of the previous step on every second step
        // (measured in the ISA: vmcnt(5..8) instead)
        constexpr int kBu = 4;
        const __amdgpu_buffer_rsrc_t brs = buf_rsrc(A.Bu, A.bu_bytes);
        T bt[kBu];
        const int last = nus > 0 ? nus - 1 : 0;
#pragma unroll
        for (int c = 0; c < kBu; ++c) {
            const int x = (int)threadIdx.x + c * TH;
            bt[c] = buf_ld<16, T>(brs, (uint32_t)(ulo + (x < last ? x : last)) * (uint32_t)sizeof(T));
        }
        // unconditional LDS writes (lanes past the slice rewrite its last
        // entry with the value they loaded from it): a load whose register
        // is consumed only on some paths would again cost a full drain at
        // the top of the step loop
#pragma unroll
        for (int c = 0; c < kBu; ++c) {
            const int x = (int)threadIdx.x + c * TH;
            Bus[x < last ? x : last] = bt[c];
        }
        for (int x = (int)threadIdx.x + kBu * TH; x < nus; x += TH)
            Bus[x] = buf_ld<16, T>(brs, (uint32_t)(ulo + x) * (uint32_t)sizeof(T));
        lds_barrier();
    }
    hook();
    // Whole unrolled groups inside the loop, the remainder after it: a group
    // cut short inside the loop body would give the compiler a back-edge on
    // which a prefetched row is never consumed, and it then drains every
    // memory operation (vmcnt(0)) at the top of each iteration.
    if constexpr (DEPTH == 2) {
        // copies by t mod 3: rows R[t%3] applied at t; triples of t+2 in
        // T[(t+2)%3], the load of t+4 goes to T[(t+1)%3] (consumed at t-1)
        auto sweep2 = [&](auto full) __attribute__((always_inline)) {
            int t = 0;
            for (; t + 2 < nst; t += 3) {
                step2(t, tc, tb, ra, rc, full);
                step2(t + 1, ta, tc, rb, ra, full);
                step2(t + 2, tb, ta, rc, rb, full);
            }
            if (t < nst) step2(t, tc, tb, ra, rc, full);
            if (t + 1 < nst) step2(t + 1, ta, tc, rb, ra, full);
        };
        if (kv == GS * V) sweep2(std::true_type{});
        else sweep2(std::false_type{});
    } else {
        auto sweep = [&](auto full) __attribute__((always_inline)) {
            int t = 0;
            for (; t + 1 < nst; t += 2) {
                step(t, ta, tb, ra, rb, full);
                step(t + 1, tb, ta, rb, ra, full);
            }
            if (t < nst) step(t, ta, tb, ra, rb, full);
        };
        if (kv == GS * V) sweep(std::true_type{});
        else sweep(std::false_type{});
    }
}

// Stage the item slab (+ biases) of item range [ilo, ilo + nqi).
template <typename T, int W, int KERN, int TH = kStrataThreads>
__device__ __forceinline__ void strata_stage_slab(const StrataArgs<T>& A, int ilo, int nqi, T* Qs,
                                                  T* Bis) {
    using VT = typename VecOf<T, W>::type;
    const int k = A.k;
    const VT* src = reinterpret_cast<const VT*>(A.Q + (int64_t)ilo * k);
    VT* dst = reinterpret_cast<VT*>(Qs);
    const int nv = nqi * (k / W);
#pragma unroll 4
    for (int t = threadIdx.x; t < nv; t += TH) dst[t] = src[t];
    if constexpr (KERN != MF_RBF)
        for (int t = threadIdx.x; t < nqi; t += TH) Bis[t] = A.Bi[ilo + t];
}

// Write the item slab (+ biases) back.
template <typename T, int W, int KERN, int TH = kStrataThreads>
__device__ __forceinline__ void strata_store_slab(const StrataArgs<T>& A, int ilo, int nqi,
                                                  const T* Qs, const T* Bis) {
    using VT = typename VecOf<T, W>::type;
    if (!A.upd_item) return;
    const int k = A.k;
    VT* dst = reinterpret_cast<VT*>(A.Q + (int64_t)ilo * k);
    const VT* src = reinterpret_cast<const VT*>(Qs);
    const int nv = nqi * (k / W);
#pragma unroll 4
    for (int t = threadIdx.x; t < nv; t += TH) dst[t] = src[t];
    if constexpr (KERN != MF_RBF)
        for (int t = threadIdx.x; t < nqi; t += TH) A.Bi[ilo + t] = Bis[t];
}

// Delta-out end of the persistent epoch (user-sharded multi-GPU): Q and Bi
// were not written during the epoch (the slab lived in LDS), so the local
// update of this slab is LDS - global; it goes to Dq / Dbi and the replica
// stays at its start-of-epoch value for the exchange to update.
template <typename T, int W, int KERN, int TH = kStrataThreads>
__device__ __forceinline__ void strata_delta_slab(const StrataArgs<T>& A, int ilo, int nqi,
                                                  const T* Qs, const T* Bis) {
    using VT = typename VecOf<T, W>::type;
    const int k = A.k;
    const VT* q0 = reinterpret_cast<const VT*>(A.Q + (int64_t)ilo * k);
    VT* dst = reinterpret_cast<VT*>(A.Dq + (int64_t)ilo * k);
    const VT* src = reinterpret_cast<const VT*>(Qs);
    const int nv = nqi * (k / W);
#pragma unroll 4
    for (int t = threadIdx.x; t < nv; t += TH) dst[t] = src[t] - q0[t];
    if constexpr (KERN != MF_RBF)
        for (int t = threadIdx.x; t < nqi; t += TH)
            A.Dbi[ilo + t] = Bis[t] - A.Bi[ilo + t];
}

// Fallback form of delta-out (one launch per stratum writes Q as it goes):
// before the strata D holds a copy of the start values S, after them cur
// holds the new values X; this leaves cur = S, D = X - S.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_delta_swap(T* __restrict__ cur, T* __restrict__ d,
                                                       int64_t n) {
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * kBlock) {
        const T x = cur[j], s0 = d[j];
        cur[j] = s0;
        d[j] = x - s0;
    }
}

__device__ __forceinline__ Hyper<float> hyper_regs(const Hyper<float>& s) {
    // field by field: an aggregate copy of the kernel-argument struct ends up
    // in scratch once the step lambdas capture it
    Hyper<float> h;
    h.mu = s.mu; h.lr = s.lr; h.reg = s.reg; h.gamma = s.gamma;
    h.a = s.a; h.c = s.c; h.lo = s.lo; h.hi = s.hi;
    return h;
}
__device__ __forceinline__ Hyper<double> hyper_regs(const Hyper<double>& s) {
    Hyper<double> h;
    h.mu = s.mu; h.lr = s.lr; h.reg = s.reg; h.gamma = s.gamma;
    h.a = s.a; h.c = s.c; h.lo = s.lo; h.hi = s.hi;
    return h;
}

// One stratum per launch: workgroup w applies block (A.s, w).
template <typename T, int W, int GS, int V, int KERN, int S, int NW = kStrataWaves>
__global__ __launch_bounds__(NW * kWave) void k_sgd_strata(StrataArgs<T> A) {
    constexpr int TH = NW * kWave;
    extern __shared__ __align__(16) unsigned char smem[];
    const int B = A.B;
    const int w = blockIdx.x;
    const int ub = (A.s + A.cls * w) % (A.cls * B);
    const int64_t blk = (int64_t)A.s * B + w;
    const int ilo = A.ibnd[w], nqi = A.ibnd[w + 1] - ilo;
    const int ulo = A.ubnd[ub], nus = A.ubnd[ub + 1] - ulo;
    T* Qs = reinterpret_cast<T*>(smem);
    T* Bis = Qs + (size_t)nqi * A.k;
    T* Bus = Bis + nqi;
    strata_stage_slab<T, W, KERN, TH>(A, ilo, nqi, Qs, Bis);
    if constexpr (KERN != MF_RBF)
        for (int t = threadIdx.x; t < nus; t += TH) Bus[t] = A.Bu[ulo + t];
    __syncthreads();
    strata_block<T, W, GS, V, KERN, S, false, false, 1, NW>(A, blk, ulo, ilo, Qs, Bis, Bus, hyper_regs(A.h));
    __syncthreads();
    strata_store_slab<T, W, KERN, TH>(A, ilo, nqi, Qs, Bis);
    if constexpr (KERN != MF_RBF) {
        if (A.upd_user)
            for (int t = threadIdx.x; t < nus; t += TH) A.Bu[ulo + t] = Bus[t];
    }
}

// Bounded wait of the persistent kernel (~1 s of polling, then give up: the
// error flag is set and the workgroup leaves, so the grid always drains).
constexpr int64_t kStrataSpinLimit = (int64_t)1 << 24;

// The stratum order of one persistent launch travels in the kernel arguments
// (no host-to-device copy per launch): C*B strata of B <= 256 workgroups (one
// per CU) and C <= MF_STRATA_MAX_CLASSES, 16-bit entries (2 KiB).
constexpr int kStrataSeqArg = 256 * MF_STRATA_MAX_CLASSES;
struct StrataSeq { uint16_t s[kStrataSeqArg]; };

// The whole epoch in one launch (MF_FLAG_PERSISTENT): workgroup w keeps item
// slab w in LDS for every stratum and walks the strata of `seq`; before
// position t it waits until the workgroup that applied the same user range
// last, at position t - C (seq cycles through the C classes; the launcher
// checks it), w' = (w + j_t - j_{t-C}) mod B with j = seq[.] / C, has
// published done[w'] >= base + t - C + 1.  With C = 1 that is the previous
// position, so every block waits for the chain's jitter and the hand-off's
// latency; with C > 1 the user range was released C - 1 whole blocks ago.  The counters only grow (no reset per launch): every
// workgroup ends a launch at the same count, so each reads its own counter at
// the start as `base` (zeroed once with the workspace, and again whenever
// the caller clears the error word).  Hand-off (cdna_hip_programming.md Guideline 16, R1): the
// block's user rows and user-bias slice are stored write-through (sc1), every
// storing wave drains (vmcnt(0)), a barrier, one relaxed agent-scope flag
// store; the consumer polls relaxed and reads every handed-off byte with sc1
// loads (L2-served), so no fence is needed on either side.  The user rows
// cross XCDs through memory; the item slab never leaves the CU.  The result is the same sequential order as one
// launch per stratum.  All B workgroups must be co-resident: the launcher
// checks occupancy, then launches cooperatively (hipLaunchCooperativeKernel:
// the runtime refuses a grid that cannot be resident at once, and the epoch
// then runs as one launch per stratum).
template <typename T, int W, int GS, int V, int KERN, int S, int DEPTH = 1, int NW = kStrataWaves,
          bool CLS = false>
__global__ __launch_bounds__(NW * kWave) void k_sgd_strata_epoch(StrataArgs<T> A,
                                                                    const StrataSeq seq,
                                                                    int32_t n_seq, int32_t* done,
                                                                    int32_t* err) {
    constexpr int TH = NW * kWave;
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_abort, s_base, s_l2ok, s_next;
    const int B = A.B;
    const int w = blockIdx.x;
    const int ilo = A.ibnd[w], nqi = A.ibnd[w + 1] - ilo;
    if (threadIdx.x == 0) {               // this workgroup's count at the end of the last launch
        s_base = __hip_atomic_load(done + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (A.xtab) {                     // publish (launch tag, XCC id); tag != 0,
            unsigned v;                   // so a zeroed entry never looks published
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
            __hip_atomic_store(A.xtab + w, (int)((((unsigned)s_base + 1u) & 0x7FFFFFFu) << 4) |
                                               (int)(v & 0xf),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    T* Qs = reinterpret_cast<T*>(smem);
    T* Bis = Qs + (size_t)nqi * A.k;
    T* Bus = Bis + nqi;
    const Hyper<T> h = hyper_regs(A.h);
    strata_stage_slab<T, W, KERN, TH>(A, ilo, nqi, Qs, Bis);
    // probe: s_memrealtime (100 MHz) at wait start / wait end / block end /
    // signal, 4 stamps per (position t, workgroup w)
    auto stamp = [&](int t, int q) __attribute__((always_inline)) {
        if (A.probe && threadIdx.x == 0)
            A.probe[((int64_t)t * B + w) * 4 + q] = (int64_t)__builtin_amdgcn_s_memrealtime();
    };
    __syncthreads();
    const int base = s_base;
    // MF_FLAG_L2_HANDOFF: once every workgroup has published its XCC id for
    // this launch, wave 0 checks that the id depends on w mod 8 alone and that
    // the 8 residues sit on 8 different XCDs.  With the XCD-class stratum
    // order (checked by the launcher) a user range then moves between
    // workgroups of ONE XCD inside a class and visits every XCD once per
    // launch, so rows it leaves in an L2 are never read stale there.  The
    // verdict must be the same in every workgroup (a plain-storing holder
    // and a write-through successor on another XCD would race): it depends
    // only on the complete table, which every workgroup waits for; one that
    // cannot see it complete within the bounded wait fails the launch (error
    // word; the caller replays the epoch per stratum) instead of deciding alone.
    bool l2ok = false;
    if (A.xtab) {
        if (threadIdx.x < kWave) {
            const int ln = threadIdx.x;
            const int want = (int)((((unsigned)base + 1u) & 0x7FFFFFFu) << 4);
            bool ok = true;
            bool timeout = false;
            for (int64_t spins = 0;; ++spins) {          // wave-uniform
                bool all = true;
                for (int j = ln; j < B; j += kWave)
                    all &= (__hip_atomic_load(A.xtab + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                            ~0xf) == want;
                if (__builtin_amdgcn_ballot_w64(!all) == 0) break;
                if (spins > kStrataSpinLimit ||
                    __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                    timeout = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (timeout) {
                ok = false;
                if (ln == 0)
                    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (!timeout) {
                bool bad = false;
                for (int j = ln; j < B; j += kWave)
                    bad |= (__hip_atomic_load(A.xtab + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xf) !=
                           (__hip_atomic_load(A.xtab + j % 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xf);
                if (ln < 8) {
                    const int mine = __hip_atomic_load(A.xtab + ln, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT) & 0xf;
                    for (int j = 0; j < 8; ++j)
                        bad |= j != ln && (__hip_atomic_load(A.xtab + j, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT) & 0xf) == mine;
                }
                ok = __builtin_amdgcn_ballot_w64(bad) == 0;
            }
            if (ln == 0) s_l2ok = timeout ? -1 : ok ? 1 : 0;
        }
        __syncthreads();
        if (s_l2ok < 0) return;           // the launch failed: nothing applied here
        l2ok = s_l2ok != 0;
    }
    if constexpr (!CLS) {
        // one class: the next position's holder is the previous position's
        // workgroup, finishing right now -- nothing to poll early or publish
        // late; the geometry is read at the top of each position, where the
        // poll's round trip hides it (the multi-class loop below, run with
        // one class, was 1-7 % slower: same-box A/B r04y / r04z)
        const int C = A.cls;
        for (int t = 0; t < n_seq; ++t) {
            const int s = seq.s[t];
            const int ub = (s + C * w) % (C * B);
            const int ulo = A.ubnd[ub], nus = A.ubnd[ub + 1] - ulo;
            stamp(t, 0);
            if (threadIdx.x == 0) {
                int ab = 0;
                if (t >= C) {
                    // the user range's previous holder: same class, C positions back
                    const int wd = (w + s / C - (int)seq.s[t - C] / C + 2 * B) % B;
                    int64_t spins = 0;
                    while (__hip_atomic_load(done + wd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                           base + t - C + 1) {
                        __builtin_amdgcn_s_sleep(2);
                        if (++spins > kStrataSpinLimit ||
                            __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            ab = 1;
                            break;
                        }
                    }
                    // every load of handed-off bytes below is sc1: no L1 invalidate,
                    // only keep the compiler from hoisting them above the poll
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
                s_abort = ab;
            }
            __syncthreads();
            if (s_abort) return;
            stamp(t, 1);
            // the user-bias slice is staged inside the block, behind its prologue
            // the next holder of this user range, w + s_t - s_{t+1}, on this XCD
            // (same residue mod 8, B a multiple of 8): rows stored plainly stay
            // in the L2 it reads; otherwise write-through, as always
            const bool keep = l2ok && t + 1 < n_seq && ((s - (int)seq.s[t + 1]) & 7) == 0;
            strata_block<T, W, GS, V, KERN, S, true, true, DEPTH, NW>(A, (int64_t)s * B + w, ulo, ilo, Qs,
                                                                  Bis, Bus, h, nus, keep);
            __syncthreads();
            stamp(t, 2);
            if constexpr (KERN != MF_RBF) {
                if (A.upd_user)
                    for (int x = threadIdx.x; x < nus; x += TH)
                        __hip_atomic_store(A.Bu + ulo + x, Bus[x], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);     // write-through
            }
            // every storing wave drains its write-through stores, then one lane
            // signals (no L2 write-back fence: nothing handed off sits dirty in L2)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                // L2 hand-offs: rows of this range stored plainly by earlier blocks
                // on this XCD must reach memory before another XCD reads them
                if (l2ok && !keep && t + 1 < n_seq) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                __hip_atomic_store(done + w, base + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            stamp(t, 3);
        }
    } else {
        const int C = A.cls;
        // Early poll (C > 1): the next position's user range was released C - 1
        // blocks before it is needed, so its holder's counter is read ONCE,
        // during the current block (issued after the block's prologue, read at
        // its end); when that shows the range released, the next position starts
        // without the poll's round trip and its barrier.  The next position's
        // geometry (scalar loads) is read beside the current block's drain.
        const __amdgpu_buffer_rsrc_t drs = buf_rsrc(done, (uint64_t)B * sizeof(int32_t));
        // position geometry: stratum, user range, and the workgroup that held the
        // range C positions back (scalar loads; each position's are issued two
        // positions ahead, inside a block, so no wait at a block boundary meets
        // them)
        struct Geo { int s, ulo, nus, wd; };
        auto geo = [&](int t) __attribute__((always_inline)) {
            Geo g;
            g.s = seq.s[t];
            const int ub = (g.s + C * w) % (C * B);
            g.ulo = A.ubnd[ub];
            g.nus = A.ubnd[ub + 1] - g.ulo;
            g.wd = t >= C ? (w + g.s / C - (int)seq.s[t - C] / C + 2 * B) % B : 0;
            return g;
        };
        Geo gc = geo(0);
        Geo gn = n_seq > 1 ? geo(1) : gc;
        bool ready = false;                  // position t's range seen released (uniform)
        for (int t = 0; t < n_seq; ++t) {
            stamp(t, 0);
            if (!ready) {
                if (threadIdx.x == 0) {
                    int ab = 0;
                    if (t >= C) {
                        // the user range's previous holder: same class, C positions back
                        int64_t spins = 0;
                        while (__hip_atomic_load(done + gc.wd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                               base + t - C + 1) {
                            __builtin_amdgcn_s_sleep(2);
                            if (++spins > kStrataSpinLimit ||
                                __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                ab = 1;
                                break;
                            }
                        }
                        // every load of handed-off bytes below is sc1: no L1 invalidate,
                        // only keep the compiler from hoisting them above the poll
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                    s_abort = ab;
                }
                __syncthreads();
                if (s_abort) return;
            }
            stamp(t, 1);
            const bool more = t + 1 < n_seq;
            // the early poll: one sc1 buffer load of the next range's holder's
            // counter, every lane the same word, dropped (no access) when unused
            const bool ep = A.early && more && C > 1 && t + 1 >= C;
            int poll = 0;
            Geo g2 = gn;
            auto hook = [&]() __attribute__((always_inline)) {
                poll = buf_ld<16, int>(drs, ep ? (uint32_t)gn.wd * (uint32_t)sizeof(int32_t) : kBufDrop);
                if (t + 2 < n_seq) g2 = geo(t + 2);
            };
            // the user-bias slice is staged inside the block, behind its prologue
            // the next holder of this user range, w + s_t - s_{t+1}, on this XCD
            // (same residue mod 8, B a multiple of 8): rows stored plainly stay
            // in the L2 it reads; otherwise write-through, as always
            const bool keep = false;             // (the L2 hand-off needs one class)
            strata_block<T, W, GS, V, KERN, S, true, true, DEPTH, NW>(A, (int64_t)gc.s * B + w, gc.ulo, ilo,
                                                                  Qs, Bis, Bus, h, gc.nus, keep, hook);
            // lane 0 decides for the workgroup (the barrier below publishes it);
            // every wave's loads of the next range come after that barrier
            if (threadIdx.x == 0)
                s_next = A.early && more && C > 1 && (t + 1 < C || poll >= base + t + 2 - C);
            __syncthreads();
            stamp(t, 2);
            const bool rdy = s_next != 0;
            if constexpr (KERN != MF_RBF) {
                if (A.upd_user)
                    for (int x = threadIdx.x; x < gc.nus; x += TH)
                        __hip_atomic_store(A.Bu + gc.ulo + x, Bus[x], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);     // write-through
            }
            // every storing wave drains its write-through stores, then one lane
            // signals (no L2 write-back fence: nothing handed off sits dirty in L2).
            // With C > 1 a range's next holder comes C positions later, so the
            // drain and the signal are taken every D = C - 1 positions (and at the
            // last): the counter then jumps by D, each range is published at most
            // D - 1 blocks late, i.e. still before its next holder's position --
            // D - 1 of every D drains off the chain.  In between, a barrier only
            // (the next block rewrites the bias slice the stores above read).
            const int D = C > 1 ? C - 1 : 1;
            if (!more || t % D == D - 1) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0) {
                    // L2 hand-offs: rows of this range stored plainly by earlier blocks
                    // on this XCD must reach memory before another XCD reads them
                    if (l2ok && !keep && more) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    __hip_atomic_store(done + w, base + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                __syncthreads();
            }
            stamp(t, 3);
            ready = rdy;
            gc = gn;
            gn = g2;
        }
    }
    __syncthreads();
    if (A.Dq)
        strata_delta_slab<T, W, KERN, TH>(A, ilo, nqi, Qs, Bis);
    else
        strata_store_slab<T, W, KERN, TH>(A, ilo, nqi, Qs, Bis);
}

// ---------------------------------------------------------------------------
// The stream form of the multi-class persistent epoch (MF_FLAG_STREAM; C > 1,
// the depth-2 pipeline).  k_sgd_strata_epoch runs each position (block) as
// its own software pipeline: a prologue of two dependent global round trips
// (the block's triples, then its user rows) and the user-bias slice staged
// behind them, then the steps, then a drain -- at C3 with 4 classes the
// blocks are 6.45 steps long and that prologue is ~1.9 us of a 12 us
// position ("stream").  Here ONE pipeline runs through
// all positions of the launch: the triples are loaded 4 steps ahead and the
// user rows gathered 2 steps ahead across block boundaries, so the next
// block's first rows are in flight while the current block's last steps
// apply.  What a boundary still needs:
//  * the next position's user range released by its previous holder (C
//    positions back, another workgroup): polled every step from the start
//    of the current block (one sc1 load per wave, its value read two steps
//    later); the wave that has not seen it released by the step whose gathers
//    enter the next block spins there (per wave: a wave's rows are its own
//    slots', nothing else of the wave depends on other waves);
//  * the next block's user-bias slice, staged into the other of two LDS
//    slices: its sc1 loads issued with those first gathers, written to LDS
//    at the end of the next step (one barrier before the block's first
//    step); the finished slice is stored back (write-through) at the first
//    step of the following block;
//  * the hand-off: a drain (vmcnt(0)), a barrier and one flag store at the
//    end of the SECOND step of a block, publishing every position before it
//    -- taken every D = C - 1 positions as in k_sgd_strata_epoch.  A wait
//    (at step nv - 2 >= 2 of position p, for position p + 1) depends only on
//    publications made at step 1 of positions <= p by other workgroups,
//    which precede their own waits: no cycle.
// Blocks shorter than kStreamMinSteps are run with idle steps added (no
// load, no store), so the lookahead of 4 steps never crosses two
// boundaries.  Every global load and store is issued on every step (a
// dropped buffer offset when not needed) and every loaded register is
// consumed on every step, so the compiler's memory-counter waits stay exact
// (a load consumed on some paths only costs a full drain).  The same
// sequential order as k_sgd_strata_epoch (bit for bit; tests/test_gpu_strata.py).
constexpr int kStreamMinSteps = 4;

// geometry of one position (LDS table built at the start of the launch)
struct StreamGeo {
    int st0, nst, rot, nv, ulo, nus, wd;
};

template <typename T>
__host__ __device__ inline size_t strata_stream_lds_bytes(int max_items, int cap, int k, int th,
                                                          int n_seq) {
    const size_t tb = sizeof(T) * ((size_t)max_items * (size_t)k + (size_t)max_items +
                                   2 * (size_t)cap + (size_t)th);
    return ((tb + 15) / 16) * 16 + 16 * (size_t)n_seq;
}

template <typename T, int W, int GS, int V, int KERN, int S, int NW, int KB>
__global__ __launch_bounds__(NW * kWave) void k_sgd_strata_stream(StrataArgs<T> A,
                                                                     const StrataSeq seq,
                                                                     int32_t n_seq, int32_t* done,
                                                                     int32_t* err, int32_t cap) {
    using VT = typename VecOf<T, W>::type;
    constexpr int TH = NW * kWave;
    constexpr int R = kWave / GS;
    constexpr int RPW = S * R;
    constexpr int NS = NW * RPW;
    constexpr bool BIAS = KERN != MF_RBF;
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_base;
    const int B = A.B, C = A.cls;
    const int w = blockIdx.x;
    const int ilo = A.ibnd[w], nqi = A.ibnd[w + 1] - ilo;
    const int k = A.k;
    const int kv = k / W;
    T* Qs = reinterpret_cast<T*>(smem);
    T* Bis = Qs + (size_t)nqi * k;
    T* Bus = Bis + nqi;                  // two slices of `cap`, then one dummy entry per thread
    // the geometry table follows this workgroup's slab and slices (16-B
    // aligned); the launcher sized the LDS for the largest slab
    const size_t gofs = ((sizeof(T) * ((size_t)nqi * k + nqi + 2 * (size_t)cap + TH) + 15) / 16) * 16;
    int4* Geo = reinterpret_cast<int4*>(smem + gofs);
    // probe (mf_strata_set_probe): per position, in LDS during the launch
    // (no global store on the step path): s_memrealtime when the apply
    // cursor enters it, wave 0's spin time waiting for its range, the time
    // of the drain + barrier publishing before it -- copied out at the end
    uint32_t* Pr = A.probe ? reinterpret_cast<uint32_t*>(Geo + n_seq) : nullptr;
    auto now = []() __attribute__((always_inline)) {
        return (uint32_t)__builtin_amdgcn_s_memrealtime();
    };
    if (threadIdx.x == 0)
        s_base = __hip_atomic_load(done + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const Hyper<T> h = hyper_regs(A.h);
    strata_stage_slab<T, W, KERN, TH>(A, ilo, nqi, Qs, Bis);
    for (int p = threadIdx.x; p < n_seq; p += TH) {
        if (Pr) Pr[p] = Pr[n_seq + p] = Pr[2 * n_seq + p] = 0u;
        const int s = seq.s[p];
        const int64_t blk = (int64_t)s * B + w;
        const int64_t st0 = A.bstep[blk];
        const int nst = (int)(A.bstep[blk + 1] - st0);
        if (nst > 0xFFFF && err)       // (16-bit table entry: the caller replays per stratum)
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int rot = nst > 0 ? (int)(strata_mix(A.seed, (uint32_t)blk) % (uint32_t)nst) : 0;
        const int ub = (s + C * w) % (C * B);
        const int ulo = A.ubnd[ub], nus = A.ubnd[ub + 1] - ulo;
        const int wd = p >= C ? (w + s / C - (int)seq.s[p - C] / C + 2 * B) % B : 0;
        Geo[p] = make_int4((int)st0, (nst & 0xFFFF) | (rot << 16), ulo,
                           (nus & 0xFFFFFF) | (wd << 24));
    }
    __syncthreads();
    const int base = s_base;

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int g = lane / GS;
    const int l = lane % GS;
    const uint32_t lslot = (uint32_t)(wv * RPW + (lane < RPW ? lane : 0));
    const uint32_t kb = (uint32_t)k * (uint32_t)sizeof(T);
    const __amdgpu_buffer_rsrc_t prs = buf_rsrc(A.P, A.p_bytes);
    const __amdgpu_buffer_rsrc_t tru = buf_rsrc(A.u, A.tri_bytes);
    const __amdgpu_buffer_rsrc_t tri = buf_rsrc(A.i, A.tri_bytes);
    const __amdgpu_buffer_rsrc_t trr =
        buf_rsrc(A.r, (uint64_t)A.tri_bytes / sizeof(int32_t) * sizeof(T));
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t brs = buf_rsrc(A.Bu, A.bu_bytes);
    const __amdgpu_buffer_rsrc_t drs = buf_rsrc(done, (uint64_t)B * sizeof(int32_t));

    auto rfl = [](int v) __attribute__((always_inline)) { return __builtin_amdgcn_readfirstlane(v); };
    auto geo = [&](int p) __attribute__((always_inline)) {
        StreamGeo q;
        if (p < n_seq) {
            const int4 e = Geo[p];
            q.st0 = rfl(e.x);
            const uint32_t y = (uint32_t)rfl(e.y), z = (uint32_t)rfl(e.w);
            q.nst = (int)(y & 0xFFFFu);
            q.rot = (int)(y >> 16);
            q.ulo = rfl(e.z);
            q.nus = (int)(z & 0xFFFFFFu);
            q.wd = (int)(z >> 24);
        } else {
            q.st0 = q.nst = q.rot = q.ulo = q.nus = q.wd = 0;
        }
        q.nv = q.nst > kStreamMinSteps ? q.nst : kStreamMinSteps;
        return q;
    };
    // cursors: apply at (pA, jA); geometry of pA - 1, pA, pA + 1, pA + 2
    int pA = 0, jA = 0;
    StreamGeo gP = geo(n_seq);           // (empty)
    StreamGeo gA = geo(0), gN = geo(1), gNN = geo(2);
    bool relN = true;                    // position pA + 1 needs no (more) waiting
    const int D = C > 1 ? C - 1 : 1;
    int nextsig = D - 1;                 // publish after this position

    struct Tri { int u, i; T r; bool real; };
    struct Rows { int u[S], i[S]; bool have[S]; T r[S]; VT p[S][V]; };
    struct Stage { T v[KB]; bool on; };
    struct Poll { int v; int p; };

    // triples of the step `d` ahead of the apply cursor (d <= 4: at most one
    // boundary ahead, since every position has >= 4 steps)
    auto load_tri = [&](int d, Tri& o) __attribute__((always_inline)) {
        int j = jA + d;
        const bool nx = j >= gA.nv;
        if (nx) j -= gA.nv;
        const int nst = nx ? gN.nst : gA.nst;
        const int rot = nx ? gN.rot : gA.rot;
        const int st0 = nx ? gN.st0 : gA.st0;
        const bool real = j < nst;
        int c = rot + j;
        if (c >= nst) c -= nst;
        const uint32_t e = (uint32_t)(st0 + c) * (uint32_t)NS + lslot;        // < 2^30
        o.u = buf_ld<2, int>(tru, real ? e * 4u : kBufDrop);
        o.i = buf_ld<2, int>(tri, real ? e * 4u : kBufDrop);
        o.r = buf_ld<2, T>(trr, real ? e * (uint32_t)sizeof(T) : kBufDrop);
        o.real = real;
    };
    auto unpack_gather = [&](const Tri& tr, Rows& o, auto full) __attribute__((always_inline)) {
        constexpr bool FULL = decltype(full)::value;
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const int src = x * R + g;
            const int uv = take_i<GS>(tr.u, src);
            const int iv = take_i<GS>(tr.i, src);
            o.have[x] = tr.real && uv >= 0;
            o.u[x] = o.have[x] ? uv : 0;                   // idle: row 0, never stored
            o.i[x] = o.have[x] ? iv - ilo : 0;
            o.r[x] = take_f<GS>(tr.r, src);
        }
#pragma unroll
        for (int x = 0; x < S; ++x) {
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int vi = v * GS + l;
                const int vc = FULL || vi < kv ? vi : kv - 1;
                o.p[x][v] = buf_ld<16, VT>(
                    prs, mad_u24((uint32_t)o.u[x], kb, (uint32_t)(vc * W * (int)sizeof(T))));
            }
        }
    };
    auto qrow = [&](int i) __attribute__((always_inline)) -> VT* {
        return reinterpret_cast<VT*>(reinterpret_cast<char*>(Qs) + mad_u24((uint32_t)i, kb, 0u));
    };
    int uprev[S], uprev2[S];
    VT pprev[S][V], pprev2[S][V];
#pragma unroll
    for (int x = 0; x < S; ++x) uprev[x] = uprev2[x] = -1;

    // one step: rows of g+2 gathered from Tc, triples of g+4 -> Tn, apply Ra;
    // staging loads -> Sn, staged values of the last step (Sp) -> LDS; poll
    // -> Pn, the poll of two steps ago (Po) read
    auto step = [&](Tri& Tc, Tri& Tn, Rows& Ra, Rows& Rc, Stage& Sn, Stage& Sp, Poll& Pn,
                    Poll& Po, auto full) __attribute__((always_inline)) {
        constexpr bool FULL = decltype(full)::value;
        // (1) the poll issued two steps ago: next range released?
        if (!relN && Po.p == pA + 1 && rfl(Po.v) >= base + pA + 2 - C) relN = true;
        // (2) the first gathers of position pA + 1 are issued this step: its
        // user range must be released (per wave)
        const bool enter = jA + 2 == gA.nv;
        if (enter && !relN) {
            const int tgt = base + pA + 2 - C;
            const uint32_t ts0 = Pr ? now() : 0u;
            int64_t spins = 0;
            while (rfl(buf_ld<16, int>(drs, (uint32_t)gN.wd * 4u)) < tgt) {
                if (++spins > kStrataSpinLimit ||
                    __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                    if (lane == 0)
                        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            relN = true;
            if (Pr && threadIdx.x == 0) Pr[n_seq + pA + 1] = now() - ts0;
            // every load of handed-off bytes below is sc1 (no stale L1 line):
            // only keep the compiler from hoisting them above the poll
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // (3) loads, oldest first: staging of the next slice, the poll, the
        // rows of g+2, the triples of g+4
        // (each only on the steps that need it: a vector-memory instruction
        // costs the CU's address unit ~16+ cycles even with every lane
        // dropped, and a position needs its slice once, not every step)
        if constexpr (BIAS) {
            const bool on = enter && pA + 1 < n_seq;
            Sn.on = on;
            if (on) {
#pragma unroll
                for (int q = 0; q < KB; ++q) {
                    const int x = (int)threadIdx.x + q * TH;
                    Sn.v[q] = buf_ld<16, T>(brs, x < gN.nus ? (uint32_t)(gN.ulo + x) *
                                                                 (uint32_t)sizeof(T)
                                                           : kBufDrop);
                }
            }
        }
        {
            // polled at the first two steps of a position (read two steps
            // later); a range not seen released by then is waited for at
            // the step that first gathers from it
            const bool need = !relN && pA + 1 < n_seq && jA < 2;
            Pn.p = need ? pA + 1 : -1;
            if (need) Pn.v = buf_ld<16, int>(drs, (uint32_t)gN.wd * 4u);
        }
        unpack_gather(Tc, Rc, full);
        load_tri(4, Tn);
        // (4) apply the rows of this step
        const int bofs = (pA & 1) * cap - gA.ulo;
        VT p[S][V], q[S][V];
        T bu[S], bi[S];
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const bool f1 = uprev[x] == Ra.u[x];
            const bool f2 = !f1 && uprev2[x] == Ra.u[x];
            const VT* row = qrow(Ra.i[x]);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int vi = v * GS + l;
                const bool in = FULL || vi < kv;
                const VT qv = row[in ? vi : kv - 1];
                p[x][v] = in ? (f1 ? pprev[x][v] : (f2 ? pprev2[x][v] : Ra.p[x][v])) : (VT)(T)0;
                q[x][v] = in ? qv : (VT)(T)0;
            }
            if constexpr (BIAS) {
                bu[x] = Bus[Ra.have[x] ? Ra.u[x] + bofs : 0];
                bi[x] = Bis[Ra.i[x]];
            } else {
                bu[x] = bi[x] = (T)0;
            }
        }
#pragma unroll
        for (int x = 0; x < S; ++x) {
            const T sm = group_sum<GS>(lane_partial<T, W, V, KERN, true>(p[x], q[x]));
            T e, d;
            sgd_error<T, KERN>(sm, bu[x], bi[x], Ra.r[x], h, e, d);
            const bool lead = Ra.have[x] && l == 0;
            if constexpr (BIAS) {
                if (A.upd_user && lead) Bus[Ra.u[x] + bofs] = sgd_bias<T, KERN>(bu[x], e, d, h);
                if (A.upd_item && lead) Bis[Ra.i[x]] = sgd_bias<T, KERN>(bi[x], e, d, h);
            }
            VT* qw = qrow(Ra.i[x]);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int vi = v * GS + l;
                VT np, nq;
                sgd_rows<T, KERN>(p[x][v], q[x][v], e, d, h, np, nq);
                pprev2[x][v] = pprev[x][v];
                pprev[x][v] = np;
                const bool ok = Ra.have[x] && (FULL || vi < kv);
                const uint32_t off = (ok && A.upd_user)
                    ? mad_u24((uint32_t)Ra.u[x], kb, (uint32_t)(vi * W * (int)sizeof(T)))
                    : kBufDrop;
                buf_st<16>(prs, off, np);
                if (ok && A.upd_item) qw[vi] = nq;
            }
            uprev2[x] = uprev[x];
            uprev[x] = (Ra.have[x] && A.upd_user) ? Ra.u[x] : -1;
        }
        if constexpr (BIAS) {
            // (5) the previous position's slice back to memory (write-through),
            // at the first step of this one
            const bool wb = jA == 0 && pA >= 1 && pA < n_seq && A.upd_user;
            const int sb = ((pA + 1) & 1) * cap;           // = slice of pA - 1
            if (wb) {
#pragma unroll
                for (int q2 = 0; q2 < KB; ++q2) {
                    const int x = (int)threadIdx.x + q2 * TH;
                    const T v = Bus[sb + (x < cap ? x : cap - 1)];
                    buf_st<16>(brs, x < gP.nus ? (uint32_t)(gP.ulo + x) * (uint32_t)sizeof(T)
                                               : kBufDrop, v);
                }
            }
            // (6) the slice staged last step into the next position's LDS slice
            const int nb = ((pA + 1) & 1) * cap;
            if (Sp.on) {
#pragma unroll
                for (int q2 = 0; q2 < KB; ++q2) {
                    const int x = (int)threadIdx.x + q2 * TH;
                    if (x < cap) Bus[nb + x] = Sp.v[q2];
                }
            }
        }
        lds_barrier();
        // (7) publish: every position before pA is complete (its rows were
        // stored before this point, its bias slice at step 0)
        if (jA == 1 && pA >= 1 && pA < n_seq && pA - 1 == nextsig) {
            nextsig += D;
            const uint32_t td0 = Pr ? now() : 0u;
            __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)
            __syncthreads();
            if (Pr && threadIdx.x == 0) Pr[2 * n_seq + pA] = now() - td0;
            if (threadIdx.x == 0)
                __hip_atomic_store(done + w, base + pA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // (8) advance the apply cursor
        if (++jA == gA.nv) {
            ++pA;
            jA = 0;
            gP = gA;
            gA = gN;
            gN = gNN;
            gNN = geo(pA + 2);
            relN = pA + 1 < C || pA + 1 >= n_seq;
            if (Pr && threadIdx.x == 0 && pA < n_seq) Pr[pA] = now();
        }
    };

    // prologue: position 0's bias slice staged; triples of steps 0..3, rows
    // of steps 0 and 1
    Tri ta, tb, tc;
    Rows ra, rb, rc;
    Stage sa, sb, sc;
    Poll pa, pb, pc;
    sa.on = sb.on = sc.on = false;
    pa.p = pb.p = pc.p = -1;
#pragma unroll
    for (int q = 0; q < KB; ++q) sa.v[q] = sb.v[q] = sc.v[q] = (T)0;
    pa.v = pb.v = pc.v = 0;
    load_tri(0, ta);
    load_tri(1, tb);
    load_tri(2, tc);
    unpack_gather(ta, ra, std::false_type{});
    load_tri(3, ta);
    unpack_gather(tb, rb, std::false_type{});
    if constexpr (BIAS) {
        if (n_seq > 0)
            for (int x = threadIdx.x; x < gA.nus; x += TH)
                Bus[x] = buf_ld<16, T>(brs, (uint32_t)(gA.ulo + x) * (uint32_t)sizeof(T));
    }
    lds_barrier();
    if (Pr && threadIdx.x == 0 && n_seq > 0) Pr[0] = now();
    auto run = [&](auto full) __attribute__((always_inline)) {
        // copies by step mod 3 (no register with a load in flight is copied):
        // step s applies R[s%3], gathers rows of s+2 from T[(s+2)%3] into
        // R[(s+2)%3], loads triples of s+4 into T[(s+1)%3], stages into
        // S[s%3] and writes S[(s+2)%3], polls into P[s%3] and reads P[(s+1)%3]
        while (pA < n_seq) {
            step(tc, tb, ra, rc, sa, sc, pa, pb, full);
            step(ta, tc, rb, ra, sb, sa, pb, pc, full);
            step(tb, ta, rc, rb, sc, sb, pc, pa, full);
        }
    };
    if (kv == GS * V) run(std::true_type{});
    else run(std::false_type{});
    // epilogue: the last position's slice back, then publish the launch's end
    if constexpr (BIAS) {
        if (n_seq > 0 && A.upd_user) {
            const StreamGeo gl = geo(n_seq - 1);
            const int sb = ((n_seq - 1) & 1) * cap;
            for (int x = threadIdx.x; x < gl.nus; x += TH)
                buf_st<16>(brs, (uint32_t)(gl.ulo + x) * (uint32_t)sizeof(T), Bus[sb + x]);
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(done + w, base + n_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (Pr) {
        const uint32_t tend = now();
        for (int p = threadIdx.x; p < n_seq; p += TH) {
            int64_t* o = A.probe + ((int64_t)p * B + w) * 4;
            o[0] = Pr[p];
            o[1] = Pr[n_seq + p];
            o[2] = Pr[2 * n_seq + p];
            o[3] = tend;
        }
    }
    if (A.Dq)
        strata_delta_slab<T, W, KERN, TH>(A, ilo, nqi, Qs, Bis);
    else
        strata_store_slab<T, W, KERN, TH>(A, ilo, nqi, Qs, Bis);
}

// Is `seq` an XCD-class order (engine.stratum_order "xcd"): B a multiple of
// 8 and the strata of each class s mod 8 one contiguous run, every class
// once?  Then a user range's holder changes XCD only between runs and meets
// each XCD in one run (MF_FLAG_L2_HANDOFF needs exactly that).
inline bool strata_xcd_classes(const int32_t* seq, int32_t n_seq, int32_t B) {
    if (B % 8 != 0 || B < 16 || n_seq < 1) return false;
    bool seen[8] = {false, false, false, false, false, false, false, false};
    int cur = -1;
    for (int32_t t = 0; t < n_seq; ++t) {
        const int c = ((seq[t] % 8) + 8) % 8;
        if (c != cur) {
            if (seen[c]) return false;
            seen[c] = true;
            cur = c;
        }
    }
    return true;
}

// user-range classes C from the flags (bits 24..27 = C - 1)
inline int strata_classes(int32_t flags) {
    return (int)(((uint32_t)flags >> MF_FLAG_CLASSES_SHIFT) & 0xFu) + 1;
}

// Does `seq` cycle through the C classes (seq[t] mod C == seq[t mod C] mod C,
// the first C of distinct classes)?  Then the user range of position t was
// last used at t - C, which is what the persistent kernel waits for.
inline bool strata_class_cycle(const int32_t* seq, int32_t n_seq, int C) {
    if (C == 1) return true;
    bool seen[MF_STRATA_MAX_CLASSES] = {};
    for (int32_t t = 0; t < n_seq && t < C; ++t) {
        const int c = seq[t] % C;
        if (seen[c]) return false;
        seen[c] = true;
    }
    for (int32_t t = C; t < n_seq; ++t)
        if (seq[t] % C != seq[t % C] % C) return false;
    return true;
}

// diagnostic: device buffer for the persistent kernel's phase stamps
// (mf_strata_set_probe; 4 * n_seq * B int64), nullptr = off
int64_t* strata_probe_ptr();

struct StrataParams {
    const int32_t* u; const int32_t* i; const void* r;
    const int32_t* ubnd; const int32_t* ibnd; const int64_t* bstep;
    int32_t B; int32_t n_slots; int32_t max_items; int32_t max_users;
    const int32_t* seq; int32_t n_seq; uint32_t seed;
    double mu; void* bu; void* bi; void* P; void* Q; int32_t k; int32_t kernel;
    double gamma, lr, reg, lo, hi; int32_t uu, ui, flags;
    void* ws; size_t ws_bytes; int64_t n_users;
    hipStream_t stream; double* kernel_ms;
    int64_t n_items; void* dq; void* dbi;    // delta-out (nullable)
    int64_t n_positions;                     // entries of each triple array
};

// workspace of the persistent kernel (int32): done[B] (position counters,
// growing across launches), err, then n_seq words no longer used (the
// stratum order travels in the kernel arguments; the size is kept for the ABI)
inline size_t strata_ws_bytes(int32_t B, int32_t n_seq) {
    return sizeof(int32_t) * ((size_t)B + 1 + (size_t)n_seq);
}

// Fault-injection hook for the callers' recovery paths (tests only,
// mf_strata_inject_fail): the next n persistent launches of this process
// start with the error word set, as if a neighbour wait had timed out
// (workgroups that poll see it and leave; the word stays set, so the caller
// must detect the failure and recover exactly as after a real timeout).
// True (and one fewer left) if this launch is one of them.
bool strata_inject_fail();

// Can all B workgroups of `kfn` be resident at once (the persistent kernel's
// waits need it)?
inline bool strata_coresident(const void* kfn, int B, size_t lds, int threads) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, threads, lds) !=
        hipSuccess)
        return false;
    return (int64_t)cus * per_cu >= B;
}

// NS of the row layout (W, GS, V) that dispatch_rows picks for (k, dtype)
// Workgroup sizes of the strata kernels: 16 waves (the default), and 8 waves
// for plans whose blocks are bound by the item degree rather than by the slot
// count -- half the slots per step, half the per-step VALU of a CU, about the
// same number of steps (C2: DESIGN.md section 5).  The 8-wave kernels exist
// for rows of one vector per lane (FP32 k <= 64, FP64 k <= 32) and for FP64
// rows of two (k <= 64) -- FP64 since round 4: C2 in FP64 filled 54 % of the
// 16-wave plan's slots, C3 with 4 user-range classes 65 %.
template <typename T, int V>
constexpr bool strata_has_8_waves() {
    return V == 1 || (std::is_same<T, double>::value && V == 2);
}

// the narrow form (MF_FLAG_NARROW): 4 waves whose lane groups are half as
// wide, two vectors per lane -- the 8-wave kernel's slot count on half the
// waves, i.e. fewer instructions per slot and step (the dot product's group
// sum one DPP level shorter, the sigmoid / bias / address work per slot
// spread over half the lanes).  FP32 rows of one vector per lane whose slot
// count matches (k <= 32 here).
template <typename T, int W, int GS, int V>
constexpr bool strata_has_narrow() {
    if constexpr (!std::is_same<T, float>::value || !strata_has_8_waves<T, V>() || GS < 2)
        return false;
    else return strata_slots<T, W, GS / 2, 2 * V, 4>() == strata_slots<T, W, GS, V, 8>();
}

template <typename T>
struct StrataSlots {
    int waves;
    template <int W, int GS, int V, int KERN>
    int run() {
        if (waves == 16) return strata_slots<T, W, GS, V, 16>();
        if constexpr (strata_has_8_waves<T, V>())
            if (waves == 8) return strata_slots<T, W, GS, V, 8>();
        if constexpr (strata_has_narrow<T, W, GS, V>())
            if (waves == 4) return strata_slots<T, W, GS / 2, 2 * V, 4>();
        return -1;
    }
};

template <typename T>
struct StrataRun {
    const StrataParams& p;

    template <int W, int GS, int V, int KERN>
    int run() {
        constexpr int S = strata_group_slots<T, W, GS, V>();
        if (p.n_slots == strata_slots<T, W, GS, V, 16>()) return go<W, GS, V, KERN, S, 16>();
        if constexpr (strata_has_8_waves<T, V>()) {
            if (p.n_slots == strata_slots<T, W, GS, V, 8>()) {
                if constexpr (strata_has_narrow<T, W, GS, V>()) {
                    if (p.flags & MF_FLAG_NARROW) {
                        constexpr int GS2 = GS / 2, V2 = 2 * V;
                        return go<W, GS2, V2, KERN, strata_group_slots<T, W, GS2, V2>(), 4>();
                    }
                }
                return go<W, GS, V, KERN, S, 8>();
            }
        }
        set_error("plan has %d slots per step, the n_factors=%d layout needs %d (16 waves)%s",
                  p.n_slots, p.k, strata_slots<T, W, GS, V, 16>(),
                  strata_has_8_waves<T, V>() ? " or half that (8 waves)" : "");
        return MF_ERR_INVALID;
    }

    template <int W, int GS, int V, int KERN, int S, int NW>
    int go() {
        constexpr int TH = NW * kWave;
        const size_t lds = strata_lds_bytes<T>(p.max_items, p.max_users, p.k);
        if (lds > (size_t)kLdsLimit) {
            set_error("strata block needs %zu B of LDS (> %d): use more blocks", lds, kLdsLimit);
            return MF_ERR_INVALID;
        }
        if (p.k < 1) {
            set_error("the strata schedule needs n_factors >= 1");
            return MF_ERR_INVALID;
        }
        auto kfn = k_sgd_strata<T, W, GS, V, KERN, S, NW>;
        MF_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        StrataArgs<T> a;
        a.u = p.u; a.i = p.i; a.r = static_cast<const T*>(p.r);
        a.P = static_cast<T*>(p.P); a.Q = static_cast<T*>(p.Q);
        a.Bu = static_cast<T*>(p.bu); a.Bi = static_cast<T*>(p.bi);
        a.ubnd = p.ubnd; a.ibnd = p.ibnd; a.bstep = p.bstep;
        a.B = p.B; a.seed = p.seed; a.k = p.k; a.upd_user = p.uu; a.upd_item = p.ui;
        a.cls = strata_classes(p.flags);
        if (a.cls < 1 || a.cls > MF_STRATA_MAX_CLASSES) {
            set_error("user-range classes %d outside [1, %d]", a.cls, MF_STRATA_MAX_CLASSES);
            return MF_ERR_INVALID;
        }
        for (int32_t t = 0; t < p.n_seq; ++t)
            if (p.seq[t] < 0 || p.seq[t] >= a.cls * p.B) {
                set_error("stratum %d outside [0, %d)", p.seq[t], a.cls * p.B);
                return MF_ERR_INVALID;
            }
        a.p_bytes = (uint64_t)p.n_users * (uint64_t)p.k * sizeof(T);
        a.bu_bytes = (uint64_t)p.n_users * sizeof(T);
        // the persistent kernel's 32-bit offsets (strata_block, WT): user ids
        // and k * sizeof(T) below 2^24, P and the triple arrays below 4 GiB
        const uint64_t tri_bytes = (uint64_t)p.n_positions * std::max<uint64_t>(4, sizeof(T));
        a.tri_bytes = (uint32_t)std::min<uint64_t>((uint64_t)p.n_positions * 4, 0xFFFFFFFFull);
        const bool u32_ok = p.n_users < (1 << 24) && (uint64_t)p.k * sizeof(T) < (1u << 24) &&
                            tri_bytes < (uint64_t)kBufDrop;
        a.Dq = static_cast<T*>(p.dq);
        a.Dbi = static_cast<T*>(p.dbi);
        if (p.dq && !p.dbi && KERN != MF_RBF) {
            set_error("delta-out needs both the item-row and the item-bias delta buffers");
            return MF_ERR_INVALID;
        }
        a.h = make_hyper<T>(p.mu, p.lr, p.reg, p.gamma, p.lo, p.hi);
        a.probe = strata_probe_ptr();
        a.xtab = nullptr;
        a.early = (p.flags & MF_FLAG_NO_EARLY_POLL) ? 0 : 1;
        hipEvent_t ev[2] = {nullptr, nullptr};
        if (p.kernel_ms && !(p.flags & MF_FLAG_PREPARE)) {
            MF_HIP_CHECK(hipEventCreate(&ev[0]));
            MF_HIP_CHECK(hipEventCreate(&ev[1]));
            MF_HIP_CHECK(hipEventRecord(ev[0], p.stream));
        }
        bool persistent = false;
        if ((p.flags & MF_FLAG_PERSISTENT) && p.ws && p.n_seq <= kStrataSeqArg && u32_ok &&
            p.ws_bytes >= strata_ws_bytes(p.B, p.n_seq) && a.p_bytes < (uint64_t)kBufDrop &&
            strata_class_cycle(p.seq, p.n_seq, a.cls)) {
            // (the deep pipeline exists for the 16- and 8-wave kernels)
            constexpr int kDeep = NW >= 8 ? 2 : 1;
            // (user-range classes C > 1: the loop that polls the next range
            // during the current block and publishes every C - 1 positions)
            const bool deep = kDeep == 2 && (p.flags & MF_FLAG_DEEP_PIPE);
            auto efn = a.cls > 1
                           ? (deep ? k_sgd_strata_epoch<T, W, GS, V, KERN, S, kDeep, NW, true>
                                   : k_sgd_strata_epoch<T, W, GS, V, KERN, S, 1, NW, true>)
                           : (deep ? k_sgd_strata_epoch<T, W, GS, V, KERN, S, kDeep, NW, false>
                                   : k_sgd_strata_epoch<T, W, GS, V, KERN, S, 1, NW, false>);
            MF_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(efn),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            // the stream form (C > 1, depth-2 pipeline, MF_FLAG_STREAM): one
            // software pipeline through the launch's positions
            const void* sfn = nullptr;
            size_t slds = 0;
            int32_t cap = std::max(p.max_users, 1);
            if constexpr (kDeep == 2 && V <= 2) {      // (rows of <= 2 vectors per lane)
                if ((p.flags & MF_FLAG_STREAM) && deep && a.cls > 1 && p.B <= 256 &&
                    cap <= 4 * TH) {
                    slds = strata_stream_lds_bytes<T>(p.max_items, cap, p.k, TH, p.n_seq) +
                           (a.probe ? 12 * (size_t)p.n_seq : 0);
                    if (slds <= (size_t)kLdsLimit)
                        sfn = cap <= 2 * TH
                                  ? reinterpret_cast<const void*>(
                                        k_sgd_strata_stream<T, W, GS, V, KERN, S, NW, 2>)
                                  : reinterpret_cast<const void*>(
                                        k_sgd_strata_stream<T, W, GS, V, KERN, S, NW, 4>);
                }
            }
            const LaunchTrace lt0;
            if (sfn) {
                MF_HIP_CHECK(hipFuncSetAttribute(sfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)slds));
                lt0.mark("hipFuncSetAttribute");
                persistent = strata_coresident(sfn, p.B, slds, TH);
            } else {
                persistent = strata_coresident(reinterpret_cast<const void*>(efn), p.B, lds, TH);
            }
            lt0.mark("strata_coresident");
            if (p.flags & MF_FLAG_PREPARE) return MF_OK;       // attributes / occupancy only
            if (persistent) {
                const LaunchTrace lt1;
                int32_t* done = static_cast<int32_t*>(p.ws);
                int32_t* err = done + p.B;
                // the (otherwise unused) tail of the workspace holds the XCC
                // table: rows of whole 128-B lines in a 128-B aligned P only
                // (no line is shared by two users, so no line mixes ranges)
                const bool lines = ((size_t)p.k * sizeof(T)) % 128 == 0 &&
                                   (reinterpret_cast<uintptr_t>(p.P) & 127) == 0;
                if ((p.flags & MF_FLAG_L2_HANDOFF) && lines && p.n_seq >= p.B && a.cls == 1 &&
                    strata_xcd_classes(p.seq, p.n_seq, p.B))
                    a.xtab = err + 1;
                int32_t nseq = p.n_seq;
                StrataSeq sq;
                for (int32_t t = 0; t < kStrataSeqArg; ++t)
                    sq.s[t] = (uint16_t)(t < nseq ? p.seq[t] : 0);
                if (strata_inject_fail())
                    MF_HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(err), 1, 1,
                                                   p.stream));
                if (sfn) {
                    a.xtab = nullptr;            // (the L2 hand-off needs one class)
                    void* kargs[] = {&a, &sq, &nseq, &done, &err, &cap};
                    hipError_t ce;
                    if (p.flags & MF_FLAG_NO_COOP)
                        ce = hipLaunchKernel(sfn, dim3((unsigned)p.B), dim3(TH), kargs,
                                             slds, p.stream);
                    else
                        ce = hipLaunchCooperativeKernel(sfn, dim3((unsigned)p.B), dim3(TH),
                                                        kargs, (unsigned)slds, p.stream);
                    if (ce != hipSuccess) {
                        (void)hipGetLastError();
                        persistent = false;
                    }
                    lt1.mark("stream launch");
                } else if (p.flags & MF_FLAG_NO_COOP) {
                    hipLaunchKernelGGL(efn, dim3((unsigned)p.B), dim3(TH), lds,
                                       p.stream, a, sq, nseq, done, err);
                } else {
                    // cooperative: the runtime guarantees that all B workgroups
                    // are resident at once (the neighbour waits need it) or
                    // refuses the launch -- then one launch per stratum below
                    void* kargs[] = {&a, &sq, &nseq, &done, &err};
                    const hipError_t ce = hipLaunchCooperativeKernel(
                        reinterpret_cast<const void*>(efn), dim3((unsigned)p.B),
                        dim3(TH), kargs, (unsigned)lds, p.stream);
                    if (ce != hipSuccess) {
                        (void)hipGetLastError();
                        persistent = false;
                    }
                }
            }
        }
        if (p.flags & MF_FLAG_PREPARE) return MF_OK;
        if (!persistent) {
            const int64_t nq = p.n_items * (int64_t)p.k;
            if (p.dq) {   // delta-out: keep the start values in D (see k_delta_swap)
                MF_HIP_CHECK(hipMemcpyAsync(p.dq, p.Q, sizeof(T) * (size_t)nq,
                                            hipMemcpyDeviceToDevice, p.stream));
                if (KERN != MF_RBF)
                    MF_HIP_CHECK(hipMemcpyAsync(p.dbi, p.bi, sizeof(T) * (size_t)p.n_items,
                                                hipMemcpyDeviceToDevice, p.stream));
            }
            a.Dq = a.Dbi = nullptr;
            for (int32_t t = 0; t < p.n_seq; ++t) {
                a.s = p.seq[t];
                hipLaunchKernelGGL(kfn, dim3((unsigned)p.B), dim3(TH), lds, p.stream,
                                   a);
            }
            if (p.dq) {
                hipLaunchKernelGGL(k_delta_swap<T>, dim3(1024), dim3(kBlock), 0, p.stream,
                                   static_cast<T*>(p.Q), static_cast<T*>(p.dq), nq);
                if (KERN != MF_RBF)
                    hipLaunchKernelGGL(k_delta_swap<T>, dim3(64), dim3(kBlock), 0, p.stream,
                                       static_cast<T*>(p.bi), static_cast<T*>(p.dbi),
                                       p.n_items);
            }
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
                p.kernel_ms[1] = persistent ? 1.0 : (double)p.n_seq;
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
