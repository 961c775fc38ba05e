// mf_als.hip -- alternating least squares for the factor model (BASELINE.json
// config 5).  No reference counterpart: the closest
// is the bias-only `_als` (baseline_model.py:283-362), whose conventions this
// extends to the latent factors.  For one entity e (a user in the user
// half-sweep, an item in the item half-sweep) with ratings r_n against the
// other side's rows z_n (= q_i or p_u) and biases b'_n:
//
//   x_e = [w_e; b_e]   (factor row and bias of e)
//   y_n = [z_n; 1],    t_n = r_n - mu - b'_n
//   (sum_n y_n y_n^T + reg * I) x_e = sum_n t_n y_n
//
// i.e. the exact minimiser of sum_n (t_n - y_n . x_e)^2 + reg |x_e|^2; with
// k = 0 it is baseline_model.py:328-337 ((reg + n) b_e = sum t_n).
//
// One workgroup (4 waves) per entity:
//   1. the Gramian sum z z^T on MFMA: the entity's other-side rows are
//      gathered in chunks of 64 into LDS (software-pipelined through
//      registers) and consumed by v_mfma_f32_32x32x2_f32 (exact f32 products,
//      f32 accumulation), only the upper 32x32 tiles of the symmetric
//      Gramian, spread over the 4 waves; the right-hand columns sum t z and
//      sum z on the VALU beside them;
//   2. the tiles go to LDS as the upper triangle of the (KP) x (KP + 2)
//      augmented matrix; symmetric Gaussian elimination (A = U^T D U, no
//      pivoting: A is SPD) with one barrier per pivot row;
//   3. the bias border by the Schur complement and the back substitution on
//      wave 0: b_e = (sum t - s'.D^-1 f') / (n + reg - s'.D^-1 s'),
//      w_e = U^-1 D^-1 (f' - b_e s')   (f' = U^-T f, s' = U^-T s).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "mf_common.hpp"

namespace mf {

constexpr int kAlsThreads = 256;
constexpr int kAlsChunk = 64;        // other-side rows per LDS chunk (32 K-steps)
constexpr int kAlsMaxFactors = 128;

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;

// MFMA tiles of the symmetric Gramian: column blocks J = 0..NT-1, row blocks
// I <= J.  Tile q is computed by wave q % 4.  The two right-hand columns
// (sum t z, sum z) are VALU sums: wave w < NT accumulates column block w.
template <int NT>
struct AlsTiles {
    static constexpr int count = NT * (NT + 1) / 2;
    static constexpr int per_wave = (count + 3) / 4;
    static constexpr int I(int q) {
        for (int J = 0, n = 0; J < NT; ++J)
            for (int i = 0; i <= J; ++i, ++n)
                if (n == q) return i;
        return 0;
    }
    static constexpr int J(int q) {
        for (int J = 0, n = 0; J < NT; ++J)
            for (int i = 0; i <= J; ++i, ++n)
                if (n == q) return J;
        return 0;
    }
};

struct AlsArgs {
    const int64_t* ptr;        // n_entities + 1
    const int32_t* other;      // other-side id per rating (CSR order)
    const float* r;            // rating per rating (CSR order)
    const float* ob;           // other-side biases
    const float* oq;           // other-side factor rows (row-major, k)
    float* bias;               // solved biases (n_entities)
    float* feat;               // solved factor rows (n_entities x k)
    int32_t k;
    float mu;
    float reg;
    int64_t* probe;            // nullable: 4 wall-clock stamps per workgroup
};

// profiling probe: s_memrealtime (100 MHz) at the phase boundaries
__device__ __forceinline__ void als_stamp(const AlsArgs& A, int slot) {
    if (A.probe && threadIdx.x == 0)
        A.probe[(int64_t)blockIdx.x * 4 + slot] = (int64_t)__builtin_amdgcn_s_memrealtime();
}

// One K-step (two chunk rows) of wave WV: the MFMAs of its tiles, and the
// right-hand sums of column block WV (lane (r, h): column 32 WV + r, row h).
template <int NT, int WV>
__device__ __forceinline__ void als_kstep(const float* zr, float tv, int r,
                                          f32x16 (&acc)[AlsTiles<NT>::per_wave],
                                          float& fsum, float& ssum) {
    using TL = AlsTiles<NT>;
    float zv[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) zv[I] = zr[32 * I + r];
#pragma unroll
    for (int s = 0; s < TL::per_wave; ++s) {
        const int q = WV + 4 * s;
        if (q < TL::count)
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(zv[TL::I(q)], zv[TL::J(q)], acc[s],
                                                          0, 0, 0);
    }
    if constexpr (WV < NT) {
        fsum = __builtin_fmaf(tv, zv[WV], fsum);
        ssum = ssum + zv[WV];
    }
}

// Accumulator tiles -> M (row stride LD): the symmetric Gramian in full (an
// off-diagonal tile is also stored transposed); the right-hand sums of
// column block WV -> columns KP, KP + 1.
template <int NT, int WV>
__device__ __forceinline__ void als_dump(float* M, int LD, int lane,
                                         const f32x16 (&acc)[AlsTiles<NT>::per_wave],
                                         float fsum, float ssum) {
    using TL = AlsTiles<NT>;
    constexpr int KP = NT * 32;
    const int col = lane & 31, h = lane >> 5;
#pragma unroll
    for (int s = 0; s < TL::per_wave; ++s) {
        const int q = WV + 4 * s;
        if (q >= TL::count) continue;
        const int I = TL::I(q), J = TL::J(q);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = 32 * I + (i & 3) + 8 * (i >> 2) + 4 * h;
            M[row * LD + 32 * J + col] = acc[s][i];
            if (I < J) M[(32 * J + col) * LD + row] = acc[s][i];
        }
    }
    if constexpr (WV < NT) {
        // rows h = 0 and h = 1 of every K-step: lanes r and r + 32
        fsum = fsum + __shfl_xor(fsum, 32, kWave);
        ssum = ssum + __shfl_xor(ssum, 32, kWave);
        if (h == 0) {
            M[(32 * WV + col) * LD + KP] = fsum;
            M[(32 * WV + col) * LD + KP + 1] = ssum;
        }
    }
}

// The Gramian of one entity on wave WV's tiles.  Chunks of kAlsChunk other-
// side rows are software-pipelined through registers: while the MFMAs
// consume chunk c from LDS, the rows of chunk c + 1 (ids loaded one chunk
// earlier) are in flight.  Thread t moves float4 column c4 = t % C4 of rows
// n = t / C4 + (256 / C4) * w; thread t < kAlsChunk also fetches the rating
// and the other-side bias of row t (the right-hand side t_n), summing them.
template <int NT, int WV>
__device__ __forceinline__ void als_gram_wave(const AlsArgs& A, float* Zc, float* tc, int64_t p0,
                                              int64_t cnt, int lane, float* M, int LD,
                                              float& tsum) {
    using TL = AlsTiles<NT>;
    constexpr int KP = NT * 32;
    constexpr int C4 = KP / 4;                    // float4 per row
    constexpr int RPP = kAlsThreads / C4;         // rows per pass of the block
    constexpr int NW = kAlsChunk / RPP;           // float4 per thread per chunk
    static_assert(kAlsThreads % C4 == 0 && kAlsChunk % RPP == 0, "chunk tiling");
    const int tid = threadIdx.x;
    const int c4 = tid % C4, n0 = tid / C4;
    const int k = A.k;
    const bool vec = (k & 3) == 0;
    const bool col_ok = vec ? 4 * c4 < k : true;
    f32x16 acc[TL::per_wave];
#pragma unroll
    for (int s = 0; s < TL::per_wave; ++s)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[s][i] = 0.f;
    const int r = lane & 31, h = lane >> 5;
    float fsum = 0.f, ssum = 0.f;

    auto load_ids = [&](int64_t c0, int (&ids)[NW], int& tid_id, float& rr) __attribute__((always_inline)) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const int64_t n = c0 + n0 + RPP * w;
            ids[w] = n < cnt ? A.other[p0 + n] : -1;
        }
        const int64_t nt = c0 + tid;
        tid_id = (tid < kAlsChunk && nt < cnt) ? A.other[p0 + nt] : -1;
        rr = (tid < kAlsChunk && nt < cnt) ? A.r[p0 + nt] : 0.f;
    };
    auto load_rows = [&](const int (&ids)[NW], float4 (&v)[NW]) __attribute__((always_inline)) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const int id = ids[w] >= 0 ? ids[w] : 0;
            const float* row = A.oq + (int64_t)id * k;
            if (vec) {
                v[w] = *reinterpret_cast<const float4*>(row + (col_ok ? 4 * c4 : 0));
            } else {
                const int c = 4 * c4;
                v[w].x = c + 0 < k ? row[c + 0] : 0.f;
                v[w].y = c + 1 < k ? row[c + 1] : 0.f;
                v[w].z = c + 2 < k ? row[c + 2] : 0.f;
                v[w].w = c + 3 < k ? row[c + 3] : 0.f;
            }
        }
    };

    int ids[NW], tid_id;
    float rr;
    float4 v[NW];
    load_ids(0, ids, tid_id, rr);
    load_rows(ids, v);
    float ob = tid_id >= 0 ? A.ob[tid_id] : 0.f;
    float rr_cur = rr;
    load_ids(kAlsChunk, ids, tid_id, rr);         // chunk 1's ids (may be empty)
    for (int64_t c0 = 0; c0 < cnt; c0 += kAlsChunk) {
        const int m = (int)min((int64_t)kAlsChunk, cnt - c0);
        __syncthreads();                          // previous chunk consumed
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const bool ok = (c0 + n0 + RPP * w < cnt) && col_ok;
            *reinterpret_cast<float4*>(Zc + (n0 + RPP * w) * KP + 4 * c4) =
                ok ? v[w] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (tid < kAlsChunk) {
            const float t = tid < m ? (rr_cur - A.mu) - ob : 0.f;
            tc[tid] = t;
            tsum += t;
        }
        __syncthreads();
        // next chunk: rows from the ids already loaded, then the ids after it
        const float rr_next = rr;
        const int id_next = tid_id;
        load_rows(ids, v);
        load_ids(c0 + 2 * kAlsChunk, ids, tid_id, rr);
        ob = id_next >= 0 ? A.ob[id_next] : 0.f;
        rr_cur = rr_next;
        const int steps = (m + 1) >> 1;
        for (int s = 0; s < steps; ++s) {
            const int n = 2 * s + h;                  // rows past m are zero rows
            als_kstep<NT, WV>(Zc + n * KP, tc[n], r, acc, fsum, ssum);
        }
    }
    __syncthreads();                              // Zc is reused as M below
    als_dump<NT, WV>(M, LD, lane, acc, fsum, ssum);
}

template <int NT>
__global__ __launch_bounds__(kAlsThreads, 2) void k_als_solve(AlsArgs A) {
    constexpr int KP = NT * 32;
    constexpr int LD = KP + 3;                    // odd stride: column reads conflict-free
    extern __shared__ __align__(16) float lds[];
    float* Zc = lds;                              // [kAlsChunk][KP]   (Gramian phase)
    float* tc = lds + kAlsChunk * KP;             // [kAlsChunk]
    float* M = lds;                               // [KP][LD]          (solve phase)
    __shared__ float red[kAlsThreads / kWave];

    const int e = blockIdx.x;
    const int64_t p0 = A.ptr[e], cnt = A.ptr[e + 1] - p0;
    if (cnt == 0) return;                         // no ratings: parameters kept
    als_stamp(A, 0);
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int k = A.k;

    // the Gramian; wave 0 also sums the right-hand side t over the ratings
    float ts = 0.f;
    switch (wv) {
        case 0: als_gram_wave<NT, 0>(A, Zc, tc, p0, cnt, lane, M, LD, ts); break;
        case 1: als_gram_wave<NT, 1>(A, Zc, tc, p0, cnt, lane, M, LD, ts); break;
        case 2: als_gram_wave<NT, 2>(A, Zc, tc, p0, cnt, lane, M, LD, ts); break;
        default: als_gram_wave<NT, 3>(A, Zc, tc, p0, cnt, lane, M, LD, ts); break;
    }
    if (wv == 0) {
        ts = wave_sum(ts);
        if (lane == 0) red[0] = ts;
    }
    __syncthreads();
    als_stamp(A, 1);
    const float g = red[0];

    // ---- symmetric elimination, register-tiled: thread (ty, tx) of a 16 x 16
    // grid holds rows ty + 16x and columns tx + 16y of [A | f | s] (the full
    // symmetric trailing block is updated, so row j is also column j).  Per
    // pivot: the 16 owners of row j publish it to a double-buffered LDS row,
    // one barrier, every thread applies the rank-1 update to its elements.
    constexpr int RX = KP / 16;                   // rows per thread
    constexpr int CY = KP / 16 + 1;               // columns per thread (+ f, s)
    constexpr int CW = 16 * CY;                   // published row width
    __shared__ float rowbuf[2][4][CW];            // four pivot rows, double-buffered
    const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
    float m[RX][CY];
#pragma unroll
    for (int x = 0; x < RX; ++x) {
        const int a = ty + 16 * x;
#pragma unroll
        for (int y = 0; y < CY; ++y) {
            const int b = tx + 16 * y;
            float v = b < KP + 2 ? M[a * LD + b] : 0.f;
            // + reg on the diagonal; padding dimensions (k <= a < KP) are
            // decoupled zero rows: pivot 1, solution 0
            if (a == b) v = a < k ? v + A.reg : 1.f;
            m[x][y] = v;
        }
    }
    // Pivots in groups of four, one barrier per group: the wave holding rows
    // j0..j0+3 (ty = 4 jq .. 4 jq + 3) publishes them; every thread eliminates
    // the 4 x 4 diagonal block redundantly on the entries it needs (its
    // columns tx + 16y, its rows' columns ty + 16x, by symmetry) and applies
    // the rank-4 update to its trailing elements.  The row-block index jb is
    // a compile-time constant in each unrolled copy, so finished rows and
    // columns (x, y < jb) are skipped statically.
#pragma unroll
    for (int jb = 0; jb < RX; ++jb) {
#pragma clang loop unroll(disable)
        for (int jq = 0; jq < 4; ++jq) {
            const int j0 = 16 * jb + 4 * jq;
            float (*rb)[CW] = rowbuf[jq & 1];
            const bool owner = (ty >> 2) == jq;
            if (owner) {
#pragma unroll
                for (int y = jb; y < CY; ++y) rb[ty & 3][tx + 16 * y] = m[jb][y];
            }
            __syncthreads();
            float D[4][4], PR[4][CY], inv[4], f[4][4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int c = 0; c < 4; ++c) D[r][c] = rb[r][j0 + c];
#pragma unroll
                for (int y = jb; y < CY; ++y) PR[r][y] = rb[r][tx + 16 * y];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                inv[r] = 1.f / D[r][r];
#pragma unroll
                for (int r2 = r + 1; r2 < 4; ++r2) {
                    f[r][r2] = D[r][r2] * inv[r];
#pragma unroll
                    for (int c = r2; c < 4; ++c)
                        D[r2][c] = __builtin_fmaf(-f[r][r2], D[r][c], D[r2][c]);
#pragma unroll
                    for (int y = jb; y < CY; ++y)
                        PR[r2][y] = __builtin_fmaf(-f[r][r2], PR[r][y], PR[r2][y]);
                }
            }
            // rank-4 update; element (a, b) takes pivot j0 + r when a and b
            // both lie past it -- for the pivot rows' owners this yields the
            // row eliminated by the earlier pivots of the group (final).  The
            // multipliers of row a are the pivot rows at column a (symmetry),
            // read here and eliminated like PR.
#pragma unroll
            for (int x = jb; x < RX; ++x) {
                const int a = ty + 16 * x;
                float pc[4], l4[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) pc[r] = rb[r][a];
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int r2 = r + 1; r2 < 4; ++r2)
                        pc[r2] = __builtin_fmaf(-f[r][r2], pc[r], pc[r2]);
#pragma unroll
                for (int r = 0; r < 4; ++r) l4[r] = a > j0 + r ? pc[r] * inv[r] : 0.f;
#pragma unroll
                for (int y = jb; y < CY; ++y) {
                    const int b = tx + 16 * y;
                    float upd = m[x][y];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float lr = b > j0 + r ? l4[r] : 0.f;
                        upd = __builtin_fmaf(-lr, PR[r][y], upd);
                    }
                    m[x][y] = upd;
                }
            }
        }
    }
    // eliminated rows (D U | f' | s') back to M for the back substitution
#pragma unroll
    for (int x = 0; x < RX; ++x)
#pragma unroll
        for (int y = 0; y < CY; ++y) {
            const int b = tx + 16 * y;
            if (b < KP + 2) M[(ty + 16 * x) * LD + b] = m[x][y];
        }
    __syncthreads();
    als_stamp(A, 2);

    // ---- border (Schur complement) and back substitution: wave 0
    if (wv != 0) return;
    const int a0 = lane, a1 = lane + kWave;       // rows owned by this lane
    const bool v0 = a0 < KP, v1 = a1 < KP;
    const float d0 = v0 ? M[a0 * LD + a0] : 1.f, d1 = v1 ? M[a1 * LD + a1] : 1.f;
    const float i0 = 1.f / d0, i1 = 1.f / d1;
    const float f0 = v0 ? M[a0 * LD + KP] : 0.f, s0 = v0 ? M[a0 * LD + KP + 1] : 0.f;
    const float f1 = v1 ? M[a1 * LD + KP] : 0.f, s1 = v1 ? M[a1 * LD + KP + 1] : 0.f;
    const float num = wave_sum((s0 * f0) * i0 + (s1 * f1) * i1);
    const float den = wave_sum((s0 * s0) * i0 + (s1 * s1) * i1);
    const float b = (g - num) / (((float)cnt + A.reg) - den);
    const float w0 = (f0 - b * s0) * i0, w1 = (f1 - b * s1) * i1;
    float acc0 = 0.f, acc1 = 0.f, x0 = 0.f, x1 = 0.f;
    // Columns j of rows a0, a1 come from LDS in blocks of 8, one block ahead
    // (a load one column ahead left most of the LDS latency on the critical
    // path of the readlane chain); two register blocks used alternately.
    constexpr int BJ = 8;
    static_assert(KP % (2 * BJ) == 0, "back substitution blocks");
    float cA0[BJ], cA1[BJ], cB0[BJ], cB1[BJ];
    auto load_cols = [&](int jb, float (&c0)[BJ], float (&c1)[BJ]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < BJ; ++u) {
            c0[u] = v0 ? M[a0 * LD + jb + u] : 0.f;
            c1[u] = v1 ? M[a1 * LD + jb + u] : 0.f;
        }
    };
    auto solve_cols = [&](int jb, const float (&c0)[BJ], const float (&c1)[BJ])
                          __attribute__((always_inline)) {
#pragma unroll
        for (int u = BJ - 1; u >= 0; --u) {
            const int j = jb + u;
            const float cand = j >= kWave ? (w1 - acc1) : (w0 - acc0);
            const float xj =
                __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cand), j & (kWave - 1)));
            if (lane == (j & (kWave - 1))) {
                if (j >= kWave) x1 = xj;
                else x0 = xj;
            }
            if (v0 && a0 < j) acc0 = acc0 + (c0[u] * i0) * xj;
            if (v1 && a1 < j) acc1 = acc1 + (c1[u] * i1) * xj;
        }
    };
    load_cols(KP - BJ, cA0, cA1);
    for (int jb = KP - BJ; jb >= 0; jb -= 2 * BJ) {
        load_cols(jb - BJ, cB0, cB1);             // jb - BJ >= 0: KP % (2 BJ) == 0
        solve_cols(jb, cA0, cA1);
        if (jb - 2 * BJ >= 0) load_cols(jb - 2 * BJ, cA0, cA1);
        solve_cols(jb - BJ, cB0, cB1);
    }
    float* out = A.feat + (int64_t)e * k;
    if (v0 && a0 < k) out[a0] = x0;
    if (v1 && a1 < k) out[a1] = x1;
    if (lane == 0) A.bias[e] = b;
    als_stamp(A, 3);
}

// ---- one wave per entity ---------------------------------------------------
//
// k_als_wave: the same system, solved by ONE wave with no cross-wave
// synchronisation (one-wave workgroups; at rank 128 four per CU, one per
// SIMD):
//   1. Gramian, fed by an all-DMA pipeline (nothing the loop consumes is a
//      VMEM register load, so no vmcnt(0) drain): per chunk of kAlsRingRows
//      rows, stage A moves the ids and ratings (global_load_lds, 4 B per
//      lane) into LDS slots four chunks ahead; stage B, two chunks ahead,
//      reads the ids back and moves the rows (16 B per lane, 1 KiB = 8 / NT
//      rows per wave-instruction) into a 3-chunk ring and the other side's
//      biases into their slot; counted vmcnt waits + the (one-wave) barrier
//      order them for the ds_reads.  Lane (c, h) of K-step s reads column
//      32 I + c of chunk row 2 s + h, which is both the A and the B operand
//      of tile (I, J); every upper tile of the KP x KP Gramian accumulates
//      in the wave's own registers.  The right-hand columns (sum t z, sum z)
//      on the VALU beside the MFMAs.
//   2. symmetric elimination in registers.  Pivot j's row is extracted from
//      its tile register (wave-uniform dynamic index), swapped across the
//      lane halves (v_permlane32_swap) and readlane'd for the pivot; its
//      values at a lane's columns come from registers, the multipliers of a
//      lane's rows from the row published in LDS (zeros at columns <= j).
//      The row of pivot j + 1 is extracted and published as soon as its own
//      tile row is updated, so that LDS round trip overlaps the rest of
//      pivot j's update.  The two right-hand columns live row-per-lane
//      (rows L, L + 64).  The eliminated rows (D U) go to LDS packed.
//   3. the bias border (Schur complement) and the back substitution, as in
//      k_als_solve.
// Ranks with n_factors % 4 != 0 (rows not 16-byte aligned for the DMA) use
// k_als_solve.
constexpr int kAlsRingRows = 16;       // rows per ring chunk (8 K-steps)
constexpr int kAlsRowBufs = 2;         // ring chunks (rows one chunk ahead)
constexpr int kAlsIdSlots = 4;         // id / rating / bias slots (ids three chunks ahead)

__device__ __forceinline__ int upk_off(int j, int KP) { return j * KP - ((j * (j - 1)) >> 1); }

template <int NT>
struct AlsWaveShape {
    static constexpr int KP = 32 * NT;
    static constexpr int NR = (KP + kWave - 1) / kWave;   // row-per-lane slots
    static constexpr int CR = kAlsRingRows;
    static constexpr int RPP = 8 / NT;                     // rows per 1-KiB DMA piece
    static constexpr int LPR = 8 * NT;                     // lanes per row (16 B each)
    static constexpr int PPC = CR / RPP;                   // pieces per chunk
    static constexpr int elim_floats = 2 * KP + 32 * 33;   // pivot rows + transpose scratch
    static constexpr int gram_floats = kAlsRowBufs * CR * KP + 3 * kAlsIdSlots * kWave;
    static constexpr int lds_floats = elim_floats > gram_floats ? elim_floats : gram_floats;
    static constexpr int q(int I, int J) {                 // tile index of (I <= J)
        int n = 0;
        for (int JJ = 0; JJ < NT; ++JJ)
            for (int II = 0; II <= JJ; ++II, ++n)
                if (II == I && JJ == J) return n;
        return -1;
    }
};

__device__ __forceinline__ void als_lds_dma4(const void* src, void* lds_dst) {
    __builtin_amdgcn_global_load_lds(
        (__attribute__((address_space(1))) void*)const_cast<void*>(src),
        (__attribute__((address_space(3))) void*)lds_dst, 4, 0, 0);
}
__device__ __forceinline__ void als_lds_dma16(const void* src, void* lds_dst) {
    __builtin_amdgcn_global_load_lds(
        (__attribute__((address_space(1))) void*)const_cast<void*>(src),
        (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

template <int NT>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(2))) void k_als_wave(AlsArgs A) {
    using TL = AlsTiles<NT>;
    using SH = AlsWaveShape<NT>;
    constexpr int KP = SH::KP, NR = SH::NR, NQ = TL::count;
    constexpr int CR = SH::CR, RPP = SH::RPP, LPR = SH::LPR, PPC = SH::PPC;
    extern __shared__ __align__(16) float lds[];

    const int e = blockIdx.x;
    const int64_t p0 = A.ptr[e], cnt = A.ptr[e + 1] - p0;
    if (cnt == 0) return;                         // no ratings: parameters kept
    als_stamp(A, 0);
    const int L = threadIdx.x, c = L & 31, h = L >> 5;
    const int k = A.k;

    // ---- 1. Gramian ---------------------------------------------------------
    constexpr int NB = kAlsRowBufs, NS = kAlsIdSlots;
    float* Zb = lds;                              // [NB][CR][KP] row ring (DMA image)
    int* ids = reinterpret_cast<int*>(lds + NB * CR * KP);   // [NS][64]
    float* rts = lds + NB * CR * KP + NS * kWave;           // [NS][64] ratings
    float* obs = rts + NS * kWave;                          // [NS][64] other-side biases
    f32x16 m[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int i = 0; i < 16; ++i) m[q][i] = 0.f;
    float fz[NT], sz[NT], ts = 0.f;
#pragma unroll
    for (int I = 0; I < NT; ++I) fz[I] = sz[I] = 0.f;
    bool colok[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) colok[I] = 32 * I + c < k;
    const int nch = (int)((cnt + CR - 1) / CR);
    // stage A: ids and ratings of chunk X (lane L: row X CR + L, clamped to
    // the entity's last rating so every id is a real one)
    auto stage_a = [&](int X) __attribute__((always_inline)) {
        const int64_t n = min((int64_t)X * CR + L, cnt - 1);
        const int sl = X % NS;
        als_lds_dma4(A.other + p0 + n, ids + sl * kWave);
        als_lds_dma4(A.r + p0 + n, rts + sl * kWave);
    };
    // stage B: rows and other-side biases of chunk X (ids landed): piece p
    // covers chunk rows p RPP .. p RPP + RPP-1, lane L 16 B of row p RPP +
    // L / LPR (columns past k read the row start: masked where read)
    auto stage_b = [&](int X) __attribute__((always_inline)) {
        const int sl = X % NS;
        float* dst = Zb + (X % NB) * CR * KP;
        const int c4 = 4 * (L % LPR);
#pragma unroll
        for (int p = 0; p < PPC; ++p) {
            const int idr = ids[sl * kWave + p * RPP + L / LPR];
            als_lds_dma16(A.oq + (int64_t)idr * k + (c4 < k ? c4 : 0), dst + p * RPP * KP);
        }
        als_lds_dma4(A.ob + ids[sl * kWave + L], obs + sl * kWave);
    };
    // iteration cc issues B(cc+1) then A(cc+3); at its start chunk cc's rows
    // (B, previous iteration) and chunk cc+1's ids (A, two back) must have
    // landed, so only A(cc+2), issued after B(cc), may still be in flight
    stage_a(0);
    if (nch > 1) stage_a(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stage_b(0);
    if (nch > 2) stage_a(2);
    for (int cc = 0; cc < nch; ++cc) {
        if (cc + 2 < nch) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (cc + 1 < nch) stage_b(cc + 1);
        if (cc + 3 < nch) stage_a(cc + 3);
        const float* Zc = Zb + (cc % NB) * CR * KP;
        const float* rc = rts + (cc % NS) * kWave;
        const float* bc = obs + (cc % NS) * kWave;
        const int64_t base = (int64_t)cc * CR;
        // K-steps of this chunk (the last one stops at the entity's end);
        // the LDS reads of step s + 1 are issued before the MFMAs of step s
        const int steps = (int)min((int64_t)(CR / 2), (cnt - base + 1) >> 1);
        float vn[NT], rn, bn;
        auto ld = [&](int s_) __attribute__((always_inline)) {
            const int n = 2 * s_ + h;
#pragma unroll
            for (int I = 0; I < NT; ++I) vn[I] = Zc[n * KP + 32 * I + c];
            rn = rc[n];
            bn = bc[n];
        };
        ld(0);
#pragma unroll
        for (int s = 0; s < CR / 2; ++s) {
            if (s >= steps) break;
            // the empty asm pins the values here (the loads stay unconditional
            // and in flight across the previous step's MFMAs)
#pragma unroll
            for (int I = 0; I < NT; ++I) asm volatile("" : "+v"(vn[I]));
            asm volatile("" : "+v"(rn), "+v"(bn));
            const bool ok = base + 2 * s + h < cnt;
            float zv[NT];
#pragma unroll
            for (int I = 0; I < NT; ++I) zv[I] = ok && colok[I] ? vn[I] : 0.f;
            const float tv = ok ? (rn - A.mu) - bn : 0.f;
            if (s + 1 < CR / 2) ld(s + 1);        // row s + 1 < CR: in the chunk
            __builtin_amdgcn_sched_barrier(0);    // keep those reads ahead of the MFMAs
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                m[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(zv[TL::I(q)], zv[TL::J(q)], m[q],
                                                            0, 0, 0);
#pragma unroll
            for (int I = 0; I < NT; ++I) {
                fz[I] = __builtin_fmaf(tv, zv[I], fz[I]);
                sz[I] = sz[I] + zv[I];
            }
            ts += c == 0 ? tv : 0.f;
        }
    }
    // column sums over both row halves; g = sum t over the rows (lanes c == 0)
#pragma unroll
    for (int I = 0; I < NT; ++I) {
        fz[I] = fz[I] + __shfl_xor(fz[I], 32, kWave);
        sz[I] = sz[I] + __shfl_xor(sz[I], 32, kWave);
    }
    const float gsum = wave_sum(ts);
    // right-hand columns row-per-lane: slot x holds row a = L + 64 x
    float fr[NR], sr[NR];
#pragma unroll
    for (int x = 0; x < NR; ++x) {
        const int a = L + 64 * x;
        float fv = 0.f, sv = 0.f;
#pragma unroll
        for (int I = 2 * x; I < 2 * x + 2 && I < NT; ++I)
            if ((I & 1) == h) { fv = fz[I]; sv = sz[I]; }
        fr[x] = a < KP ? fv : 0.f;
        sr[x] = a < KP ? sv : 0.f;
    }
    // + reg on the diagonal; padding dimensions (k <= a < KP) pivot 1
#pragma unroll
    for (int I = 0; I < NT; ++I) {
        const int q = SH::q(I, I);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int ra = (i & 3) + 8 * (i >> 2) + 4 * h;
            const float dg = 32 * I + c < k ? m[q][i] + A.reg : 1.f;
            m[q][i] = ra == c ? dg : m[q][i];
        }
    }
    __syncthreads();                              // the ring is reused below
    als_stamp(A, 1);

    // ---- 2. elimination -----------------------------------------------------
    float* prow = lds;                            // [2][KP] published pivot rows
    // pivot state: u[J] = row j at column 32 J + c (both halves), d, r = 1 / d
    float u[NT], r, dpiv;
    float dreg[NR];                               // D_a, row-per-lane (rows L + 64 x)
#pragma unroll
    for (int x = 0; x < NR; ++x) dreg[x] = 1.f;
    // extract row j (tile row Ij) into u / d / r and publish it to prow[j & 1]
    auto publish = [&](int Ij, int j) __attribute__((always_inline)) {
        const int jl = j - 32 * Ij;
        const int ij = (jl & 3) | ((jl >> 3) << 2);   // register of row j in its tile
        const int hj = (jl >> 2) & 1;                 // lane half holding it
        float* pr = prow + (j & 1) * KP;
        float dv = 0.f;
#pragma unroll
        for (int J = 0; J < NT; ++J) {
            if (J < Ij) continue;
            const float v = m[SH::q(Ij, J)][ij];
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v),
                                                             false, false);
            const float uv = __uint_as_float(hj ? sw[1] : sw[0]);
            const int b = 32 * J + c;
            u[J] = b > j ? uv : 0.f;
            pr[b] = u[J];                         // both halves: same address, same value
            if (J == Ij) dv = uv;
        }
        dpiv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dv), jl));
        // 1/d: v_rcp_f32 (1 ulp) and one Newton step
        float rr = __builtin_amdgcn_rcpf(dpiv);
        r = rr * __builtin_fmaf(-dpiv, rr, 2.f);
    };
    // rank-1 update of tile row I by pivot j (published in prow[j & 1])
    auto update_row = [&](int I, const float* pr, const float (&w)[NT]) __attribute__((always_inline)) {
        float l[16];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const float4 v4 = *reinterpret_cast<const float4*>(pr + 32 * I + 8 * qq + 4 * h);
            l[4 * qq + 0] = v4.x; l[4 * qq + 1] = v4.y;
            l[4 * qq + 2] = v4.z; l[4 * qq + 3] = v4.w;
        }
#pragma unroll
        for (int J = 0; J < NT; ++J) {
            if (J < I) continue;
            const int q = SH::q(I, J);
            const f32x2 wv = {w[J], w[J]};
#pragma unroll
            for (int i = 0; i < 16; i += 2) {     // v_pk_fma_f32: two rows per instruction
                f32x2 mv = {m[q][i], m[q][i + 1]};
                const f32x2 lv = {l[i], l[i + 1]};
                mv = __builtin_elementwise_fma(lv, wv, mv);
                m[q][i] = mv[0];
                m[q][i + 1] = mv[1];
            }
        }
    };
#pragma unroll
    for (int Ij = 0; Ij < NT; ++Ij) {
        publish(Ij, 32 * Ij);
#pragma clang loop unroll(disable)
        for (int jl = 0; jl < 32; ++jl) {
            const int j = 32 * Ij + jl;
            const float* pr = prow + (j & 1) * KP;
            float w[NT];                          // -(row j at this lane's columns) / d
#pragma unroll
            for (int J = 0; J < NT; ++J) w[J] = J < Ij ? 0.f : u[J] * -r;
            const float fjr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fr[Ij >> 1]), j & 63)) * -r;
            const float sjr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sr[Ij >> 1]), j & 63)) * -r;
            dreg[Ij >> 1] = L == (j & 63) ? dpiv : dreg[Ij >> 1];
            // the published row is read from LDS, never forwarded from this
            // lane's own stores: one wave, so the barrier is the lgkmcnt drain
            __syncthreads();
            update_row(Ij, pr, w);
            if (jl < 31) publish(Ij, j + 1);      // overlaps the updates below
#pragma unroll
            for (int I = Ij + 1; I < NT; ++I) update_row(I, pr, w);
#pragma unroll
            for (int x = 0; x < NR; ++x) {
                // rows up to j keep their value (the published row only
                // covers tile columns >= Ij; earlier columns are stale)
                const int a = L + 64 * x;
                const float la = a > j && a < KP ? pr[a] : 0.f;
                fr[x] = __builtin_fmaf(la, fjr, fr[x]);
                sr[x] = __builtin_fmaf(la, sjr, sr[x]);
            }
        }
    }
    als_stamp(A, 2);

    // ---- 3. border (Schur complement) and back substitution -------------------
    // The eliminated rows D U stay in the tile registers (row j is never
    // updated after its pivot).  Bottom-up per tile row I: (i) the solved
    // tiles J > I contribute U_IJ x_J, lane partials reduced through LDS;
    // (ii) the diagonal tile, transposed through LDS, is solved in 32
    // sequential column steps: lane (c, h) keeps row 32 I + c's partial sum
    // over the columns its half holds, x_t = (r_t - both halves' sums) / D_t.
    float* S = lds + 2 * KP;                      // [32][33] transpose scratch
    float dinv[NR], y[NR];
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int x = 0; x < NR; ++x) {
        dinv[x] = 1.f / dreg[x];
        num += (sr[x] * fr[x]) * dinv[x];
        den += (sr[x] * sr[x]) * dinv[x];
    }
    num = wave_sum(num);
    den = wave_sum(den);
    const float bias = (gsum - num) / (((float)cnt + A.reg) - den);
#pragma unroll
    for (int x = 0; x < NR; ++x) y[x] = fr[x] - bias * sr[x];
    float xc[NT];                                 // x_{32 J + c} at lane c (both halves)
#pragma unroll
    for (int J = 0; J < NT; ++J) xc[J] = 0.f;
#pragma unroll
    for (int I = NT - 1; I >= 0; --I) {
        const int src = 32 * (I & 1) + c;         // row 32 I + c in the row-per-lane slots
        const float yc = __shfl(y[I >> 1], src, kWave);
        const float dc = __shfl(dinv[I >> 1], src, kWave);
        float off = 0.f;
        if (I < NT - 1) {
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float pv = 0.f;
#pragma unroll
                for (int J = I + 1; J < NT; ++J) pv = __builtin_fmaf(m[SH::q(I, J)][i], xc[J], pv);
                S[((i & 3) + 8 * (i >> 2) + 4 * h) * 33 + c] = pv;
            }
            __syncthreads();
            float sacc = 0.f;
#pragma unroll
            for (int cc2 = 0; cc2 < 16; ++cc2) sacc += S[c * 33 + 16 * h + cc2];
            off = sacc + __shfl_xor(sacc, 32, kWave);
        }
        const float rc = yc - off;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) S[((i & 3) + 8 * (i >> 2) + 4 * h) * 33 + c] = m[SH::q(I, I)][i];
        __syncthreads();
        float T[16];                              // T[i] = U[32 I + c][32 I + ra(i, h)]
#pragma unroll
        for (int i = 0; i < 16; ++i) T[i] = S[c * 33 + (i & 3) + 8 * (i >> 2) + 4 * h];
        float acc = 0.f, xi = 0.f;
#pragma unroll
        for (int tl = 31; tl >= 0; --tl) {
            const int it = (tl & 3) + 4 * (tl >> 3), ht = (tl >> 2) & 1;
            const float s0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rc - acc), tl));
            const float s1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), 32 + tl));
            const float dt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dc), tl));
            const float xv = (s0 - s1) * dt;
            xi = c == tl ? xv : xi;
            const float uct = (h == ht && c < tl) ? T[it] : 0.f;
            acc = __builtin_fmaf(uct, xv, acc);
        }
        xc[I] = xi;
        float* out = A.feat + (int64_t)e * k;
        if (h == 0 && 32 * I + c < k) out[32 * I + c] = xi;
    }
    if (L == 0) A.bias[e] = bias;
    als_stamp(A, 3);
}

template <int NT>
int als_go_wave(const AlsArgs& a, int32_t n, hipStream_t stream) {
    const size_t lds = (size_t)AlsWaveShape<NT>::lds_floats * sizeof(float);
    auto kfn = k_als_wave<NT>;
    MF_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kfn, dim3((unsigned)n), dim3(kWave), lds, stream, a);
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}

template <int NT>
int als_go(const AlsArgs& a, int32_t n, hipStream_t stream) {
    constexpr int KP = NT * 32;
    const size_t lds = std::max((size_t)KP * (KP + 3), (size_t)kAlsChunk * KP + kAlsChunk) *
                       sizeof(float);
    auto kfn = k_als_solve<NT>;
    MF_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kfn, dim3((unsigned)n), dim3(kAlsThreads), lds, stream, a);
    MF_HIP_CHECK(hipGetLastError());
    return MF_OK;
}

void touch_als(hipStream_t s) { hipLaunchKernelGGL(k_touch<7>, dim3(1), dim3(64), 0, s); }

}  // namespace mf

using namespace mf;

extern "C" int32_t mf_als_max_factors(void) { return kAlsMaxFactors; }

static int als_sweep(const int64_t* entity_ptr, const int32_t* other_ids,
                            const void* ratings, int32_t n_entities, double global_mean,
                            const void* other_biases, const void* other_features,
                            void* biases, void* features, int32_t n_factors, int32_t dtype,
                            double reg, void* stream, int64_t* probe) {
    if (n_entities < 0 || n_factors < 1 || n_factors > kAlsMaxFactors) {
        set_error("mf_als_sweep: n_entities=%d / n_factors=%d (must be in [1, %d])", n_entities,
                  n_factors, kAlsMaxFactors);
        return MF_ERR_INVALID;
    }
    if (dtype != MF_F32) {
        set_error("mf_als_sweep: float32 only (f32-input MFMA Gramian)");
        return MF_ERR_INVALID;
    }
    if (n_entities == 0) return MF_OK;
    if (!entity_ptr || !other_biases || !other_features || !biases || !features) {
        set_error("mf_als_sweep: NULL argument");
        return MF_ERR_INVALID;
    }
    AlsArgs a;
    a.ptr = entity_ptr; a.other = other_ids; a.r = static_cast<const float*>(ratings);
    a.ob = static_cast<const float*>(other_biases);
    a.oq = static_cast<const float*>(other_features);
    a.bias = static_cast<float*>(biases); a.feat = static_cast<float*>(features);
    a.k = n_factors; a.mu = (float)global_mean; a.reg = (float)reg; a.probe = probe;
    hipStream_t s = (hipStream_t)stream;
    // k_als_wave (default); MF_ALS_KERNEL=block selects the 4-wave
    // k_als_solve (A/B probes)
    const char* ev = std::getenv("MF_ALS_KERNEL");
    if (ev && std::strcmp(ev, "block") == 0) {
        if (n_factors <= 32) return als_go<1>(a, n_entities, s);
        if (n_factors <= 64) return als_go<2>(a, n_entities, s);
        return als_go<4>(a, n_entities, s);       // 96 columns do not tile 256 lanes
    }
    if (n_factors % 4 != 0) {                     // rows not 16-byte aligned for the DMA
        if (n_factors <= 32) return als_go<1>(a, n_entities, s);
        if (n_factors <= 64) return als_go<2>(a, n_entities, s);
        return als_go<4>(a, n_entities, s);
    }
    if (n_factors <= 32) return als_go_wave<1>(a, n_entities, s);
    if (n_factors <= 64) return als_go_wave<2>(a, n_entities, s);
    return als_go_wave<4>(a, n_entities, s);
}

extern "C" int mf_als_sweep(const int64_t* entity_ptr, const int32_t* other_ids,
                            const void* ratings, int32_t n_entities, double global_mean,
                            const void* other_biases, const void* other_features,
                            void* biases, void* features, int32_t n_factors, int32_t dtype,
                            double reg, void* stream) {
    return als_sweep(entity_ptr, other_ids, ratings, n_entities, global_mean, other_biases,
                     other_features, biases, features, n_factors, dtype, reg, stream, nullptr);
}

extern "C" int mf_als_sweep_probe(const int64_t* entity_ptr, const int32_t* other_ids,
                                  const void* ratings, int32_t n_entities, double global_mean,
                                  const void* other_biases, const void* other_features,
                                  void* biases, void* features, int32_t n_factors,
                                  int32_t dtype, double reg, void* stream, int64_t* probe) {
    return als_sweep(entity_ptr, other_ids, ratings, n_entities, global_mean, other_biases,
                     other_features, biases, features, n_factors, dtype, reg, stream, probe);
}
