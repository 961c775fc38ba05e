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
#include <utility>

#include "mf_common.hpp"

namespace mf {

constexpr int kAlsThreads = 256;
constexpr int kAlsChunk = 64;        // other-side rows per LDS chunk (32 K-steps)
constexpr int kAlsMaxFactors = 128;

using f32x16 = __attribute__((ext_vector_type(16))) float;

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
    if (n_factors <= 32) return als_go<1>(a, n_entities, s);
    if (n_factors <= 64) return als_go<2>(a, n_entities, s);
    return als_go<4>(a, n_entities, s);           // 96 columns do not tile 256 lanes
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
