// mf_common.hpp -- shared device helpers for the gfx950 kernels of libmf_hip.
//
// Layout conventions:
//   * factor rows are row-major, n_factors contiguous values per row;
//   * a rating is handled by a GROUP of GS lanes (GS = min(KPAD, 64)), lane l
//     of the group owns factors f = l, l + GS, ... (V = KPAD / GS values);
//     R = 64 / GS ratings share one wave64 instruction;
//   * dot products / squared distances are reduced inside the group by an
//     xor butterfly, which leaves the bit-identical sum in every lane.
#pragma once

#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdint.h>

#include "../../include/mf_hip.h"

namespace mf {

constexpr int kWave = 64;
constexpr int kBlock = 256;               // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kMaxFactors = 1024;

void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

#define MF_HIP_CHECK(expr)                                   \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return ::mf::hip_fail(_e, #expr); \
    } while (0)

// Bijective XCD-aware block remap (guide T1).  Workgroups b, b+8, b+16, ...
// are dealt to the same XCD; give that XCD a contiguous range of tiles so
// neighbouring tiles (which touch neighbouring item rows after the colour
// scheduler's item sort) share its L2.
__device__ __forceinline__ int64_t xcd_swizzle(int64_t b, int64_t nb) {
    constexpr int64_t X = 8;
    const int64_t x = b % X, w = b / X;
    const int64_t q = nb / X, r = nb % X;
    const int64_t start = x * q + (x < r ? x : r);
    return start + w;
}

// ---- group sums on DPP (no LDS crossbar traffic) ------------------------
// Row (16-lane) all-reduce: quad_perm xor1, quad_perm xor2, row_half_mirror,
// row_mirror.  Each step adds two values that are uniform over the lanes
// being combined, so every lane of a row ends with the bit-identical sum.
// 64 lanes: + row_bcast:15 / row_bcast:31, then lane 63 is read as a scalar.
// 32 lanes: + one xor-16 swap (ds_bpermute).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(dpp_i<CTRL, ROWS>(__float_as_int(v)));
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i<CTRL, ROWS>((int)(b & 0xffffffffLL));
    const int hi = dpp_i<CTRL, ROWS>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int kDppXor1 = 0xB1;          // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;          // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;   // row_half_mirror
constexpr int kDppMirror = 0x140;       // row_mirror
constexpr int kDppBcast15 = 0x142;      // row_bcast:15
constexpr int kDppBcast31 = 0x143;      // row_bcast:31

template <typename T>
__device__ __forceinline__ T row_sum(T v) {
    v = v + dpp<kDppXor1>(v);
    v = v + dpp<kDppXor2>(v);
    v = v + dpp<kDppHalfMirror>(v);
    v = v + dpp<kDppMirror>(v);
    return v;
}

__device__ __forceinline__ float lane63(float v) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ double lane63(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int GS, typename T>
__device__ __forceinline__ T group_sum(T v) {
    static_assert(GS == 1 || GS == 2 || GS == 4 || GS == 8 || GS == 16 || GS == 32 || GS == 64,
                  "group of 1..64 lanes (power of two)");
    if constexpr (GS < 16) {
        if constexpr (GS >= 2) v = v + dpp<kDppXor1>(v);
        if constexpr (GS >= 4) v = v + dpp<kDppXor2>(v);
        if constexpr (GS >= 8) v = v + dpp<kDppHalfMirror>(v);
        return v;
    }
    v = row_sum(v);
    if constexpr (GS == 32) {
        v = v + __shfl_xor(v, 16, kWave);
    } else if constexpr (GS == 64) {
        v = v + dpp<kDppBcast15, 0xa>(v);      // rows 1, 3 += rows 0, 2
        v = v + dpp<kDppBcast31, 0xc>(v);      // rows 2, 3 += rows 0 + 1
        v = lane63(v);                         // (R3 + R2) + (R1 + R0), uniform
    }
    return v;
}

// Whole-wave sum for integer/FP64 partials (block reductions; not hot).
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) v = v + __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ int bcast_i32(int v, int src) {
    return __shfl(v, src, kWave);
}
__device__ __forceinline__ float bcast_f(float v, int src) {
    return __shfl(v, src, kWave);
}
__device__ __forceinline__ double bcast_f(double v, int src) {
    return __shfl(v, src, kWave);
}

// wave-uniform source lane (GS == 64): v_readlane, no LDS crossbar traffic
__device__ __forceinline__ int rl_i32(int v, int src) {
    return __builtin_amdgcn_readlane(v, src);
}
__device__ __forceinline__ float rl_f(float v, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
__device__ __forceinline__ double rl_f(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// W consecutive values of a row moved by one lane (16 B for float4/double2)
template <typename T, int W> struct VecOf;
template <typename T> struct VecOf<T, 1> { using type = T; };
template <typename T> struct VecOf<T, 2> { typedef T type __attribute__((ext_vector_type(2))); };
template <typename T> struct VecOf<T, 4> { typedef T type __attribute__((ext_vector_type(4))); };

template <typename T> __device__ __forceinline__ T dexp(T x);
template <> __device__ __forceinline__ float dexp<float>(float x) { return expf(x); }
template <> __device__ __forceinline__ double dexp<double>(double x) { return exp(x); }

// Kernel-family parameters, already converted to the compute type.
template <typename T>
struct Hyper {
    T mu, lr, reg, gamma, a, c, lo, hi;
};

template <typename T>
inline Hyper<T> make_hyper(double mu, double lr, double reg, double gamma,
                           double min_rating, double max_rating) {
    Hyper<T> h;
    h.mu = (T)mu; h.lr = (T)lr; h.reg = (T)reg; h.gamma = (T)gamma;
    h.a = (T)min_rating; h.c = (T)(max_rating - min_rating);
    h.lo = (T)min_rating; h.hi = (T)max_rating;
    return h;
}

inline int kpad_of(int k) {
    int kp = 16;
    while (kp < k) kp <<= 1;
    return kp;
}

// MF_LAUNCH_TRACE=1: host time of the launcher's runtime calls on stderr
// (diagnostic: where a first epoch's host time goes)
struct LaunchTrace {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    static bool on() {
        static const bool v = std::getenv("MF_LAUNCH_TRACE") != nullptr;
        return v;
    }
    void mark(const char* what) const {
        if (!on()) return;
        const double ms = std::chrono::duration<double, std::milli>(
                              std::chrono::steady_clock::now() - t0).count();
        std::fprintf(stderr, "[mf launch] %-24s %9.3f ms\n", what, ms);
    }
};

// One empty kernel per translation unit (U: the unit's number).  HIP loads a
// unit's code object at the first launch of one of its kernels -- ~6-10 ms
// for the large units (MF_LAUNCH_TRACE, profiles/r05) -- so mf_warmup
// launches every unit's k_touch<U> once per device up front, and an engine's
// first epoch does not pay it.
template <int U>
__global__ void k_touch() {}
void touch_rows_f32(hipStream_t s);
void touch_rows_f64(hipStream_t s);
void touch_strata_f32(hipStream_t s);
void touch_strata_f64(hipStream_t s);
void touch_bias(hipStream_t s);
void touch_topk(hipStream_t s);
void touch_als(hipStream_t s);

}  // namespace mf
