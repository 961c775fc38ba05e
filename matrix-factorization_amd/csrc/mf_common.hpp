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

template <int GS, typename T>
__device__ __forceinline__ T group_sum(T v) {
#pragma unroll
    for (int o = 1; o < GS; o <<= 1) v = v + __shfl_xor(v, o, kWave);
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

}  // namespace mf
