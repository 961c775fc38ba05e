// mf_dispatch.hpp -- runtime (dtype, n_factors, kernel) -> template dispatch.
#pragma once

#include "mf_common.hpp"

namespace mf {

// ------------------------------------------------------------ dispatch
// Calls F.template run<T, GS, V, KERN>() for the runtime (dtype, k, kernel).
template <typename F>
inline int dispatch(int dtype, int k, int kernel, F&& f) {
    if (k < 0 || k > kMaxFactors) {
        set_error("n_factors=%d outside [0, %d]", k, kMaxFactors);
        return MF_ERR_INVALID;
    }
    if (kernel < MF_LINEAR || kernel > MF_RBF) {
        set_error("unknown kernel code %d", kernel);
        return MF_ERR_INVALID;
    }
    if (dtype != MF_F32 && dtype != MF_F64) {
        set_error("unknown dtype code %d", dtype);
        return MF_ERR_INVALID;
    }
    const int kp = kpad_of(k);
#define MF_KCASE(T, KP, GS, V)                                                   \
    if (kp == KP) {                                                              \
        if (kernel == MF_LINEAR) return f.template run<T, GS, V, MF_LINEAR>();   \
        if (kernel == MF_SIGMOID) return f.template run<T, GS, V, MF_SIGMOID>(); \
        return f.template run<T, GS, V, MF_RBF>();                               \
    }
#define MF_TCASES(T)                \
    MF_KCASE(T, 16, 16, 1)          \
    MF_KCASE(T, 32, 32, 1)          \
    MF_KCASE(T, 64, 64, 1)          \
    MF_KCASE(T, 128, 64, 2)         \
    MF_KCASE(T, 256, 64, 4)         \
    MF_KCASE(T, 512, 64, 8)         \
    MF_KCASE(T, 1024, 64, 16)
    if (dtype == MF_F32) { MF_TCASES(float) }
    else { MF_TCASES(double) }
#undef MF_TCASES
#undef MF_KCASE
    set_error("internal: no kernel for n_factors=%d", k);
    return MF_ERR_INVALID;
}

}  // namespace mf
