// mf_rows_f32.hip -- float instantiations of the SGD-batch and SSE kernels
// (split per dtype so the two halves compile in parallel).
#include "mf_rows.hpp"

namespace mf {

int sgd_launch_f32(const SgdParams& p) {
    SgdRun<float> r{p};
    return dispatch_rows<float>(p.k, p.kernel, r);
}

int sse_launch_f32(const SseParams& p) {
    SseRun<float> r{p};
    return dispatch_rows<float>(p.k, p.kernel, r);
}


void touch_rows_f32(hipStream_t s) { hipLaunchKernelGGL(k_touch<1>, dim3(1), dim3(64), 0, s); }

}  // namespace mf
