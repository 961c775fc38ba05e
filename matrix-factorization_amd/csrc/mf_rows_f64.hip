// mf_rows_f64.hip -- double instantiations of the SGD-batch and SSE kernels
// (split per dtype so the two halves compile in parallel).
#include "mf_rows.hpp"

namespace mf {

int sgd_launch_f64(const SgdParams& p) {
    SgdRun<double> r{p};
    return dispatch_rows<double>(p.k, p.kernel, r);
}

int sse_launch_f64(const SseParams& p) {
    SseRun<double> r{p};
    return dispatch_rows<double>(p.k, p.kernel, r);
}


void touch_rows_f64(hipStream_t s) { hipLaunchKernelGGL(k_touch<2>, dim3(1), dim3(64), 0, s); }

}  // namespace mf
