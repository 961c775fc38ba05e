// mf_strata_f32.hip -- float instantiations of the stratified SGD kernels
// (mf_strata.hpp), apart from the batch / SSE kernels so each compiles alone.
#include "mf_rows.hpp"
#include "mf_strata.hpp"

namespace mf {

int strata_launch_f32(const StrataParams& p) {
    StrataRun<float> r{p};
    return dispatch_rows<float>(p.k, p.kernel, r);
}

void touch_strata_f32(hipStream_t s) { hipLaunchKernelGGL(k_touch<3>, dim3(1), dim3(64), 0, s); }

}  // namespace mf
