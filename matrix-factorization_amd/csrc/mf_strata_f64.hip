// mf_strata_f64.hip -- double instantiations of the stratified SGD kernels
// (mf_strata.hpp), apart from the batch / SSE kernels so each compiles alone.
#include "mf_rows.hpp"
#include "mf_strata.hpp"

namespace mf {

int strata_launch_f64(const StrataParams& p) {
    StrataRun<double> r{p};
    return dispatch_rows<double>(p.k, p.kernel, r);
}

void touch_strata_f64(hipStream_t s) { hipLaunchKernelGGL(k_touch<4>, dim3(1), dim3(64), 0, s); }

}  // namespace mf
