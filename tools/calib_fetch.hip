// calib_fetch.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access shape of the SGD kernels: one 256-B row per wave-instruction
// (64 lanes x 4 B), rows picked at random from a table far larger than the
// Infinity Cache.  Known bytes: n_rows * 256 read (k_gather), n_rows * 256
// written (k_scatter).  Build: hipcc --offload-arch=gfx950 -O3 -o calib calib_fetch.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

__global__ void k_gather(const float* __restrict__ T, const int* __restrict__ idx, int n,
                         float* out) {
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
    if (w >= n) return;
    float v = T[(size_t)idx[w] * 64 + lane];
    v += __shfl_xor(v, 1);
    if (lane == 0 && v == 12345.f) out[0] = v;   // keep the load alive
}
// 16-B lanes: 16 lanes per 256-B row, 4 rows per wave instruction (the
// float4 layout of k_sgd_batch / k_sse_stream at k = 64)
__global__ void k_gather4(const float4* __restrict__ T, const int* __restrict__ idx, int n,
                          float* out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int row = t / 16, l = t & 15;
    if (row >= n) return;
    float4 v = T[(size_t)idx[row] * 16 + l];
    if (v.x + v.y + v.z + v.w == 12345.f) out[0] = v.x;
}
__global__ void k_scatter4(float4* __restrict__ T, const int* __restrict__ idx, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int row = t / 16, l = t & 15;
    if (row >= n) return;
    T[(size_t)idx[row] * 16 + l] = make_float4(l, l, l, l);
}
__global__ void k_scatter(float* __restrict__ T, const int* __restrict__ idx, int n) {
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
    if (w >= n) return;
    T[(size_t)idx[w] * 64 + lane] = (float)lane;
}

int main() {
    const size_t rows = 8u << 20;          // 8M rows x 256 B = 2 GiB table
    const int n = 1 << 20;                 // 1M rows touched = 256 MiB
    float *T, *out; int* idx;
    hipMalloc(&T, rows * 256); hipMalloc(&out, 4); hipMalloc(&idx, n * 4);
    hipMemset(T, 0, rows * 256);
    std::vector<int> h(rows);
    for (size_t j = 0; j < rows; ++j) h[j] = (int)j;
    std::mt19937 g(1); std::shuffle(h.begin(), h.end(), g);
    hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_gather, dim3(n / 4), dim3(256), 0, 0, T, idx, n, out);
        hipLaunchKernelGGL(k_scatter, dim3(n / 4), dim3(256), 0, 0, T, idx, n);
        hipLaunchKernelGGL(k_gather4, dim3(n / 16), dim3(256), 0, 0, (const float4*)T, idx, n, out);
        hipLaunchKernelGGL(k_scatter4, dim3(n / 16), dim3(256), 0, 0, (float4*)T, idx, n);
    }
    hipDeviceSynchronize();
    printf("known bytes per dispatch: gather read %zu, scatter write %zu (+ %d B of indices)\n",
           (size_t)n * 256, (size_t)n * 256, n * 4);
    return 0;
}
