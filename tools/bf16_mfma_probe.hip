// tools/bf16_mfma_probe.hip -- numerics of v_mfma_f32_32x32x16_bf16 on this
// GPU, for k_topk_mw's error bound (mf_topk.hip): are bf16 x bf16 products
// exact, how are the 16 products and the f32 accumulator summed (rounding),
// and the worst |mfma - exact| / sum |a b| over random data.
// Build: hipcc -O2 --offload-arch=gfx950 tools/bf16_mfma_probe.hip -o tools/bf16_mfma_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// A: 32 x 16 (row-major floats, bf16-exact), B: 16 x 32, C: 32 x 32 (in / out)
__global__ void k_mm(const float* A, const float* B, float* C) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)A[r * 16 + 8 * h + j];
        b[j] = (__bf16)B[(8 * h + j) * 32 + r];
    }
    f32x16 c;
    for (int i = 0; i < 16; ++i) c[i] = C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 16; ++i) C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}

static float bf(float x) {                    // round to bf16 (RNE), as float
    unsigned u;
    std::memcpy(&u, &x, 4);
    u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
    float y;
    std::memcpy(&y, &u, 4);
    return y;
}

static void run(const std::vector<float>& A, const std::vector<float>& B, std::vector<float>& C) {
    float *dA, *dB, *dC;
    hipMalloc(&dA, 4 * 512); hipMalloc(&dB, 4 * 512); hipMalloc(&dC, 4 * 1024);
    hipMemcpy(dA, A.data(), 4 * 512, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 4 * 512, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), 4 * 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mm, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(C.data(), dC, 4 * 1024, hipMemcpyDeviceToHost);
    hipFree(dA); hipFree(dB); hipFree(dC);
}

int main() {
    std::vector<float> A(512), B(512), C(1024);
    // 1. products exact?  (1 + 2^-7)^2 = 1 + 2^-6 + 2^-14, 16 of them
    const float x = 1.0f + 0x1p-7f;
    for (auto& v : A) v = x;
    for (auto& v : B) v = x;
    for (auto& v : C) v = 0.f;
    run(A, B, C);
    printf("products: got %.10f, exact %.10f (products rounded to bf16: %.10f)\n", C[0],
           16.0 + 0x1p-2 + 0x1p-10, 16.0 + 0x1p-2);
    // 2. rounding of the sum: C = 2^20, sixteen products of 2^-5 * (1 + ...)
    for (int t = 0; t < 3; ++t) {
        const float p = t == 0 ? 0x1p-5f : t == 1 ? 0x1p-6f * 1.5f : 0x1p-8f * 3.0f;
        for (auto& v : A) v = p;
        for (auto& v : B) v = 1.0f;
        for (auto& v : C) v = 0x1p20f;
        run(A, B, C);
        printf("sum onto 2^20 of 16 x %.9g: got %.9f exact %.9f\n", p, C[0],
               (double)0x1p20 + 16.0 * p);
    }
    // 3. random: worst |mfma - exact| / (sum |a b| + |c|) and in units of 2^-24
    std::mt19937 g(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    double worst = 0, worst_nc = 0;
    for (int rep = 0; rep < 2000; ++rep) {
        for (auto& v : A) v = bf(nd(g) * (rep % 3 == 0 ? 1e-3f : 1.f));
        for (auto& v : B) v = bf(nd(g));
        const bool withc = rep % 2;
        for (auto& v : C) v = withc ? nd(g) : 0.f;
        std::vector<float> C0 = C;
        run(A, B, C);
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) {
                double ex = C0[i * 32 + j], ab = fabs(C0[i * 32 + j]);
                for (int kk = 0; kk < 16; ++kk) {
                    ex += (double)A[i * 16 + kk] * B[kk * 32 + j];
                    ab += fabs((double)A[i * 16 + kk] * B[kk * 32 + j]);
                }
                const double e = fabs(C[i * 32 + j] - ex) / ab / 0x1p-24;
                if (withc) worst = fmax(worst, e);
                else worst_nc = fmax(worst_nc, e);
            }
    }
    printf("random: worst |err| / (sum|ab| + |c|) = %.3f x 2^-24 (with C), %.3f x 2^-24 (C = 0)\n",
           worst, worst_nc);
    return 0;
}
