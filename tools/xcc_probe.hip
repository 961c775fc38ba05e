// xcc_probe.hip -- which XCD (HW_REG_XCC_ID) runs each workgroup, over
// several launches: checks the round-robin dealing and its per-launch offset.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    if (threadIdx.x == 0) out[blockIdx.x] = (int)(v & 0xf);
}
int main() {
    const int nb = 4096;
    int* d; (void)hipMalloc(&d, nb * 4);
    int h[nb];
    for (int rep = 0; rep < 6; ++rep) {
        hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, d);
        (void)hipMemcpy(h, d, nb * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int b = 8; b < nb; ++b) bad += h[b] != h[b % 8];
        printf("launch %d: xcc(b=0..15) =", rep);
        for (int b = 0; b < 16; ++b) printf(" %d", h[b]);
        printf("  | blocks not matching b%%8 rule: %d\n", bad);
    }
    return 0;
}
