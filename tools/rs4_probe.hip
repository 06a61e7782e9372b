// Probe: 4-register reduce-scatter over the 4 lane rows (16 lanes each) with
// v_permlane32_swap / v_permlane16_swap, as the GEMM tail epilogue uses it (dpk_kernels.hip
// rs4rows): lane l must end with sum over rows of register (l>>4) at position l&15.
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ float rs4(float v0, float v1, float v2, float v3) {
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(v0), "+v"(v2));
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(v1), "+v"(v3));
    float a = v0 + v2, b = v1 + v3;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return a + b;
}
__global__ void k(float* o) {
    const int l = threadIdx.x;
    // value of register r at lane l: r*1000 + (l>>4)*100 + (l&15) -> sum over rows = 4*(r*1000 + (l&15)) + 600
    float v[4];
    for (int r = 0; r < 4; ++r) v[r] = r * 1000 + (l >> 4) * 100 + (l & 15);
    o[l] = rs4(v[0], v[1], v[2], v[3]);
}
int main() {
    float* d;
    hipMalloc(&d, 64 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    float h[64];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const float want = 4.f * ((l >> 4) * 1000 + (l & 15)) + 600;
        if (h[l] != want) { if (bad < 8) printf("lane %d got %.0f want %.0f\n", l, h[l], want); ++bad; }
    }
    printf("rs4: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    return 0;
}
