// Probe: __builtin_amdgcn_permlane{16,32}_swap on gfx950 — distinct operands, identical
// operands, and identical operands laundered through an empty asm (row all-reduce use).
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ float sum4(float v, bool launder) {
    unsigned u = __builtin_bit_cast(unsigned, v), u2 = u;
    if (launder) asm volatile("s_nop 4" : "+v"(u2));
    auto r = __builtin_amdgcn_permlane32_swap(u, u2, false, false);
    float a = __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
    unsigned ua = __builtin_bit_cast(unsigned, a), ua2 = ua;
    if (launder) asm volatile("s_nop 4" : "+v"(ua2));
    auto r2 = __builtin_amdgcn_permlane16_swap(ua, ua2, false, false);
    return __builtin_bit_cast(float, r2[0]) + __builtin_bit_cast(float, r2[1]);
}
__device__ float sum4_asm(float v) {
    float a = v, b = v;
    asm volatile("s_nop 4\n v_permlane32_swap_b32 %0, %1\n s_nop 4" : "+v"(a), "+v"(b));
    float s1 = a + b, c = s1, d = s1;
    asm volatile("s_nop 4\n v_permlane16_swap_b32 %0, %1\n s_nop 4" : "+v"(c), "+v"(d));
    return c + d;
}
__global__ void k(unsigned* o, float* f) {
    const unsigned l = threadIdx.x;
    auto a = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
    o[l] = a[0]; o[64 + l] = a[1];
    f[l] = sum4((float)l, false);
    f[64 + l] = sum4((float)l, true);
    f[128 + l] = sum4_asm((float)l);
}
int main() {
    unsigned* d; float* fd; hipMalloc(&d, 128 * 4); hipMalloc(&fd, 192 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, fd);
    unsigned h[128]; float f[192];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost); hipMemcpy(f, fd, sizeof(f), hipMemcpyDeviceToHost);
    printf("p32[0]:"); for (int l = 0; l < 64; l += 8) printf(" %u", h[l]); printf("\n");
    printf("sum4 same-operand  :"); for (int l = 0; l < 64; l += 8) printf(" %.0f", f[l]); printf("   (expect l%%16*4+96)\n");
    printf("sum4 laundered     :"); for (int l = 0; l < 64; l += 8) printf(" %.0f", f[64 + l]); printf("\n");
    printf("sum4 asm           :"); for (int l = 0; l < 64; l += 8) printf(" %.0f", f[128 + l]); printf("\n");
    return 0;
}
