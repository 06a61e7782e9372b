// Probe: lane maps and issue cost of v_mfma_f32_4x4x1_16b_f32 on gfx950, and the cost of
// mixing it with v_mfma_f32_16x16x4_f32 (the sampler's tail-row scheme).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma4_probe.hip -o build/mfma4_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// D[reg][lane] for A(l) = a_of(l), B(l) = b_of(l), C = 0
__global__ void layout(float* out, int mode) {
    const int l = threadIdx.x;
    const float a = mode == 0 ? (float)(l + 1) : 1.0f;
    const float b = mode == 0 ? 1.0f : (float)(l + 1);
    f32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[r * 64 + l] = c[r];
}

template <int NACC>
__global__ void __launch_bounds__(256, 1) rate4(float* out, long long* cyc, int iters) {
    f32x4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0, 0, 0, 0};
    float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
        asm volatile("" : "+v"(a));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// per iteration: 8 x 16x16x4 (2 row tiles x 4 j) + NT4 x 4x4x1 (tail), as in one (col tile, k-block)
template <int NT4>
__global__ void __launch_bounds__(256, 1) mixed(float* out, long long* cyc, int iters) {
    f32x4 acc[6], tacc[3];
    for (int i = 0; i < 6; ++i) acc[i] = f32x4{0, 0, 0, 0};
    for (int i = 0; i < 3; ++i) tacc[i] = f32x4{0, 0, 0, 0};
    float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[2 * c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[2 * c], 0, 0, 0);
                acc[2 * c + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[2 * c + 1], 0, 0, 0);
                if (j < NT4) tacc[c] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, tacc[c], 0, 0, 0);
            }
        }
        asm volatile("" : "+v"(a));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 6; ++i) s += acc[i][0];
    for (int i = 0; i < 3; ++i) s += tacc[i][1];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* d;
    long long* cyc;
    hipMalloc(&d, 256 * 256 * 4);
    hipMalloc(&cyc, 256 * 8);
    float h[2][256];
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h[mode], d, 256 * 4, hipMemcpyDeviceToHost);
    }
    printf("4x4x1_16b: D[reg r][lane l] = A(lane a) * B(lane b)\n");
    for (int l = 0; l < 64; ++l) {
        printf("lane %2d:", l);
        for (int r = 0; r < 4; ++r) printf("  r%d:(a%2d,b%2d)", r, (int)h[0][r * 64 + l] - 1, (int)h[1][r * 64 + l] - 1);
        printf("\n");
    }
    const int iters = 4096;
#define RATE(NA)                                                                                      \
    {                                                                                                 \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(rate4<NA>, dim3(256), dim3(256), 0, 0, d, cyc, iters); \
        hipDeviceSynchronize();                                                                       \
        long long c0;                                                                                 \
        hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);                                                \
        printf("4x4x1 NACC=%d: %.2f cyc/MFMA\n", NA, (double)c0 / ((double)iters * NA));              \
    }
    RATE(1) RATE(2) RATE(4) RATE(8)
#define MIX(N4)                                                                                       \
    {                                                                                                 \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(mixed<N4>, dim3(256), dim3(256), 0, 0, d, cyc, iters); \
        hipDeviceSynchronize();                                                                       \
        long long c0;                                                                                 \
        hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);                                                \
        printf("mixed 24x16x16x4 + %2d x 4x4x1 per iter: %.1f cyc/iter (ideal %d)\n", 3 * N4,          \
               (double)c0 / iters, 24 * 32 + 3 * N4 * 8);                                              \
    }
    MIX(0) MIX(2) MIX(4)
    return 0;
}
