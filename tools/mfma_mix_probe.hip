// Probe: cost of the 4 GEMM tail rows (v_mfma_f32_4x4x1_16b_f32) mixed into a QKV-shaped k-block of
// v_mfma_f32_16x16x4_f32 (2 row tiles x 9 column tiles x 4 k-steps = 72, tails 5 tiles x 4 = 20),
// for several placements.  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_mix_probe.hip -o build/mfma_mix_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define M16(acc) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0)
#define M4(acc) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc, 0, 0, 0)

// MODE 0: no tails; 1: per j, mains then the 5 tails (current); 2: all tails after the block;
// 3: all tails after the block, 2 accumulators per tail tile; 4: one tail after every ~4 mains;
// 5: tails first in the block
template <int MODE>
__global__ void __launch_bounds__(256, 1) mix(float* out, long long* cyc, int iters) {
    f32x4 acc[18], t[10];
    for (int i = 0; i < 18; ++i) acc[i] = f32x4{0, 0, 0, 0};
    for (int i = 0; i < 10; ++i) t[i] = f32x4{0, 0, 0, 0};
    float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 5) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int q = 0; q < 5; ++q) M4(t[q]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int u = 0; u < 18; ++u) {
                M16(acc[u]);
                if (MODE == 4 && (u % 4) == 3 && u / 4 < 5) M4(t[u / 4]);
            }
            if (MODE == 1) {
#pragma unroll
                for (int q = 0; q < 5; ++q) M4(t[q]);
            }
        }
        if (MODE == 2) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int q = 0; q < 5; ++q) M4(t[q]);
        }
        if (MODE == 3) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int q = 0; q < 5; ++q) M4(t[q + 5 * (j & 1)]);
        }
        asm volatile("" : "+v"(a));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 18; ++i) s += acc[i][0];
    for (int i = 0; i < 10; ++i) s += t[i][1];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* d;
    long long* cyc;
    hipMalloc(&d, 256 * 256 * 4);
    hipMalloc(&cyc, 256 * 8);
    const int iters = 2000;
#define RUN(M)                                                                                   \
    {                                                                                            \
        long long c0 = 0;                                                                        \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(mix<M>, dim3(256), dim3(256), 0, 0, d, cyc, iters); \
        hipDeviceSynchronize();                                                                  \
        hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);                                           \
        printf("mode %d: %.1f cyc per k-block (72 x 16x16x4 = 2304 ideal)\n", M, (double)c0 / iters); \
    }
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5)
    return 0;
}
