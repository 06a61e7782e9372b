// Probe: do fp32 MFMA work of one wave and VALU work of ANOTHER wave on the same SIMD overlap?
// (The sampler runs one wave per SIMD, and there a wave's own VALU work and its f32 MFMAs add;
// DESIGN.md §6.  Two co-resident workgroups per CU would only pay if the answer here is yes.)
// One 512-thread workgroup per CU: waves 0-3 (one per SIMD) are "MFMA waves" running QKV-shaped
// k-blocks of v_mfma_f32_16x16x4_f32 (18 independent accumulators x 4 k-steps); waves 4-7 (the
// SIMD partners) are "VALU waves" running either 8 independent fma chains (issue-bound), one
// dependent chain (latency-bound) or an LDS read + fma + LDS write loop.  Each configuration runs
// alone and together; "overlap" means together ~ max(alone) rather than the sum.
// Build: hipcc --offload-arch=gfx950 -O3 tools/overlap_probe.hip -o build/overlap_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// MK: the MFMA of the "MFMA waves": 0 = v_mfma_f32_16x16x4_f32 (fp32 mode), 1 =
// v_mfma_f32_16x16x32_f16 (split-fp16 mode; 8x the k per instruction)
template <int MK>
__device__ __forceinline__ f32x4 mma(float a, float b, f16x8 ah, f16x8 bh, f32x4 c) {
    if constexpr (MK == 0) return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
}

// WHO: 1 = MFMA waves only, 2 = VALU waves only, 3 = both.  VK: 0 = 8 independent chains,
// 1 = one dependent chain, 2 = LDS round trips.  SAME: MFMA and VALU work in the same wave
// (waves 0-3 only), interleaved per k-step.
template <int WHO, int VK, bool SAME, int MK = 0>
__global__ void __launch_bounds__(512, 1) probe(float* out, long long* cyc, int mfma_iters, int valu_iters) {
    __shared__ float lds[512 * 4];
    const int wave = threadIdx.x >> 6;
    const bool mw = SAME ? wave < 4 : wave < 4, vw = SAME ? wave < 4 : wave >= 4;
    float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
    f16x8 ah, bh;
    for (int i = 0; i < 8; ++i) {
        ah[i] = (_Float16)(a + i * 1e-2f);
        bh[i] = (_Float16)(b - i * 1e-2f);
    }
    f32x4 acc[18];
    for (int i = 0; i < 18; ++i) acc[i] = f32x4{0, 0, 0, 0};
    float v[8];
    for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * (i + 1) * 1e-4f;
    lds[threadIdx.x] = a;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    const bool run_m = (WHO & 1) && mw, run_v = (WHO & 2) && vw;
    if (SAME) {
        if (run_m || run_v) {
            for (int it = 0; it < mfma_iters; ++it) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
#pragma unroll
                    for (int u = 0; u < 18; ++u) {
                        if (run_m) acc[u] = mma<MK>(a, b, ah, bh, acc[u]);
                        if (run_v && (u & 1)) {
#pragma unroll
                            for (int i = 0; i < 8; ++i) v[i] = fmaf(v[i], 0.999f, 1e-3f);
                        }
                    }
                }
                asm volatile("" : "+v"(a), "+v"(ah));
            }
        }
    } else {
        if (run_m) {
            for (int it = 0; it < mfma_iters; ++it) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int u = 0; u < 18; ++u) acc[u] = mma<MK>(a, b, ah, bh, acc[u]);
                asm volatile("" : "+v"(a), "+v"(ah));
            }
        }
        if (run_v) {
            if (VK == 0) {
                for (int it = 0; it < valu_iters; ++it) {
#pragma unroll
                    for (int r = 0; r < 16; ++r)
#pragma unroll
                        for (int i = 0; i < 8; ++i) v[i] = fmaf(v[i], 0.999f, 1e-3f);
                }
            } else if (VK == 1) {
                for (int it = 0; it < valu_iters; ++it) {
#pragma unroll
                    for (int r = 0; r < 128; ++r) v[0] = fmaf(v[0], 0.999f, 1e-3f);
                }
            } else {
                const int base = (threadIdx.x & 255) * 4;
                for (int it = 0; it < valu_iters; ++it) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        float x = lds[(base + r) & 2047];
                        x = fmaf(x, 0.999f, v[r]);
                        lds[(base + r + 512) & 2047] = x;
                        v[r] = x;
                    }
                }
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 18; ++i) s += acc[i][0];
    for (int i = 0; i < 8; ++i) s += v[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

static long long run_max(void (*k)(float*, long long*, int, int), float* d, long long* cyc, int mi, int vi) {
    static long long h[256 * 8];
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, d, cyc, mi, vi);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    long long m = 0;
    for (int i = 0; i < 8; ++i) m = h[i] > m ? h[i] : m;   // workgroup 0: slowest wave
    return m;
}

int main() {
    float* d;
    long long* cyc;
    hipMalloc(&d, 256 * 512 * 4);
    hipMalloc(&cyc, 256 * 8 * 8);
    const int mi = 200;
    // VALU iteration counts sized so each VALU-only run is near the MFMA-only run
    const int vi[3] = {900, 450, 2000};
#define ROW(VK, MK, MI)                                                                                   \
    {                                                                                                     \
        const long long m = run_max(probe<1, VK, false, MK>, d, cyc, MI, vi[VK]);                        \
        const long long v = run_max(probe<2, VK, false, MK>, d, cyc, MI, vi[VK]);                         \
        const long long b = run_max(probe<3, VK, false, MK>, d, cyc, MI, vi[VK]);                         \
        printf("%s, valu kind %d (%s): mfma alone %lld, valu alone %lld, both %lld cycles -> %s (sum %lld, max %lld)\n", \
               MK ? "f16 16x16x32" : "f32 16x16x4", VK, VK == 0 ? "8 independent fma chains" : VK == 1 ? "1 dependent chain" : "lds read+fma+write", \
               m, v, b, b < (m + v) * 0.75 ? "OVERLAP" : "ADD", m + v, m > v ? m : v);                    \
    }
    ROW(0, 0, mi) ROW(1, 0, mi) ROW(2, 0, mi)
    // 16x16x32 f16 is 8 passes (vs 8 for 16x16x4 f32 too, but 8x the k): same iteration count
    ROW(0, 1, mi) ROW(1, 1, mi) ROW(2, 1, mi)
    {
        const long long m = run_max(probe<1, 0, true>, d, cyc, mi, 0);
        const long long v = run_max(probe<2, 0, true>, d, cyc, mi, 0);
        const long long b = run_max(probe<3, 0, true>, d, cyc, mi, 0);
        printf("same wave, 8 fma per 2 MFMAs: mfma alone %lld, valu alone %lld, interleaved %lld cycles\n", m, v, b);
    }
    printf("ideal MFMA-only: %d k-blocks x 72 x 32 cycles = %d\n", mi, mi * 72 * 32);
    return 0;
}
