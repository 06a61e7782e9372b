// Cycle cost of the half-width MFMAs the gemm modes 1/2 use (gemmh_pass), one wave per SIMD, back to back:
// v_mfma_f32_16x16x32_{bf16,f16}, v_mfma_f32_4x4x4_16b_{bf16,f16} (the tail rows), alone and mixed.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_h_probe.hip -o build/mfma_h_probe && build/mfma_h_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
constexpr int IT = 2000;
template <int KIND>
__global__ void __launch_bounds__(256) probe(float* out, long long* cyc, float seed) {
    f16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(seed * (threadIdx.x + i)); b[i] = (_Float16)(seed * i); }
    f32x4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0, 0, 0, 0};
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < IT; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc[i], 0, 0, 0);
            if constexpr (KIND == 1) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
            if constexpr (KIND == 2) acc[i] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(__builtin_bit_cast(s16x4, __builtin_shufflevector(a, a, 0, 1, 2, 3)), __builtin_bit_cast(s16x4, __builtin_shufflevector(b, b, 0, 1, 2, 3)), acc[i], 0, 0, 0);
            if constexpr (KIND == 3) acc[i] = __builtin_amdgcn_mfma_f32_4x4x4f16(__builtin_shufflevector(a, a, 0, 1, 2, 3), __builtin_shufflevector(b, b, 0, 1, 2, 3), acc[i], 0, 0, 0);
            if constexpr (KIND == 4) {   // 3 x 16x16x32 bf16 + 1 x 4x4x4 (a QKV-shaped k-block mix, 6:2)
                if (i < 6) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc[i], 0, 0, 0);
                else acc[i] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(__builtin_bit_cast(s16x4, __builtin_shufflevector(a, a, 0, 1, 2, 3)), __builtin_bit_cast(s16x4, __builtin_shufflevector(b, b, 0, 1, 2, 3)), acc[i], 0, 0, 0);
            }
            if constexpr (KIND == 5) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(seed, seed * 2.f, acc[i], 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    float* o; long long* c;
    hipMalloc(&o, 256 * 256 * 4); hipMalloc(&c, 256 * 8);
    const char* names[] = {"16x16x32 bf16", "16x16x32 f16", "4x4x4 bf16_1k", "4x4x4 f16", "6x 16x16x32 bf16 + 2x 4x4x4 bf16", "16x16x4 f32"};
    auto run = [&](auto k, int kind) {
        hipLaunchKernelGGL(k, dim3(256), dim3(256), 0, 0, o, c, 0.001f);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(k, dim3(256), dim3(256), 0, 0, o, c, 0.001f);
        long long h[256]; hipMemcpy(h, c, 256 * 8, hipMemcpyDeviceToHost);
        double m = 0; for (int i = 0; i < 256; ++i) m += h[i]; m /= 256;
        // s_memtime counts at the 100 MHz reference on gfx950? report raw and per-MFMA
        printf("%-36s %.3f s_memtime ticks per MFMA\n", names[kind], m / (IT * 8.0));
    };
    run(probe<0>, 0); run(probe<1>, 1); run(probe<2>, 2); run(probe<3>, 3); run(probe<4>, 4); run(probe<5>, 5);
    return 0;
}
