// Microbenchmark: cycles per v_mfma_f32_16x16x4_f32 for one wave per SIMD (4 waves/CU),
// with NACC independent accumulators, operands in registers; and a variant that streams
// B fragments from global memory / A fragments from LDS like the sampler GEMM.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o build/mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void __launch_bounds__(256, 1) probe_reg(float* out, long long* cyc, int iters) {
    f32x4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0, 0, 0, 0};
    float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
        asm volatile("" : "+v"(a));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// streaming variant: NR A-fragments (LDS) x NCW B-fragments (global, 1 KiB coalesced each)
template <int NR, int NCW, int NBLK = 8 * NCW * 4>
__global__ void __launch_bounds__(256, 1) probe_stream(const f32x4* __restrict__ B, float* out, long long* cyc, int iters) {
    __shared__ float lds[68 * 104];
    for (int i = threadIdx.x; i < 68 * 104; i += 256) lds[i] = i * 1e-5f;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    f32x4 acc[NR][NCW];
    for (int i = 0; i < NR; ++i)
        for (int c = 0; c < NCW; ++c) acc[i][c] = f32x4{0, 0, 0, 0};
    const f32x4* Bl = B + (size_t)wave * NCW * 64 + lane;
    int aoff[NR];
    for (int i = 0; i < NR; ++i) aoff[i] = ((i * 16 + (lane & 15)) % 68) * 104 + (lane >> 4) * 4;
    long long t0 = __builtin_amdgcn_s_memtime();
    f32x4 b0[NCW], b1[NCW], a0[NR], a1[NR];
    for (int c = 0; c < NCW; ++c) b0[c] = Bl[c * 64];
    for (int i = 0; i < NR; ++i) a0[i] = *(const f32x4*)(lds + aoff[i]);
    for (int it = 0; it < iters; it += 2) {
        for (int c = 0; c < NCW; ++c) b1[c] = Bl[((c + (it + 1) * NCW * 4) % NBLK) * 64];
        for (int i = 0; i < NR; ++i) a1[i] = *(const f32x4*)(lds + aoff[i] + ((it + 1) % 6) * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < NR; ++i)
#pragma unroll
                for (int c = 0; c < NCW; ++c) acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[i][j], b0[c][j], acc[i][c], 0, 0, 0);
        for (int c = 0; c < NCW; ++c) b0[c] = Bl[((c + (it + 2) * NCW * 4) % NBLK) * 64];
        for (int i = 0; i < NR; ++i) a0[i] = *(const f32x4*)(lds + aoff[i] + ((it + 2) % 6) * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < NR; ++i)
#pragma unroll
                for (int c = 0; c < NCW; ++c) acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][j], b1[c][j], acc[i][c], 0, 0, 0);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < NR; ++i)
        for (int c = 0; c < NCW; ++c) s += acc[i][c][0] + acc[i][c][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(const char* name, K kernel, int nmfma_per_iter, int iters, int grid, const f32x4* B, bool stream) {
    float* out;
    long long* cyc;
    hipMalloc(&out, grid * 256 * 4);
    hipMalloc(&cyc, grid * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (stream)
            hipLaunchKernelGGL(kernel, dim3(grid), dim3(256), 0, 0, B, out, cyc, iters);
        else
            hipLaunchKernelGGL(kernel, dim3(grid), dim3(256), 0, 0, (const f32x4*)nullptr, out, cyc, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c[4];
    hipMemcpy(c, cyc, 32, hipMemcpyDeviceToHost);
    double per = (double)c[0] / ((double)iters * nmfma_per_iter);
    double wall_cyc = ms * 1e-3 * 2.4e9 / ((double)iters * nmfma_per_iter);
    printf("%-28s grid %4d: s_memtime %.1f cyc/MFMA, wall %.3f ms (%.1f cyc@2.4GHz/MFMA)\n", name, grid, per, ms, wall_cyc);
    hipFree(out);
    hipFree(cyc);
}

template <int NACC>
__global__ void probe_reg_wrap(const f32x4*, float* out, long long* cyc, int iters) {}

int main() {
    f32x4* B;
    hipMalloc(&B, 64 << 20);
    hipMemset(B, 0, 64 << 20);
    const int iters = 4096;
    auto reg1 = [](const f32x4*, float* o, long long* c, int it) {};
    (void)reg1;
    // register-only
    {
        float* out; long long* cyc; hipMalloc(&out, 256 * 256 * 4); hipMalloc(&cyc, 256 * 8);
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
#define REG(NA)                                                                                  \
        for (int grid : {1, 256}) {                                                              \
            for (int rep = 0; rep < 2; ++rep) {                                                  \
                hipEventRecord(e0);                                                              \
                hipLaunchKernelGGL(probe_reg<NA>, dim3(grid), dim3(256), 0, 0, out, cyc, iters); \
                hipEventRecord(e1); hipEventSynchronize(e1);                                     \
            }                                                                                    \
            float ms; hipEventElapsedTime(&ms, e0, e1); long long c0;                             \
            hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);                                       \
            printf("reg NACC=%-3d grid %4d: s_memtime %.1f cyc/MFMA, wall %.3f ms\n", NA, grid,  \
                   (double)c0 / ((double)iters * NA), ms);                                       \
        }
        REG(1) REG(2) REG(4) REG(8) REG(24)
    }
    run("stream NR=4 NCW=6", probe_stream<4, 6>, 4 * 4 * 6, iters, 256, B, true);
    run("stream NR=4 NCW=2", probe_stream<4, 2>, 4 * 4 * 2, iters, 256, B, true);
    run("stream NR=1 NCW=6", probe_stream<1, 6>, 4 * 1 * 6, iters, 256, B, true);
    run("stream NR=4 NCW=6 516KB", probe_stream<4, 6, 516>, 4 * 4 * 6, iters, 256, B, true);
    run("stream NR=4 NCW=6 2.6MB", probe_stream<4, 6, 2600>, 4 * 4 * 6, iters, 256, B, true);
    run("stream NR=4 NCW=2 2.6MB", probe_stream<4, 2, 2600>, 4 * 4 * 2, iters, 256, B, true);
    run("stream NR=1 NCW=6 2.6MB", probe_stream<1, 6, 2600>, 4 * 1 * 6, iters, 256, B, true);
    run("stream NR=4 NCW=6 (1 WG)", probe_stream<4, 6>, 4 * 4 * 6, iters, 1, B, true);
    return 0;
}
