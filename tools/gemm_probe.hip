// Microbenchmark of the sampler's GEMM phase in isolation (tools/gemm_probe.hip).
// Includes the kernel source and times gemm_wave variants with s_memtime, one workgroup per CU,
// every CU busy, ITER back-to-back calls separated by a workgroup barrier (as in the sampler).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -Iinclude \
//        tools/gemm_probe.hip -o build/gemm_probe
#include <hip/hip_runtime.h>
// per-wave phase accounting: [0] barrier + prefetch + setup, [1] k-loop, [2] epilogue
__device__ long long g_acc[3][256 * 4];
__device__ long long g_last[256 * 4];
__device__ __forceinline__ void probe_stamp(int tag) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long t = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        if (g_last[w]) g_acc[tag][w] += t - g_last[w];
        g_last[w] = t;
    }
}
#define DPK_GEMM_HOOK(tag) do { __builtin_amdgcn_sched_barrier(0); probe_stamp(tag); __builtin_amdgcn_sched_barrier(0); } while (0)
#ifndef PROBE_SRC
#define PROBE_SRC "../diffpose-nw_amd/csrc/dpk_kernels.hip"
#endif
#include PROBE_SRC

using namespace dpk;

template <int NC, int KB, int TM>
__global__ void __launch_bounds__(NT, 1) probe(const float* W, float* out, long long* cyc, int iters) {
    __shared__ __attribute__((aligned(16))) float sm[SM_FLOATS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < SM_FLOATS; i += NT) sm[i] = ((i % 97) - 48) * 1e-2f;
    __syncthreads();
    float* A = sm + SM_B2;
    float* D = sm + SM_XS;
    const EpiArgs e{D, LDX, W + NC * KB * 256, nullptr, 0, 0, 0};
    long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        const auto pre = gemm_prefetch<NC, KB>(W, wave, lane);
        __syncthreads();
        const int half = wave >> 1;
        constexpr int NCW = NC / 2;
        if constexpr (TM == TM_MFMA4)
            gemm_wave<2, NCW, TM_MFMA4, 0, NC, KB, E_STORE>(A, LD2, W, 2 * half, (wave & 1) * NCW, col_rot<NCW>(wave), 64,
                                                            (NCW & 1) && half, lane, e, pre);
        else
            gemm_wave<2, NCW, TM, 2, NC, KB, E_STORE>(A, LD2, W, 2 * half, (wave & 1) * NCW, 0, 64 + 2 * half, false,
                                                      lane, e, pre);
        __syncthreads();
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * NT + tid] = sm[tid * 7];
}

template <int NC, int KB, int TM>
static void run(const char* name, const float* W, float* out, long long* cyc) {
    const int iters = 200, grid = 256;
    hipLaunchKernelGGL((probe<NC, KB, TM>), dim3(grid), dim3(NT), 0, 0, W, out, cyc, iters);
    hipDeviceSynchronize();
    static long long zeros[3 * 1024 + 1024];
    hipMemcpyToSymbol(HIP_SYMBOL(g_acc), zeros, sizeof(long long) * 3 * 1024);
    hipMemcpyToSymbol(HIP_SYMBOL(g_last), zeros, sizeof(long long) * 1024);
    hipLaunchKernelGGL((probe<NC, KB, TM>), dim3(grid), dim3(NT), 0, 0, W, out, cyc, iters);
    hipDeviceSynchronize();
    static long long acc[3 * 1024];
    hipMemcpyFromSymbol(acc, HIP_SYMBOL(g_acc), sizeof(acc));
    double ph[3] = {0, 0, 0};
    for (int t = 0; t < 3; ++t) {
        for (int i = 0; i < 1024; ++i) ph[t] += acc[t * 1024 + i];
        ph[t] /= 1024.0 * iters;
    }
    long long c[256];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid; ++i) s += c[i];
    const double per = s / grid / iters;
    const double ideal = 2.0 * (NC / 2) * 4 * KB * 32;
    printf("%-22s NC=%2d KB=%2d TM=%d: %8.0f cyc/call  ideal %6.0f  ratio %.2f | pre+bar %6.0f loop %6.0f epi %6.0f\n", name, NC,
           KB, TM, per, ideal, per / ideal, ph[0], ph[1], ph[2]);
}

int main() {
    float* W;
    float* out;
    long long* cyc;
    hipMalloc(&W, 4 << 20);
    {   // nonzero weights (zero operands let the chip clock higher: MI355X_MICROARCH.md DVFS notes)
        static float hw[1 << 20];
        for (int i = 0; i < (1 << 20); ++i) hw[i] = ((i * 2654435761u) >> 8 & 0xffff) * (1.0f / 65536.0f) - 0.5f;
        hipMemcpy(W, hw, 4 << 20, hipMemcpyHostToDevice);
    }
    hipMalloc(&out, 256 * NT * 4);
    hipMalloc(&cyc, 256 * 8);
#ifdef PROBE_SLOPE
    // per-k-block slope and per-call intercept: each shape at KB and multiples (4x4x1 tails on)
    run<18, 6, 2>("QKV", W, out, cyc); run<18, 12, 2>("QKV x2", W, out, cyc); run<18, 18, 2>("QKV x3", W, out, cyc);
    run<12, 6, 2>("fc1", W, out, cyc); run<12, 12, 2>("fc1 x2", W, out, cyc);
    run<6, 6, 2>("O", W, out, cyc); run<6, 12, 2>("fc2 / O x2", W, out, cyc); run<6, 18, 2>("C1/C2", W, out, cyc);
    run<6, 36, 2>("C x2", W, out, cyc);
#else
    for (int tm = 0; tm < 3; ++tm) {
        if (tm == 0) { run<18, 6, 0>("QKV", W, out, cyc); run<12, 6, 0>("fc1", W, out, cyc); run<6, 12, 0>("fc2", W, out, cyc); run<6, 18, 0>("C1/C2", W, out, cyc); run<6, 6, 0>("O", W, out, cyc); }
        if (tm == 2) { run<18, 6, 2>("QKV", W, out, cyc); run<12, 6, 2>("fc1", W, out, cyc); run<6, 12, 2>("fc2", W, out, cyc); run<6, 18, 2>("C1/C2", W, out, cyc); run<6, 6, 2>("O", W, out, cyc); }
    }
#endif
    return 0;
}
