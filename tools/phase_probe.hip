// Microbenchmark of the sampler's VALU phases in isolation: one workgroup per CU, every CU busy,
// ITER back-to-back calls of one phase function of the kernel source, each followed by the
// workgroup barrier the sampler puts after it; s_memtime per call (max over the 4 waves of
// workgroup 0).  Phase 0 is the barrier alone.  Inputs are synthetic (LDS filled with small
// values); only the timing is meaningful.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -Iinclude \
//        tools/phase_probe.hip -o build/phase_probe        (-DPROBE_SRC=<kernel copy> for variants)
#include <hip/hip_runtime.h>
#include <stdio.h>
#ifndef PROBE_SRC
#define PROBE_SRC "../diffpose-nw_amd/csrc/dpk_kernels.hip"
#endif
#include PROBE_SRC

using namespace dpk;

enum { PH_BARRIER = 0, PH_LN, PH_ATTN, PH_CHEB, PH_GRAPH1, PH_GRAPH2, PH_COUNT };
static const char* kNames[PH_COUNT] = {"barrier", "layer_norm", "attention_mma", "cheb_prep", "graph_mma",
                                       "graph_mma<resid>"};

template <int PH>
__global__ void __launch_bounds__(NT, 1) probe(const float* W, float* out, long long* cyc, int iters) {
    __shared__ __attribute__((aligned(16))) float sm[SM_FLOATS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < SM_FLOATS; i += NT) sm[i] = ((i * 37) % 97) * 1e-2f - 0.4f;
    __syncthreads();
    float* XS = sm + SM_XS;
    float* B1 = sm + SM_B1;
    float* B2 = sm + SM_B2;
    const float* LNP = sm + SM_LNP;
    const GFrag gf = gfrag_load(W, lane);
    long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        if constexpr (PH == PH_LN) layer_norm(XS, B1, LNP, LNP + D, tid);
        else if constexpr (PH == PH_ATTN) attention_mma(B2, B1, 0x1ffffu, wave, lane);
        else if constexpr (PH == PH_CHEB) cheb_prep<true, true>(W + 1024, XS, B2, wave, lane);
        else if constexpr (PH == PH_GRAPH1) graph_mma<false>(gf, B1, B1, nullptr, wave, lane);
        else if constexpr (PH == PH_GRAPH2) graph_mma<true>(gf, B1, XS, W + 2048, wave, lane);
        __syncthreads();
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int i = tid; i < R * LDX; i += NT) s += XS[i] + B1[i];
    out[blockIdx.x * NT + tid] = s;
    if (lane == 0) cyc[blockIdx.x * NW + wave] = t1 - t0;
}

template <int PH>
static void run(const float* W, float* out, long long* cyc, int grid, int iters) {
    static long long h[4096];
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(probe<PH>, dim3(grid), dim3(NT), 0, 0, W, out, cyc, iters);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, cyc, sizeof(long long) * NW, hipMemcpyDeviceToHost);
    long long m = 0;
    for (int w = 0; w < NW; ++w) m = h[w] > m ? h[w] : m;
    printf("%-18s %8.1f cycles per call (incl. barrier)\n", kNames[PH], (double)m / iters);
}

int main() {
    const int grid = 256, iters = 200;
    float *W, *out;
    long long* cyc;
    (void)hipMalloc(&W, 4096 * sizeof(float));
    (void)hipMalloc(&out, grid * NT * sizeof(float));
    (void)hipMalloc(&cyc, grid * NW * sizeof(long long));
    static float hw[4096];
    for (int i = 0; i < 4096; ++i) hw[i] = ((i * 53) % 101) * 1e-3f - 0.05f;
    (void)hipMemcpy(W, hw, sizeof(hw), hipMemcpyHostToDevice);
    run<PH_BARRIER>(W, out, cyc, grid, iters);
    run<PH_LN>(W, out, cyc, grid, iters);
    run<PH_ATTN>(W, out, cyc, grid, iters);
    run<PH_CHEB>(W, out, cyc, grid, iters);
    run<PH_GRAPH1>(W, out, cyc, grid, iters);
    run<PH_GRAPH2>(W, out, cyc, grid, iters);
    return 0;
}
