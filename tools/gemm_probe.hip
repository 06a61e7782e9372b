// Microbenchmark of the sampler's GEMM phase in isolation (tools/gemm_probe.hip).
// Includes the kernel source and times gemm_wave variants with s_memtime, one workgroup per CU,
// every CU busy, ITER back-to-back calls separated by a workgroup barrier (as in the sampler).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -Iinclude \
//        tools/gemm_probe.hip -o build/gemm_probe
#include "../diffpose-nw_amd/csrc/dpk_kernels.hip"

using namespace dpk;

template <int NC, int KB, int TM>
__global__ void __launch_bounds__(NT, 1) probe(const float* W, float* out, long long* cyc, int iters) {
    __shared__ __attribute__((aligned(16))) float sm[SM_FLOATS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < SM_FLOATS; i += NT) sm[i] = (i % 97) * 1e-3f;
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
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((probe<NC, KB, TM>), dim3(grid), dim3(NT), 0, 0, W, out, cyc, iters);
    hipDeviceSynchronize();
    long long c[256];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid; ++i) s += c[i];
    const double per = s / grid / iters;
    const double ideal = 2.0 * (NC / 2) * 4 * KB * 32;
    printf("%-22s NC=%2d KB=%2d TM=%d: %8.0f cyc/call  ideal %6.0f  ratio %.2f\n", name, NC, KB, TM, per, ideal, per / ideal);
}

int main() {
    float* W;
    float* out;
    long long* cyc;
    hipMalloc(&W, 4 << 20);
    hipMemset(W, 0, 4 << 20);
    hipMalloc(&out, 256 * NT * 4);
    hipMalloc(&cyc, 256 * 8);
    for (int tm = 0; tm < 3; ++tm) {
        if (tm == 0) { run<18, 6, 0>("QKV", W, out, cyc); run<12, 6, 0>("fc1", W, out, cyc); run<6, 12, 0>("fc2", W, out, cyc); run<6, 18, 0>("C1/C2", W, out, cyc); run<6, 6, 0>("O", W, out, cyc); }
        if (tm == 1) { run<18, 6, 1>("QKV", W, out, cyc); run<12, 6, 1>("fc1", W, out, cyc); run<6, 12, 1>("fc2", W, out, cyc); run<6, 18, 1>("C1/C2", W, out, cyc); run<6, 6, 1>("O", W, out, cyc); }
        if (tm == 2) { run<18, 6, 2>("QKV", W, out, cyc); run<12, 6, 2>("fc1", W, out, cyc); run<6, 12, 2>("fc2", W, out, cyc); run<6, 18, 2>("C1/C2", W, out, cyc); run<6, 6, 2>("O", W, out, cyc); }
    }
    return 0;
}
