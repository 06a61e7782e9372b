// Probe: the sampler's GEMM phase with 8 waves per workgroup (two per SIMD) against the shipped
// 4-wave mapping, same tile work per SIMD (tools/w8_probe.hip).
//
// 4 waves (shipped): wave w = row tiles 2(w>>1), +1 x column half w&1 (NC/2 tiles), tails split
// between the two waves of a half.  8 waves: wave w = row pair pr = w>>2 x column group cg of NC/4
// tiles (sizes ceil/floor alternate: 18 -> 5,4,5,4; 6 -> 2,1,2,1; 12 -> 3,3,3,3); the waves sharing
// a SIMD (w, w+4) take complementary groups (cg = (w&3) ^ pr), so every SIMD has exactly the MFMA
// work of the 4-wave mapping, each B fragment still feeds two row tiles, and the second wave on the
// SIMD can issue while the first waits on L2 / LDS / the barrier.  One workgroup per CU, every CU busy,
// ITER back-to-back calls separated by a barrier, each with its B prefetch issued before the barrier.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize
//        -mllvm -amdgpu-mfma-vgpr-form -Iinclude tools/w8_probe.hip -o build/w8_probe
#include <hip/hip_runtime.h>
#include "../diffpose-nw_amd/csrc/dpk_kernels.hip"

using namespace dpk;

// prefetch of the first two k-blocks of NCG tiles from global tile ct0, rotated by rot
template <int NCG, int NC, int KB>
__device__ __forceinline__ BPre<NCG> pre_tiles(const float* W, int ct0, int rot, int lane) {
    const BSrc s = bsrc<NC, KB>(W, ct0, lane);
    int soff[NCG];
    tile_offsets<NCG, KB>(soff, s, rot);
    BPre<NCG> p;
#pragma unroll
    for (int c = 0; c < NCG; ++c) {
        p.b0[c] = bload(s, soff[c], 0);
        p.b1[c] = bload(s, soff[c], 1);
    }
    return p;
}

// PROBE_MODE bit 1: no barriers; bit 2: no B prefetch (the ring's first blocks are zeros)
#ifndef PROBE_MODE
#define PROBE_MODE 0
#endif
template <int NCG, int NC, int KB>
__device__ __forceinline__ void w8_gemm(const float* A, const float* W, const EpiArgs& e, int pr, int ct0, int lane) {
    const int rot = pr ? (NCG + 1) / 2 : 0;
    BPre<NCG> pre;
    if constexpr (PROBE_MODE & 2) {
        for (int c = 0; c < NCG; ++c) pre.b0[c] = pre.b1[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
        pre = pre_tiles<NCG, NC, KB>(W, ct0, rot, lane);
    }
    if constexpr (!(PROBE_MODE & 1)) __syncthreads();
    gemm_wave<2, NCG, TM_MFMA4, 0, NC, KB, E_STORE>(A, LD2, W, 2 * pr, ct0, rot, 64, (NCG & 1) && pr, lane, e, pre);
}

template <int NC, int KB, int NW8>
__global__ void __launch_bounds__(64 * NW8, 1) probe(const float* W, float* out, long long* cyc, int iters) {
    __shared__ __attribute__((aligned(16))) float sm[SM_FLOATS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < SM_FLOATS; i += 64 * NW8) sm[i] = ((i % 97) - 48) * 1e-2f;
    __syncthreads();
    const float* A = sm + SM_B2;
    const EpiArgs e{sm + SM_XS, LDX, W + NC * KB * 256, nullptr, 0, 0, 0};
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        if constexpr (NW8 == 4) {
            constexpr int NCW = NC / 2;
            const int half = wave >> 1, ch = wave & 1;
            w8_gemm<NCW, NC, KB>(A, W, e, half, ch * NCW, lane);
        } else {
            constexpr int NA = (NC + 3) / 4, NB = NC / 4;      // tiles of even / odd column groups
            const int pr = wave >> 2, cg = (wave & 3) ^ pr;
            const int ct0 = (cg >> 1) * (NA + NB) + (cg & 1) * NA;
            if ((cg & 1) == 0) w8_gemm<NA, NC, KB>(A, W, e, pr, ct0, lane);
            else w8_gemm<NB, NC, KB>(A, W, e, pr, ct0, lane);
        }
        if constexpr (!(PROBE_MODE & 1)) __syncthreads();
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 64 * NW8 + tid] = sm[(tid * 7) % SM_FLOATS];
}

template <int NC, int KB, int NW8>
static double run(const float* W, float* out, long long* cyc) {
    const int iters = 200, grid = 256;
    hipLaunchKernelGGL((probe<NC, KB, NW8>), dim3(grid), dim3(64 * NW8), 0, 0, W, out, cyc, iters);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL((probe<NC, KB, NW8>), dim3(grid), dim3(64 * NW8), 0, 0, W, out, cyc, iters);
    (void)hipDeviceSynchronize();
    long long c[256];
    (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid; ++i) s += c[i];
    return s / grid / iters;
}

template <int NC, int KB>
static void both(const char* name, const float* W, float* out, long long* cyc) {
    const double a = run<NC, KB, 4>(W, out, cyc), b = run<NC, KB, 8>(W, out, cyc);
    const double ideal = (2.0 * NC / 2 * 4 * 32 + ((NC / 2 + 1) / 2) * 4 * 8.8) * KB;   // per SIMD, tails incl.
    printf("%-8s NC=%2d KB=%2d: 4 waves %7.0f  8 waves %7.0f cyc/call (ratio %.3f)  MFMA bound %6.0f\n", name, NC, KB, a, b,
           b / a, ideal);
}

int main() {
    float* W;
    float* out;
    long long* cyc;
    (void)hipMalloc(&W, 4 << 20);
    {
        static float hw[1 << 20];
        for (int i = 0; i < (1 << 20); ++i) hw[i] = ((i * 2654435761u) >> 8 & 0xffff) * (1.0f / 65536.0f) - 0.5f;
        (void)hipMemcpy(W, hw, 4 << 20, hipMemcpyHostToDevice);
    }
    (void)hipMalloc(&out, 256 * 512 * 4);
    (void)hipMalloc(&cyc, 256 * 8);
    both<18, 6>("QKV", W, out, cyc);
    both<12, 6>("fc1", W, out, cyc);
    both<6, 6>("O", W, out, cyc);
    both<6, 12>("fc2", W, out, cyc);
    both<6, 18>("C1/C2", W, out, cyc);
    return 0;
}
