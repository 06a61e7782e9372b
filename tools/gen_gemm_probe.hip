// Generic-path GEMM probe (tools/gen_gemm_probe.hip): the round-4 LDS-staged dpkg::gemm<BM, VEC> against a
// register-fragment form with no LDS and no barriers (packed weights, each wave an independent
// (16 NI) x (16 NJ) tile, the next 16-k chunk's A/B fragments loaded before the current chunk's MFMAs),
// at the hid-128 generic shapes (M = 17 x 1024 rows).  Prints us per call, TF/s and the largest
// relative difference between the two.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
//        -Iinclude tools/gen_gemm_probe.hip -o build/gen_gemm_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../diffpose-nw_amd/csrc/dpk_kernels.hip"

typedef float f4 __attribute__((ext_vector_type(4)));

// Wp[c][t][lane] (float4 s = 0..3) = W[16c + 4 (lane >> 4) + s][16t + (lane & 15)], zero outside K x N
template <int NI, int NJ, bool VEC>
__global__ void __launch_bounds__(256) gemm_rf(const float* __restrict__ A, int lda, const f4* __restrict__ Wp,
                                               const float* __restrict__ bias, float* C, int ldc, int M, int N, int K,
                                               int mode) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, lk = lane >> 4;
    const int m0 = (blockIdx.x * 4 + wave) * 16 * NI;
    if (m0 >= M) return;
    const int t0 = blockIdx.y * NJ, NT16 = (N + 15) >> 4, KC = (K + 15) >> 4;
    f4 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const float* arow[NI];
    bool aok[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int m = m0 + 16 * i + li;
        aok[i] = m < M;
        arow[i] = A + (size_t)(aok[i] ? m : 0) * lda + 4 * lk;
    }
    bool bok[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bok[j] = t0 + j < NT16;
    const f4* wp = Wp + (size_t)t0 * 64 + lane;
    auto ld = [&](int c, f4 (&ra)[NI], f4 (&rb)[NJ]) {
        const int k = 16 * c + 4 * lk;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (VEC) {
                ra[i] = (aok[i] && k < K) ? *reinterpret_cast<const f4*>(arow[i] + 16 * c) : f4{0.f, 0.f, 0.f, 0.f};
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) ra[i][e] = (aok[i] && k + e < K) ? arow[i][16 * c + e] : 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) rb[j] = bok[j] ? wp[((size_t)c * NT16 + j) * 64] : f4{0.f, 0.f, 0.f, 0.f};
    };
    auto mma = [&](const f4 (&ra)[NI], const f4 (&rb)[NJ]) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(rb[j][s], ra[i][s], acc[i][j], 0, 0, 0);
    };
    f4 a0[NI], b0[NJ], a1[NI], b1[NJ];
    ld(0, a0, b0);
    int c = 0;
    for (; c + 2 <= KC; c += 2) {
        ld(c + 1, a1, b1);
        mma(a0, b0);
        if (c + 2 < KC) ld(c + 2, a0, b0);
        mma(a1, b1);
    }
    if (c < KC) mma(a0, b0);
    // acc[i][j] (operands swapped): lane holds row 16i + li, columns 16j + 4 lk + r
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int m = m0 + 16 * i + li;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int nb = 16 * (t0 + j) + 4 * lk;
            if (nb >= N) continue;
            float* cp = C + (size_t)m * ldc + nb;
            if (VEC && nb + 4 <= N) {
                const f4 bb = *reinterpret_cast<const f4*>(bias + nb);
                f4 v = acc[i][j] + bb;
                if (mode == dpkg::G_RELU) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
                } else if (mode == dpkg::G_RESID) {
                    v = *reinterpret_cast<const f4*>(cp) + v;
                }
                *reinterpret_cast<f4*>(cp) = v;
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (nb + r >= N) continue;
                    const float v = acc[i][j][r] + bias[nb + r];
                    cp[r] = mode == dpkg::G_RELU ? fmaxf(v, 0.f) : mode == dpkg::G_RESID ? cp[r] + v : v;
                }
            }
        }
    }
}


// Buffer-load form: A rows and packed W through buffer resources (per-lane offsets in VGPRs fixed for the
// whole loop, the chunk in soffset, the column tile in the immediate), rows past M and k past K read as 0
// by the hardware range check; no LDS, no barriers, no VALU between the MFMAs but the loop counter.
// Wpad: [KC][NTp][64][4] with NTp = NT16 rounded up to NJ (zero tiles).  K % 4 == 0, lda % 4 == 0.
template <int NI, int NJ, int PD>
__global__ void __launch_bounds__(256) gemm_rb(const float* __restrict__ A, int lda, const float* __restrict__ Wp,
                                               const float* __restrict__ bias, float* C, int ldc, int M, int N, int K,
                                               int mode) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, lk = lane >> 4;
    const int m0 = (blockIdx.x * 4 + wave) * 16 * NI;
    if (m0 >= M) return;
    const int NT16 = (N + 15) >> 4, NTp = (NT16 + NJ - 1) / NJ * NJ, KC = (K + 15) >> 4;
    const int t0 = blockIdx.y * NJ;
    const __amdgpu_buffer_rsrc_t ra_ = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, M * lda * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw_ = __builtin_amdgcn_make_buffer_rsrc((void*)(Wp + (size_t)t0 * 256), (short)0,
                                                                         0x7fffffff, 0x00020000);
    unsigned voa[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int m = m0 + 16 * i + li;
        voa[i] = m < M ? (unsigned)(m * lda + 4 * lk) * 4u : 0x80000000u;
    }
    const unsigned vow = lane * 16u;
    const int kt = K - 4 * lk;      // this lane's k-quad is in range while 16 c < kt
    f4 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    struct Frag { f4 a[NI], b[NJ]; };
    auto ld = [&](int c, Frag& f) {
        const bool kin = 16 * c < kt;
#pragma unroll
        for (int i = 0; i < NI; ++i)
            f.a[i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra_, kin ? voa[i] : 0x80000000u, c * 64, 0));
        const int so = c * NTp * 1024;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            f.b[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rw_, vow + j * 1024, so, 0));
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.b[j][s], f.a[i][s], acc[i][j], 0, 0, 0);
    };
    if constexpr (PD == 1) {
        Frag x0, x1;
        ld(0, x0);
        int c = 0;
        for (; c + 2 <= KC; c += 2) {
            ld(c + 1, x1);
            mma(x0);
            if (c + 2 < KC) ld(c + 2, x0);
            mma(x1);
        }
        if (c < KC) mma(x0);
    } else {
        Frag x0, x1, x2;
        ld(0, x0);
        if (KC > 1) ld(1, x1);
        int c = 0;
        for (; c + 3 <= KC; c += 3) {
            ld(c + 2, x2);
            mma(x0);
            if (c + 3 < KC) ld(c + 3, x0);
            mma(x1);
            if (c + 4 < KC) ld(c + 4, x1);
            mma(x2);
        }
        if (c < KC) mma(x0);
        if (c + 1 < KC) mma(x1);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int m = m0 + 16 * i + li;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int nb = 16 * (t0 + j) + 4 * lk;
            if (nb >= N) continue;
            float* cp = C + (size_t)m * ldc + nb;
            if (nb + 4 <= N) {
                const f4 bb = *reinterpret_cast<const f4*>(bias + nb);
                f4 v = acc[i][j] + bb;
                if (mode == dpkg::G_RELU) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
                } else if (mode == dpkg::G_RESID) {
                    v = *reinterpret_cast<const f4*>(cp) + v;
                }
                *reinterpret_cast<f4*>(cp) = v;
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (nb + r >= N) continue;
                    const float v = acc[i][j][r] + bias[nb + r];
                    cp[r] = mode == dpkg::G_RELU ? fmaxf(v, 0.f) : mode == dpkg::G_RESID ? cp[r] + v : v;
                }
            }
        }
    }
}

// Split-k form: the 4 waves of a workgroup share one (16 NI) x (16 NJ) output tile and take the 16-k chunks
// c = w, w + 4, ... each (buffer loads as gemm_rb, PD chunks in flight), then the four partial tiles meet in
// LDS and every thread finishes one float4 of the tile (bias, activation, residual, one 16-byte store).
template <int NI, int NJ, int PD>
__global__ void __launch_bounds__(256) gemm_sk(const float* __restrict__ A, int lda, const float* __restrict__ Wp,
                                               const float* __restrict__ bias, float* C, int ldc, int M, int N, int K,
                                               int mode) {
    constexpr int TM = 16 * NI, TN = 16 * NJ, LDR = TN + 4;
    __shared__ __attribute__((aligned(16))) float red[4][TM * LDR];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lk = lane >> 4;
    const int m0 = blockIdx.x * TM;
    const int NT16 = (N + 15) >> 4, NTp = (NT16 + NJ - 1) / NJ * NJ, KC = (K + 15) >> 4;
    const int t0 = blockIdx.y * NJ;
    const __amdgpu_buffer_rsrc_t ra_ = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, M * lda * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw_ = __builtin_amdgcn_make_buffer_rsrc((void*)(Wp + (size_t)t0 * 256), (short)0,
                                                                         0x7fffffff, 0x00020000);
    unsigned voa[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int m = m0 + 16 * i + li;
        voa[i] = m < M ? (unsigned)(m * lda + 4 * lk) * 4u : 0x80000000u;
    }
    const unsigned vow = lane * 16u;
    const int kt = K - 4 * lk;
    f4 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    struct Frag { f4 a[NI], b[NJ]; };
    auto ld = [&](int c, Frag& f) {
        const bool kin = 16 * c < kt;
#pragma unroll
        for (int i = 0; i < NI; ++i)
            f.a[i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra_, kin ? voa[i] : 0x80000000u, c * 64, 0));
        const int so = c * NTp * 1024;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            f.b[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rw_, vow + j * 1024, so, 0));
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.b[j][s], f.a[i][s], acc[i][j], 0, 0, 0);
    };
    // this wave's chunks: c = wave + 4 q, q < nq
    const int nq = (KC - wave + 3) >> 2;
    if constexpr (PD == 1) {
        Frag x0, x1;
        if (nq > 0) ld(wave, x0);
        int q = 0;
        for (; q + 2 <= nq; q += 2) {
            ld(wave + 4 * (q + 1), x1);
            mma(x0);
            if (q + 2 < nq) ld(wave + 4 * (q + 2), x0);
            mma(x1);
        }
        if (q < nq) mma(x0);
    } else {
        Frag x0, x1, x2;
        if (nq > 0) ld(wave, x0);
        if (nq > 1) ld(wave + 4, x1);
        int q = 0;
        for (; q + 3 <= nq; q += 3) {
            ld(wave + 4 * (q + 2), x2);
            mma(x0);
            if (q + 3 < nq) ld(wave + 4 * (q + 3), x0);
            mma(x1);
            if (q + 4 < nq) ld(wave + 4 * (q + 4), x1);
            mma(x2);
        }
        if (q < nq) mma(x0);
        if (q + 1 < nq) mma(x1);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            *reinterpret_cast<f4*>(&red[wave][(16 * i + li) * LDR + 16 * j + 4 * lk]) = acc[i][j];
    __syncthreads();
    constexpr int Q = TN / 4;                      // float4s per tile row
#pragma unroll
    for (int e = tid; e < TM * Q; e += 256) {
        const int r = e / Q, cq = e % Q, m = m0 + r, nb = 16 * t0 + 4 * cq;
        if (m >= M || nb >= N) continue;
        f4 v = *reinterpret_cast<const f4*>(&red[0][r * LDR + 4 * cq]);
#pragma unroll
        for (int w = 1; w < 4; ++w) v += *reinterpret_cast<const f4*>(&red[w][r * LDR + 4 * cq]);
        float* cp = C + (size_t)m * ldc + nb;
        if (nb + 4 <= N) {
            v += *reinterpret_cast<const f4*>(bias + nb);
            if (mode == dpkg::G_RELU) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
            } else if (mode == dpkg::G_RESID) {
                v = *reinterpret_cast<const f4*>(cp) + v;
            }
            *reinterpret_cast<f4*>(cp) = v;
        } else {
            for (int q = 0; q < 4 && nb + q < N; ++q) {
                const float u = v[q] + bias[nb + q];
                cp[q] = mode == dpkg::G_RELU ? fmaxf(u, 0.f) : mode == dpkg::G_RESID ? cp[q] + u : u;
            }
        }
    }
}

__global__ void __launch_bounds__(256) empty_k(float* p) {
    if (p && threadIdx.x == 1000) p[0] = 1.f;
}
__global__ void __launch_bounds__(256) copy_k(const f4* __restrict__ a, f4* __restrict__ c, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) c[i] = a[i] + 1.f;
}

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("%s: %s\n", #x, hipGetErrorString(e));                             \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

static std::vector<f4> pack(const std::vector<float>& W, int K, int N) {
    const int KC = (K + 15) / 16, NT16 = (N + 15) / 16;
    std::vector<f4> p((size_t)KC * NT16 * 64);
    for (int c = 0; c < KC; ++c)
        for (int t = 0; t < NT16; ++t)
            for (int l = 0; l < 64; ++l)
                for (int s = 0; s < 4; ++s) {
                    const int k = 16 * c + 4 * (l >> 4) + s, n = 16 * t + (l & 15);
                    p[((size_t)c * NT16 + t) * 64 + l][s] = (k < K && n < N) ? W[(size_t)k * N + n] : 0.f;
                }
    return p;
}

template <class F>
static float timeit(F go, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    go();
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) go();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / reps;
}

static std::vector<f4> pack_pad(const std::vector<float>& W, int K, int N, int NJ) {
    const int KC = (K + 15) / 16, NT16 = (N + 15) / 16, NTp = (NT16 + NJ - 1) / NJ * NJ;
    std::vector<f4> p((size_t)KC * NTp * 64);
    for (int c = 0; c < KC; ++c)
        for (int t = 0; t < NTp; ++t)
            for (int l = 0; l < 64; ++l)
                for (int s = 0; s < 4; ++s) {
                    const int k = 16 * c + 4 * (l >> 4) + s, n = 16 * t + (l & 15);
                    p[((size_t)c * NTp + t) * 64 + l][s] = (k < K && n < N) ? W[(size_t)k * N + n] : 0.f;
                }
    return p;
}

template <int NI, int NJ, int PD>
static float run_rb(const float* A, int K, const std::vector<float>& hW, const float* b, float* C, int M, int N, int reps) {
    auto hp = pack_pad(hW, K, N, NJ);
    float* Wp;
    CK(hipMalloc(&Wp, hp.size() * 16));
    CK(hipMemcpy(Wp, hp.data(), hp.size() * 16, hipMemcpyHostToDevice));
    dim3 grid((M + 64 * NI - 1) / (64 * NI), ((N + 15) / 16 + NJ - 1) / NJ);
    const float us = timeit([&] {
        hipLaunchKernelGGL((gemm_rb<NI, NJ, PD>), grid, dim3(256), 0, 0, A, K, (const float*)Wp, b, C, N, M, N, K,
                           (int)dpkg::G_BIAS);
    }, reps);
    CK(hipFree(Wp));
    return us;
}

template <int NI, int NJ, int PD>
static float run_sk(const float* A, int K, const std::vector<float>& hW, const float* b, float* C, int M, int N, int reps) {
    auto hp = pack_pad(hW, K, N, NJ);
    float* Wp;
    CK(hipMalloc(&Wp, hp.size() * 16));
    CK(hipMemcpy(Wp, hp.data(), hp.size() * 16, hipMemcpyHostToDevice));
    dim3 grid((M + 16 * NI - 1) / (16 * NI), ((N + 15) / 16 + NJ - 1) / NJ);
    const float us = timeit([&] {
        hipLaunchKernelGGL((gemm_sk<NI, NJ, PD>), grid, dim3(256), 0, 0, A, K, (const float*)Wp, b, C, N, M, N, K,
                           (int)dpkg::G_BIAS);
    }, reps);
    CK(hipFree(Wp));
    return us;
}

template <int NI, int NJ>
static float run_rf(const float* A, int K, const f4* Wp, const float* b, float* C, int M, int N, int reps) {
    dim3 grid((M + 64 * NI - 1) / (64 * NI), ((N + 15) / 16 + NJ - 1) / NJ);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((gemm_rf<NI, NJ, true>), grid, dim3(256), 0, 0, A, K, Wp, b, C, N, M, N, K, (int)dpkg::G_BIAS);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((gemm_rf<NI, NJ, true>), grid, dim3(256), 0, 0, A, K, Wp, b, C, N, M, N, K, (int)dpkg::G_BIAS);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / reps;
}

static float run_lds(const float* A, int K, const float* W, const float* b, float* C, int M, int N, int reps) {
    dim3 grid((M + 31) / 32, (N + 63) / 64);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto go = [&] {
        hipLaunchKernelGGL((dpkg::gemm<32, true>), grid, dim3(256), 0, 0, A, K, W, b, C, N, M, N, K, (int)dpkg::G_BIAS,
                           (const float*)nullptr, 0, 17);
    };
    go();
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) go();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
    const int M = 17 * 1024 * (argc > 1 ? atoi(argv[1]) : 1), reps = 50;
    {
        float *a, *c;
        const size_t n = (size_t)M * 128 / 4;
        CK(hipMalloc(&a, n * 16));
        CK(hipMalloc(&c, n * 16));
        CK(hipMemset(a, 0, n * 16));
        for (int g : {1, 256, 1088, 4352})
            printf("empty kernel, %5d workgroups: %7.2f us\n", g,
                   timeit([&] { hipLaunchKernelGGL(empty_k, dim3(g), dim3(256), 0, 0, nullptr); }, reps));
        for (int g : {1024, 2048, 4096, 8192}) {
            const float us = timeit([&] { hipLaunchKernelGGL(copy_k, dim3(g), dim3(256), 0, 0, (const f4*)a, (f4*)c, n); }, reps);
            printf("copy M x 128 fp32 (%.1f MB read + write), %5d workgroups: %7.2f us = %.2f TB/s\n", n * 16e-6, g, us,
                   2.0 * n * 16 / (us * 1e-6) * 1e-12);
        }
        CK(hipFree(a));
        CK(hipFree(c));
    }
    const int shapes[][2] = {{128, 384}, {128, 128}, {128, 256}, {256, 128}, {384, 128}, {96, 288}, {288, 96}};
    for (auto& sh : shapes) {
        const int K = sh[0], N = sh[1];
        std::vector<float> hA((size_t)M * K), hW((size_t)K * N), hb(N);
        srand(K * 1000 + N);
        for (auto& v : hA) v = (rand() % 2001 - 1000) * 1e-3f;
        for (auto& v : hW) v = (rand() % 2001 - 1000) * 1e-4f;
        for (auto& v : hb) v = (rand() % 2001 - 1000) * 1e-3f;
        auto hp = pack(hW, K, N);
        float *A, *W, *b, *C0, *C1;
        f4* Wp;
        CK(hipMalloc(&A, hA.size() * 4));
        CK(hipMalloc(&W, hW.size() * 4));
        CK(hipMalloc(&b, hb.size() * 4));
        CK(hipMalloc(&Wp, hp.size() * 16));
        CK(hipMalloc(&C0, (size_t)M * N * 4));
        CK(hipMalloc(&C1, (size_t)M * N * 4));
        CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(b, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(Wp, hp.data(), hp.size() * 16, hipMemcpyHostToDevice));
        const double gf = 2.0 * M * K * N * 1e-9;
        float t = run_lds(A, K, W, b, C0, M, N, reps);
        printf("K %3d N %3d  lds<32>     %7.2f us  %6.1f TF\n", K, N, t, gf / (t * 1e-6) * 1e-3);
        std::vector<float> r0((size_t)M * N), r1((size_t)M * N);
        CK(hipMemcpy(r0.data(), C0, r0.size() * 4, hipMemcpyDeviceToHost));
        auto report = [&](const char* name, float us) {
            CK(hipMemcpy(r1.data(), C1, r1.size() * 4, hipMemcpyDeviceToHost));
            double md = 0;
            for (size_t i = 0; i < r0.size(); ++i) md = fmax(md, fabs(r0[i] - r1[i]) / (1.0 + fabs(r0[i])));
            printf("K %3d N %3d  %-10s  %7.2f us  %6.1f TF  maxrel %.2e\n", K, N, name, us, gf / (us * 1e-6) * 1e-3, md);
        };
        report("rb<1,4,2>", run_rb<1, 4, 2>(A, K, hW, b, C1, M, N, reps));
        report("sk<1,2,1>", run_sk<1, 2, 1>(A, K, hW, b, C1, M, N, reps));
        report("sk<1,4,1>", run_sk<1, 4, 1>(A, K, hW, b, C1, M, N, reps));
        report("sk<2,2,1>", run_sk<2, 2, 1>(A, K, hW, b, C1, M, N, reps));
        report("sk<2,4,1>", run_sk<2, 4, 1>(A, K, hW, b, C1, M, N, reps));
        report("sk<1,4,2>", run_sk<1, 4, 2>(A, K, hW, b, C1, M, N, reps));
        report("sk<2,4,2>", run_sk<2, 4, 2>(A, K, hW, b, C1, M, N, reps));
        report("sk<4,4,1>", run_sk<4, 4, 1>(A, K, hW, b, C1, M, N, reps));
        report("sk<2,8,1>", run_sk<2, 8, 1>(A, K, hW, b, C1, M, N, reps));
        CK(hipFree(A));
        CK(hipFree(W));
        CK(hipFree(b));
        CK(hipFree(Wp));
        CK(hipFree(C0));
        CK(hipFree(C1));
    }
    return 0;
}
