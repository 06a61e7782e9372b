// dpk_kernels.hip — MI355X (gfx950, CDNA4) DDIM sampler for DiffPose's GCNdiff denoiser.
//
// One persistent kernel runs the whole K-step reverse-diffusion loop of the reference
// (common/utils_diff.py:46-68) for a tile of P=4 poses per workgroup: every step's
// GCNdiff forward (models/gcndiff.py:101-113) and the DDIM update happen in LDS, so the
// only HBM traffic is the (N,17,5) input, the output and the weights (L2/MALL-resident).
//
// Tile geometry: 4 poses = 68 rows of 96 features; Linear/ChebConv
// GEMMs run on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32 fma chains) over 5 row
// tiles of 16; waves 0-2 own column thirds of row tiles 0-3, wave 3 owns row tile 4
// (rows 64-67 valid).  LayerNorm, 17-joint attention and the 17x17 graph products are
// VALU work between workgroup barriers.  Weights are repacked at load time into MFMA
// B-fragment order: one 1 KiB coalesced float4-per-lane load per (16 cols x 16 k) block.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "diffpose_kernels.h"

namespace dpk {

// ---------------------------------------------------------------------------------------
// compile-time model shape (configs/human36m_diffpose_uvxyz_cpn.yml:9-16)
constexpr int J = 17;        // joints (n_pts)
constexpr int D = 96;        // hid_dim
constexpr int D2 = 192;      // GraphNet hidden (2*hid)
constexpr int D3 = 288;      // QKV / Chebyshev-stacked width
constexpr int E = 384;       // emd_dim = 4*hid
constexpr int NL = 5;        // num_layer
constexpr int NH = 4;        // n_head
constexpr int DK = 24;       // d_k
constexpr int CIN = 5;       // coords_dim[0]
constexpr int COUT = 5;      // coords_dim[1]
constexpr int PE = J * CIN;  // floats per pose (85)

// workgroup tile
constexpr int P = 4;         // poses per workgroup
constexpr int R = P * J;     // 68 rows
constexpr int RT = 5;        // 16-row MFMA tiles covering R (80 rows, 64..67 valid in the last)
constexpr int NT = 256;      // threads (4 waves, one per SIMD)
constexpr int LDX = 104;     // LDS row stride, 96-wide buffers  (≡40 mod 64: conflict-free b128 A reads)
constexpr int LD2 = 296;     // LDS row stride, 288-wide buffer  (≡40 mod 64)

// LDS carve (floats)
constexpr int SM_XS = 0;                    // residual stream   [R][LDX]
constexpr int SM_B1 = SM_XS + R * LDX;      // 96-wide scratch   [R][LDX]
constexpr int SM_B2 = SM_B1 + R * LDX;      // 288-wide scratch  [R][LD2]
constexpr int SM_XST = SM_B2 + R * LD2;     // pose state x_t    [R][5]
constexpr int SM_T1 = SM_XST + ((R * CIN + 3) / 4) * 4;
constexpr int SM_T2 = SM_T1 + 292;
constexpr int SM_LG = SM_T2 + 292;          // 5 GraphNet Laplacians [NL][17][17]
constexpr int SM_FLOATS = SM_LG + ((NL * J * J + 3) / 4) * 4;
static_assert(SM_FLOATS * 4 <= 160 * 1024, "LDS budget");

// packed-weight blocks: one block = 16 cols x 16 k = 64 lanes x float4
constexpr int BLK = 256;
constexpr int KB_D = D / 16, KB_D2 = D2 / 16, KB_D3 = D3 / 16;   // 6, 12, 18
// per-layer offsets (floats) in the weight arena
constexpr int OFF_QKV = 0;                                  // [18 ct][6 kb]
constexpr int OFF_O = OFF_QKV + 18 * KB_D * BLK;            // [6][6]
constexpr int OFF_FC1 = OFF_O + 6 * KB_D * BLK;             // [12][6]
constexpr int OFF_FC2 = OFF_FC1 + 12 * KB_D * BLK;          // [6][12]
constexpr int OFF_C1 = OFF_FC2 + 6 * KB_D2 * BLK;           // [6][18]
constexpr int OFF_C2 = OFF_C1 + 6 * KB_D3 * BLK;            // [6][18]
constexpr int OFF_BQKV = OFF_C2 + 6 * KB_D3 * BLK;
constexpr int OFF_BO = OFF_BQKV + D3;
constexpr int OFF_BFC1 = OFF_BO + D;
constexpr int OFF_BFC2 = OFF_BFC1 + D2;
constexpr int OFF_BC1 = OFF_BFC2 + D;
constexpr int OFF_BC2 = OFF_BC1 + D;
constexpr int OFF_LN0A = OFF_BC2 + D;
constexpr int OFF_LN0B = OFF_LN0A + D;
constexpr int OFF_LN1A = OFF_LN0B + D;
constexpr int OFF_LN1B = OFF_LN1A + D;
constexpr int OFF_LG = OFF_LN1B + D;                        // 17x17
constexpr int LAYER_FLOATS = ((OFF_LG + J * J + 63) / 64) * 64;
constexpr int OFF_WIN = NL * LAYER_FLOATS;                  // [6 ct][1 kb]  (K=15 padded to 16)
constexpr int OFF_WOUT = OFF_WIN + 6 * 1 * BLK;             // [1 ct][18 kb] (N=5 padded to 16)
constexpr int OFF_BIN = OFF_WOUT + 1 * KB_D3 * BLK;
constexpr int OFF_BOUT = OFF_BIN + D;                       // 16 (5 used)
constexpr int OFF_T1 = OFF_BOUT + 16;                       // 17x17 dense Chebyshev T1
constexpr int OFF_T2 = OFF_T1 + 292;
constexpr int ARENA_FLOATS = ((OFF_T2 + 292 + 63) / 64) * 64;

// timestep-MLP arena (transposed nn.Linear weights: [in][out])
constexpr int TOFF_W0 = 0;                    // [96][384]
constexpr int TOFF_B0 = TOFF_W0 + D * E;
constexpr int TOFF_W1 = TOFF_B0 + E;          // [384][384]
constexpr int TOFF_B1 = TOFF_W1 + E * E;
constexpr int TOFF_WP = TOFF_B1 + E;          // [5][384][96]
constexpr int TOFF_BP = TOFF_WP + NL * E * D; // [5][96]
constexpr int TEMB_FLOATS = TOFF_BP + NL * D;

constexpr float SQRT_DK = 4.898979485566356f;   // float(math.sqrt(24)), divisor
constexpr float LN_EPS = 1e-6f;                         // LayerNorm eps (GraFormer.py:60)

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct SampleArgs {
    const float* arena;   // packed weights
    const float* coef;    // [K][6] = sqrt(1-at), sqrt(at), sqrt(an), c1, c2, t
    const float* tproj;   // [slots][NL][D] temb_proj(swish(temb)) per step (sample) or per pose (eps)
    const float* x_in;    // [N][17][5]
    float* x_out;         // [N][17][5]  final x (sample) or eps (eps mode)
    float* xs;            // [K+1][N][17][5] or null
    float* x0s;           // [K][N][17][5]   or null
    int N;
    int K;
    unsigned mask;        // 17-bit key mask
    float eta;
    unsigned long long seed;
};

// ---------------------------------------------------------------------------------------
// counter-based normal noise for eta > 0 (Philox4x32-10 + Box-Muller)
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

__device__ __forceinline__ float normal_noise(unsigned long long seed, int step, long long idx) {
    uint32_t c[4] = {(uint32_t)idx, (uint32_t)((unsigned long long)idx >> 32), (uint32_t)step, 0x5EEDu};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = ((float)(c[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
    const float u2 = (float)(c[1] >> 8) * (1.0f / 16777216.0f);            // [0, 1)
    return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// DDIM update for one element (common/utils_diff.py:59-65), fp32, no contraction:
// x0 = (xt - et*sqrt(1-at)) / sqrt(at);  x' = sqrt(an)*x0 + c1*z + c2*et
__device__ __forceinline__ void ddim_elem(const float* cf, float xt, float et, float z, float& x0, float& xn) {
    x0 = (xt - et * cf[0]) / cf[1];
    xn = (cf[2] * x0 + cf[3] * z) + cf[4] * et;
}

// Launder a value through an empty asm so LLVM cannot hoist per-thread address math out
// of the K-step / layer loops of the persistent kernel (hoisted, it stays live across
// every phase and spills).
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// ---------------------------------------------------------------------------------------
// MFMA GEMM over one wave's units: row tiles [rt0, rt0+NR) x col tiles [ct0, ct0+NCW).
// A: LDS rows (k in [0,16*KB0) from A0, [16*KB0, 16*(KB0+KB1)) from A1); B: packed blocks.
// Lane l holds A[row rt*16+(l&15)][k = kb*16 + 4*(l>>4) + j] for MFMA sub-step j, and the
// packed B block holds W[k = same][n = ct*16 + (l&15)]: a consistent permutation of k.
template <int NR, int NCW, int KB0, int KB1, class Epi>
__device__ __forceinline__ void gemm_wave(const float* A0, int lda0, const float* A1, int lda1,
                                          const f32x4* __restrict__ Bp, int rt0, int ct0, int lane, Epi epi) {
    constexpr int KB = KB0 + KB1;
    lane = opaque(lane);
    f32x4 acc[NR][NCW];
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int c = 0; c < NCW; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int rl = lane & 15, kq = (lane >> 4) * 4;
    int row[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const int r = (rt0 + i) * 16 + rl;
        row[i] = r < R ? r : R - 1;     // clamp padding rows (outputs discarded)
    }
    f32x4 bcur[NCW];
#pragma unroll
    for (int c = 0; c < NCW; ++c) bcur[c] = Bp[((ct0 + c) * KB + 0) * 64 + lane];

#pragma unroll 1
    for (int kb = 0; kb < KB; ++kb) {
        f32x4 bnext[NCW];
        if (kb + 1 < KB) {
#pragma unroll
            for (int c = 0; c < NCW; ++c) bnext[c] = Bp[((ct0 + c) * KB + kb + 1) * 64 + lane];
        }
        f32x4 a[NR];
        if (kb < KB0) {
#pragma unroll
            for (int i = 0; i < NR; ++i) a[i] = *reinterpret_cast<const f32x4*>(A0 + row[i] * lda0 + kb * 16 + kq);
        } else {
#pragma unroll
            for (int i = 0; i < NR; ++i)
                a[i] = *reinterpret_cast<const f32x4*>(A1 + row[i] * lda1 + (kb - KB0) * 16 + kq);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < NR; ++i)
#pragma unroll
                for (int c = 0; c < NCW; ++c)
                    acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][j], bcur[c][j], acc[i][c], 0, 0, 0);
        if (kb + 1 < KB) {
#pragma unroll
            for (int c = 0; c < NCW; ++c) bcur[c] = bnext[c];
        }
    }
    // C/D map of 16x16 MFMA: col = lane&15, row = 4*(lane>>4) + r
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int c = 0; c < NCW; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int orow = (rt0 + i) * 16 + kq + r;
                if (orow < R) epi(orow, (ct0 + c) * 16 + rl, acc[i][c][r]);
            }
}

// Whole-workgroup GEMM with NC (multiple of 3) output col tiles.
template <int NC, int KB0, int KB1, class Epi>
__device__ __forceinline__ void gemm_wg(const float* A0, int lda0, const float* A1, int lda1, const float* Bp,
                                        int wave, int lane, Epi epi) {
    static_assert(NC % 3 == 0, "column tiles split in thirds");
    const f32x4* B = reinterpret_cast<const f32x4*>(Bp);
    if (wave < 3) {
        gemm_wave<4, NC / 3, KB0, KB1>(A0, lda0, A1, lda1, B, 0, wave * (NC / 3), lane, epi);
    } else {
        // wave 3: the partial row tile across all columns, in passes of <= 6 column tiles
        constexpr int CH = NC < 6 ? NC : 6;
        static_assert(NC % CH == 0, "column chunking");
#pragma unroll 1
        for (int c0 = 0; c0 < NC; c0 += CH) gemm_wave<1, CH, KB0, KB1>(A0, lda0, A1, lda1, B, 4, c0, lane, epi);
    }
}

// ---------------------------------------------------------------------------------------
// LayerNorm of GraFormer (GraFormer.py:58-70): a*(x-mean)/(std_unbiased + eps) + b.
// 16 lanes per row, 6 features per lane; mean/var accumulated in double.
__device__ __forceinline__ void layer_norm(const float* src, float* dst, const float* __restrict__ gain,
                                           const float* __restrict__ shift, int tid) {
    tid = opaque(tid);
    const int w = tid >> 6, lane = tid & 63, sub = lane >> 4, q = lane & 15;
    float g[6], b[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
        g[e] = gain[6 * q + e];
        b[e] = shift[6 * q + e];
    }
#pragma unroll 1
    for (int it = 0; it < 5; ++it) {
        const int row = it * 16 + w * 4 + sub;
        const int rr = row < R ? row : R - 1;
        const float* s = src + rr * LDX + 6 * q;
        float v[6];
#pragma unroll
        for (int e = 0; e < 6; e += 2) {
            const float2 t = *reinterpret_cast<const float2*>(s + e);
            v[e] = t.x;
            v[e + 1] = t.y;
        }
        double sum = 0.0;
#pragma unroll
        for (int e = 0; e < 6; ++e) sum += (double)v[e];
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 16);
        const double mean_d = sum / (double)D;
        double ss = 0.0;
#pragma unroll
        for (int e = 0; e < 6; ++e) {
            const double dv = (double)v[e] - mean_d;
            ss += dv * dv;
        }
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 16);
        const float mean = (float)mean_d;
        const float den = (float)sqrt(ss / (double)(D - 1)) + LN_EPS;
        if (row < R) {
            float* d = dst + row * LDX + 6 * q;
#pragma unroll
            for (int e = 0; e < 6; e += 2) {
                float2 t;
                t.x = (g[e] * (v[e] - mean)) / den + b[e];
                t.y = (g[e + 1] * (v[e + 1] - mean)) / den + b[e + 1];
                *reinterpret_cast<float2*>(d + e) = t;
            }
        }
    }
}

// 4-head attention over the 17 joints of each pose (GraFormer.py:99-140, without the
// projections).  One thread per (pose, head, query); scores/softmax/PV in registers.
__device__ __forceinline__ void attention(const float* qkv, float* out, unsigned mask, int tid) {
    tid = opaque(tid);
#pragma unroll 1
    for (int item = tid; item < P * NH * J; item += NT) {
        const int p = item / (NH * J);
        const int rem = item - p * (NH * J);
        const int h = rem / J;
        const int i = rem - h * J;
        const float* qr = qkv + (p * J + i) * LD2 + h * DK;
        float q[DK];
#pragma unroll
        for (int d = 0; d < DK; d += 4) {
            const f32x4 t = *reinterpret_cast<const f32x4*>(qr + d);
            q[d] = t[0]; q[d + 1] = t[1]; q[d + 2] = t[2]; q[d + 3] = t[3];
        }
        float s[J];
        float m = -INFINITY;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const float* kr = qkv + (p * J + j) * LD2 + D + h * DK;
            float dot = 0.f;
#pragma unroll
            for (int d = 0; d < DK; d += 4) {
                const f32x4 t = *reinterpret_cast<const f32x4*>(kr + d);
                dot = fmaf(q[d], t[0], dot);
                dot = fmaf(q[d + 1], t[1], dot);
                dot = fmaf(q[d + 2], t[2], dot);
                dot = fmaf(q[d + 3], t[3], dot);
            }
            s[j] = ((mask >> j) & 1u) ? dot / SQRT_DK : -1e9f;
            m = fmaxf(m, s[j]);
        }
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            s[j] = expf(s[j] - m);
            sum += s[j];
        }
        const float inv = 1.0f / sum;
        float o[DK];
#pragma unroll
        for (int d = 0; d < DK; ++d) o[d] = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const float pj = s[j] * inv;
            const float* vr = qkv + (p * J + j) * LD2 + 2 * D + h * DK;
#pragma unroll
            for (int d = 0; d < DK; d += 4) {
                const f32x4 t = *reinterpret_cast<const f32x4*>(vr + d);
                o[d] = fmaf(pj, t[0], o[d]);
                o[d + 1] = fmaf(pj, t[1], o[d + 1]);
                o[d + 2] = fmaf(pj, t[2], o[d + 2]);
                o[d + 3] = fmaf(pj, t[3], o[d + 3]);
            }
        }
        float* orow = out + (p * J + i) * LDX + h * DK;
#pragma unroll
        for (int d = 0; d < DK; d += 4) *reinterpret_cast<f32x4*>(orow + d) = f32x4{o[d], o[d + 1], o[d + 2], o[d + 3]};
    }
}

// dst[:, c] = M @ src[:, c] per pose (17x17 M in LDS), G columns per thread; in-place safe.
template <int G>
__device__ __forceinline__ void graph_apply(const float* M, const float* src, int lds, float* dst, int ldd,
                                            int ncols, int tid) {
    tid = opaque(tid);
    const int ng = ncols / G;      // P*ng <= NT: one item per thread, no loop (keeps M out of registers)
    {
        const int item = tid;
        if (item >= P * ng) return;
        const int p = item / ng;
        const int c = (item - p * ng) * G;
        float v[J][G];
#pragma unroll
        for (int i = 0; i < J; ++i)
#pragma unroll
            for (int g = 0; g < G; ++g) v[i][g] = src[(p * J + i) * lds + c + g];
        float o[J][G];
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float a = 0.f;
#pragma unroll
                for (int i = 0; i < J; ++i) a = fmaf(M[j * J + i], v[i][g], a);
                o[j][g] = a;
            }
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int g = 0; g < G; ++g) dst[(p * J + j) * ldd + c + g] = o[j][g];
    }
}

// Chebyshev prologue: B2[:, 0:96] = T1 src, B2[:, 96:192] = T2 src (ChebConv.py:83).
__device__ __forceinline__ void cheb_prep(const float* T1, const float* T2, const float* src, float* b2, int tid) {
    tid = opaque(tid);
    constexpr int G = 2, ng = D / G;
    static_assert(P * ng <= NT, "one item per thread");
    {
        const int item = tid;
        if (item >= P * ng) return;
        const int p = item / ng;
        const int c = (item - p * ng) * G;
        float v[J][G];
#pragma unroll
        for (int i = 0; i < J; ++i) {
            const float2 t = *reinterpret_cast<const float2*>(src + (p * J + i) * LDX + c);
            v[i][0] = t.x;
            v[i][1] = t.y;
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            float a0 = 0.f, a1 = 0.f, c0 = 0.f, c1 = 0.f;
#pragma unroll
            for (int i = 0; i < J; ++i) {
                const float t1 = T1[j * J + i], t2 = T2[j * J + i];
                a0 = fmaf(t1, v[i][0], a0);
                a1 = fmaf(t1, v[i][1], a1);
                c0 = fmaf(t2, v[i][0], c0);
                c1 = fmaf(t2, v[i][1], c1);
            }
            *reinterpret_cast<float2*>(b2 + (p * J + j) * LD2 + c) = make_float2(a0, a1);
            *reinterpret_cast<float2*>(b2 + (p * J + j) * LD2 + D + c) = make_float2(c0, c1);
        }
    }
}

// ---------------------------------------------------------------------------------------
// The sampler: K DDIM steps (or one eps evaluation) for P poses per workgroup.
template <bool EPS_MODE>
__global__ void __launch_bounds__(NT, 1) sample_kernel(SampleArgs a) {
    __shared__ __attribute__((aligned(16))) float sm[SM_FLOATS];
    float* XS = sm + SM_XS;
    float* B1 = sm + SM_B1;
    float* B2 = sm + SM_B2;
    float* XST = sm + SM_XST;
    float* T1 = sm + SM_T1;
    float* T2 = sm + SM_T2;
    float* LG = sm + SM_LG;

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int pose0 = blockIdx.x * P;
    const int npose = min(P, a.N - pose0);
    const int nvalid = npose * PE;
    const float* W = a.arena;

    for (int i = tid; i < J * J; i += NT) {
        T1[i] = W[OFF_T1 + i];
        T2[i] = W[OFF_T2 + i];
    }
    for (int i = tid; i < NL * J * J; i += NT) LG[i] = W[(i / (J * J)) * LAYER_FLOATS + OFF_LG + (i % (J * J))];
    for (int i = tid; i < R * CIN; i += NT) XST[i] = i < nvalid ? a.x_in[(size_t)pose0 * PE + i] : 0.f;
    __syncthreads();

    const int K = EPS_MODE ? 1 : a.K;
#pragma unroll 1
    for (int s = 0; s < K; ++s) {
        // ---- gconv_input: ChebConv 5->96 (gcndiff.py:108): A = [x | T1 x | T2 x | 0]
        if (tid < P * CIN) {
            const int p = tid / CIN, c = tid - p * CIN;
            float v[J];
#pragma unroll
            for (int i = 0; i < J; ++i) v[i] = XST[(p * J + i) * CIN + c];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                float a1 = 0.f, a2 = 0.f;
#pragma unroll
                for (int i = 0; i < J; ++i) {
                    a1 = fmaf(T1[j * J + i], v[i], a1);
                    a2 = fmaf(T2[j * J + i], v[i], a2);
                }
                float* rowp = B1 + (p * J + j) * LDX;
                rowp[c] = v[j];
                rowp[CIN + c] = a1;
                rowp[2 * CIN + c] = a2;
                if (c == 0) rowp[3 * CIN] = 0.f;
            }
        }
        __syncthreads();
        {
            const float* bias = W + OFF_BIN;
            gemm_wg<6, 1, 0>(B1, LDX, nullptr, 0, W + OFF_WIN, wave, lane,
                             [&](int r, int c, float v) { XS[r * LDX + c] = v + bias[c]; });
        }
        __syncthreads();

#pragma unroll 1
        for (int l = 0; l < NL; ++l) {
            const float* LW = W + l * LAYER_FLOATS;
            const float* lg = LG + l * J * J;
            // ---- x = x + MHA(LN0(x))   (GraAttenLayer, GraFormer.py:94-95)
            layer_norm(XS, B1, LW + OFF_LN0A, LW + OFF_LN0B, tid);
            __syncthreads();
            {
                const float* bias = LW + OFF_BQKV;
                gemm_wg<18, 6, 0>(B1, LDX, nullptr, 0, LW + OFF_QKV, wave, lane,
                                  [&](int r, int c, float v) { B2[r * LD2 + c] = v + bias[c]; });
            }
            __syncthreads();
            attention(B2, B1, a.mask, tid);
            __syncthreads();
            {
                const float* bias = LW + OFF_BO;
                gemm_wg<6, 6, 0>(B1, LDX, nullptr, 0, LW + OFF_O, wave, lane,
                                 [&](int r, int c, float v) { XS[r * LDX + c] = XS[r * LDX + c] + (v + bias[c]); });
            }
            __syncthreads();
            // ---- x = x + GraphNet(LN1(x))   (GraFormer.py:189-201)
            layer_norm(XS, B1, LW + OFF_LN1A, LW + OFF_LN1B, tid);
            __syncthreads();
            graph_apply<2>(lg, B1, LDX, B1, LDX, D, tid);
            __syncthreads();
            {
                const float* bias = LW + OFF_BFC1;
                gemm_wg<12, 6, 0>(B1, LDX, nullptr, 0, LW + OFF_FC1, wave, lane,
                                  [&](int r, int c, float v) { B2[r * LD2 + c] = fmaxf(v + bias[c], 0.f); });
            }
            __syncthreads();
            graph_apply<4>(lg, B2, LD2, B2, LD2, D2, tid);
            __syncthreads();
            {
                const float* bias = LW + OFF_BFC2;
                gemm_wg<6, 12, 0>(B2, LD2, nullptr, 0, LW + OFF_FC2, wave, lane,
                                  [&](int r, int c, float v) { XS[r * LDX + c] = XS[r * LDX + c] + (v + bias[c]); });
            }
            __syncthreads();
            // ---- _ResChebGC_diff (gcndiff.py:47-53): x + relu(Cheb2(relu(Cheb1(x)) + temb_proj))
            cheb_prep(T1, T2, XS, B2, tid);
            __syncthreads();
            {
                const float* bias = LW + OFF_BC1;
                const float* tp = a.tproj + (EPS_MODE ? 0 : (size_t)s * NL * D) + l * D;
                const int pstride = EPS_MODE ? NL * D : 0;
                gemm_wg<6, 6, 12>(XS, LDX, B2, LD2, LW + OFF_C1, wave, lane, [&](int r, int c, float v) {
                    const float* tpp = tp + (size_t)(EPS_MODE ? min(pose0 + r / J, a.N - 1) : 0) * pstride;
                    B1[r * LDX + c] = fmaxf(v + bias[c], 0.f) + tpp[c];
                });
            }
            __syncthreads();
            cheb_prep(T1, T2, B1, B2, tid);
            __syncthreads();
            {
                const float* bias = LW + OFF_BC2;
                gemm_wg<6, 6, 12>(B1, LDX, B2, LD2, LW + OFF_C2, wave, lane, [&](int r, int c, float v) {
                    XS[r * LDX + c] = XS[r * LDX + c] + fmaxf(v + bias[c], 0.f);
                });
            }
            __syncthreads();
        }
        // ---- gconv_output: ChebConv 96->5 (gcndiff.py:112), then the DDIM update
        cheb_prep(T1, T2, XS, B2, tid);
        __syncthreads();
        {
            const float* bias = W + OFF_BOUT;
            const f32x4* Bo = reinterpret_cast<const f32x4*>(W + OFF_WOUT);
            const float* cf = a.coef + (EPS_MODE ? 0 : s * 6);
            auto epi = [&](int r, int c, float v) {
                if (c >= COUT) return;
                const float et = v + bias[c];
                const int idx = r * CIN + c;           // same as r*COUT+c (coords 5 -> 5)
                const bool valid = idx < nvalid;
                const size_t gidx = (size_t)pose0 * PE + idx;
                if (EPS_MODE) {
                    if (valid) a.x_out[gidx] = et;
                } else {
                    const float z = a.eta != 0.f ? normal_noise(a.seed, s, (long long)gidx) : 0.f;
                    float x0, xn;
                    ddim_elem(cf, XST[idx], et, z, x0, xn);
                    XST[idx] = xn;
                    if (valid) {
                        if (a.x0s) a.x0s[(size_t)s * a.N * PE + gidx] = x0;
                        if (a.xs) a.xs[(size_t)(s + 1) * a.N * PE + gidx] = xn;
                    }
                }
            };
            gemm_wave<1, 1, 6, 12>(XS, LDX, B2, LD2, Bo, wave, 0, lane, epi);
            if (wave == 3) gemm_wave<1, 1, 6, 12>(XS, LDX, B2, LD2, Bo, 4, 0, lane, epi);
        }
        __syncthreads();
    }
    if (!EPS_MODE)
        for (int i = tid; i < nvalid; i += NT) a.x_out[(size_t)pose0 * PE + i] = XST[i];
}

// ---------------------------------------------------------------------------------------
// Timestep MLP (gcndiff.py:15-33, :103-106) and per-layer temb_proj(swish(.)) (:46, :51):
// tproj[slot][l][:] for slot t-values (one per DDIM step, or one per pose in eps mode).
// Batch-invariant in the sampler: all rows of a step share t, so it is computed once per step.
__device__ __forceinline__ float swishf(float x) { return x * (1.0f / (1.0f + expf(-x))); }

__global__ void __launch_bounds__(256) temb_kernel(const float* __restrict__ tw, const float* __restrict__ tvals,
                                                   int tstride, float* __restrict__ tproj) {
    __shared__ float emb[D];
    __shared__ float h0[E];
    __shared__ float h1[E];
    const int tid = threadIdx.x;
    const float t = tvals[(size_t)blockIdx.x * tstride];
    const float neg_scale = -(float)(9.210340371976184 / 47.0);   // -(log(10000)/(half-1)), fp32 scalar
    if (tid < D) {
        const int k = tid < D / 2 ? tid : tid - D / 2;
        const float f = expf((float)k * neg_scale);
        const float arg = t * f;
        emb[tid] = tid < D / 2 ? sinf(arg) : cosf(arg);
    }
    __syncthreads();
    for (int o = tid; o < E; o += 256) {
        float acc = 0.f;
        for (int k = 0; k < D; ++k) acc = fmaf(emb[k], tw[TOFF_W0 + k * E + o], acc);
        h0[o] = swishf(acc + tw[TOFF_B0 + o]);
    }
    __syncthreads();
    for (int o = tid; o < E; o += 256) {
        float acc = 0.f;
        for (int k = 0; k < E; ++k) acc = fmaf(h0[k], tw[TOFF_W1 + k * E + o], acc);
        h1[o] = swishf(acc + tw[TOFF_B1 + o]);     // swish(temb) as consumed by every temb_proj
    }
    __syncthreads();
    for (int o = tid; o < NL * D; o += 256) {
        const int l = o / D, c = o - l * D;
        const float* wp = tw + TOFF_WP + (size_t)l * E * D;
        float acc = 0.f;
        for (int k = 0; k < E; ++k) acc = fmaf(h1[k], wp[k * D + c], acc);
        tproj[(size_t)blockIdx.x * NL * D + o] = acc + tw[TOFF_BP + o];
    }
}

// Elementwise DDIM update for externally computed eps.
__global__ void __launch_bounds__(256) ddim_kernel(const float* __restrict__ xt, const float* __restrict__ et,
                                                   float* __restrict__ xn, float* __restrict__ x0o, long long n,
                                                   const float* __restrict__ cf, int step, float eta,
                                                   unsigned long long seed) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float z = eta != 0.f ? normal_noise(seed, step, i) : 0.f;
    float x0, x1;
    ddim_elem(cf, xt[i], et[i], z, x0, x1);
    xn[i] = x1;
    if (x0o) x0o[i] = x0;
}

}  // namespace dpk

// =======================================================================================
// Host side: handle, weight repacking, schedule, launches (the C ABI of diffpose_kernels.h)
// =======================================================================================
using namespace dpk;

struct dpk_handle {
    int device = 0;
    std::string err;
    float* arena = nullptr;        // device: packed weights + graph constants
    float* temb = nullptr;         // device: timestep-MLP weights
    float* coef = nullptr;         // device: [K][6]
    float* tproj = nullptr;        // device: [cap][NL][D]
    int tproj_cap = 0;
    std::vector<float> h_arena;    // host staging of the arena
    std::vector<float> h_temb;
    bool have_graph = false, have_weights = false, have_sched = false;
    std::vector<float> h_coef;
    int K = 0;
    float eta = 0.f;
    unsigned mask = (1u << J) - 1u;
    std::vector<float> h_adj;
    bool profiling = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used, ev_free;
};

// event pair around a sampler-kernel launch (dpk_profile)
static int prof_begin(dpk_handle* h, hipStream_t st, std::pair<hipEvent_t, hipEvent_t>& ev) {
    if (h->ev_free.empty()) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return DPK_E_HIP;
        h->ev_free.push_back({a, b});
    }
    ev = h->ev_free.back();
    h->ev_free.pop_back();
    return hipEventRecord(ev.first, st) == hipSuccess ? DPK_OK : DPK_E_HIP;
}
static int prof_end(dpk_handle* h, hipStream_t st, std::pair<hipEvent_t, hipEvent_t>& ev) {
    if (hipEventRecord(ev.second, st) != hipSuccess) return DPK_E_HIP;
    h->ev_used.push_back(ev);
    return DPK_OK;
}

static int fail(dpk_handle* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}

#define HIPCHK(h, expr)                                                                        \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail((h), DPK_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));    \
    } while (0)

// Pack W_eff (K x N, W_eff(k, n)) into MFMA B-fragment blocks [NC][KB][64][4].
template <class F>
static void pack_blocks(float* dst, int Kreal, int Nreal, int KB, int NC, F w) {
    for (int ct = 0; ct < NC; ++ct)
        for (int kb = 0; kb < KB; ++kb)
            for (int lane = 0; lane < 64; ++lane)
                for (int j = 0; j < 4; ++j) {
                    const int k = kb * 16 + 4 * (lane >> 4) + j;
                    const int n = ct * 16 + (lane & 15);
                    dst[((size_t)(ct * KB + kb) * 64 + lane) * 4 + j] = (k < Kreal && n < Nreal) ? w(k, n) : 0.f;
                }
}

// Chebyshev terms of the normalised Laplacian, fp32 in the reference's operation order
// (ChebConv.py:114-130, :90-112): d = rowsum^-1/2; L = I - (d_i g_ij) d_j; T2 = 2 L@L - I.
static void cheb_terms(const float* g, float* T1, float* T2) {
    float d[J];
    for (int i = 0; i < J; ++i) {
        float s = 0.f;
        for (int j = 0; j < J; ++j) s += g[i * J + j];
        d[i] = 1.0f / sqrtf(s);
    }
    float L[J * J];
    for (int i = 0; i < J; ++i)
        for (int j = 0; j < J; ++j) L[i * J + j] = (i == j ? 1.f : 0.f) - (d[i] * g[i * J + j]) * d[j];
    for (int i = 0; i < J; ++i)
        for (int j = 0; j < J; ++j) {
            float acc = 0.f;
            for (int k = 0; k < J; ++k) acc += L[i * J + k] * L[k * J + j];
            T1[i * J + j] = L[i * J + j];
            T2[i * J + j] = 2.f * acc - (i == j ? 1.f : 0.f);
        }
}

// GraphNet Laplacian (GraFormer.py:174-178): c_k = colsum_k + 1e-5; L = c_i^-1/2 A_ij c_j^-1/2.
static void graph_lap(const float* A, float* Lg) {
    float dh[J];
    for (int k = 0; k < J; ++k) {
        float s = 0.f;
        for (int i = 0; i < J; ++i) s += A[i * J + k];
        dh[k] = 1.0f / sqrtf(s + 1e-5f);
    }
    for (int i = 0; i < J; ++i)
        for (int j = 0; j < J; ++j) Lg[i * J + j] = (dh[i] * A[i * J + j]) * dh[j];
}

static int upload(dpk_handle* h) {
    HIPCHK(h, hipSetDevice(h->device));
    if (!h->arena) HIPCHK(h, hipMalloc(&h->arena, (size_t)ARENA_FLOATS * 4));
    if (!h->temb) HIPCHK(h, hipMalloc(&h->temb, (size_t)TEMB_FLOATS * 4));
    HIPCHK(h, hipMemcpy(h->arena, h->h_arena.data(), (size_t)ARENA_FLOATS * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->temb, h->h_temb.data(), (size_t)TEMB_FLOATS * 4, hipMemcpyHostToDevice));
    return DPK_OK;
}

extern "C" {

int dpk_version(void) { return 100; }

int dpk_kernel_geometry(int* ppw, int* tpw, int* lds) {
    if (ppw) *ppw = P;
    if (tpw) *tpw = NT;
    if (lds) *lds = SM_FLOATS * 4;
    return DPK_OK;
}

int dpk_create(const dpk_config* cfg, dpk_handle** out) {
    if (!cfg || !out) return DPK_E_INVALID;
    *out = nullptr;
    if (cfg->hid_dim != D || cfg->num_layers != NL || cfg->n_head != NH || cfg->n_pts != J ||
        cfg->coords_in != CIN || cfg->coords_out != COUT)
        return DPK_E_UNSUPPORTED;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || cfg->device < 0 || cfg->device >= ndev) return DPK_E_HIP;
    dpk_handle* h = new dpk_handle();
    h->device = cfg->device;
    h->h_arena.assign(ARENA_FLOATS, 0.f);
    h->h_temb.assign(TEMB_FLOATS, 0.f);
    *out = h;
    return DPK_OK;
}

void dpk_destroy(dpk_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->arena) (void)hipFree(h->arena);
    if (h->temb) (void)hipFree(h->temb);
    if (h->coef) (void)hipFree(h->coef);
    if (h->tproj) (void)hipFree(h->tproj);
    for (auto* v : {&h->ev_used, &h->ev_free})
        for (auto& e : *v) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
    delete h;
}

const char* dpk_last_error(const dpk_handle* h) { return h ? h->err.c_str() : "null handle"; }

int dpk_set_graph(dpk_handle* h, const float* adj) {
    if (!h || !adj) return fail(h, DPK_E_INVALID, "dpk_set_graph: null argument");
    float T1[J * J], T2[J * J];
    cheb_terms(adj, T1, T2);
    for (int i = 0; i < J * J; ++i) {
        h->h_arena[OFF_T1 + i] = T1[i];
        h->h_arena[OFF_T2 + i] = T2[i];
    }
    h->h_adj.assign(adj, adj + J * J);
    h->have_graph = true;
    if (h->have_weights) return upload(h);
    return DPK_OK;
}

int dpk_set_mask(dpk_handle* h, const uint8_t* m) {
    if (!h || !m) return fail(h, DPK_E_INVALID, "dpk_set_mask: null argument");
    unsigned bits = 0;
    for (int j = 0; j < J; ++j)
        if (m[j]) bits |= 1u << j;
    h->mask = bits;
    return DPK_OK;
}

int dpk_load_weights(dpk_handle* h, const char* const* names, const float* const* ptrs, const int64_t* numels,
                     int n) {
    if (!h || !names || !ptrs || !numels || n <= 0) return fail(h, DPK_E_INVALID, "dpk_load_weights: bad args");
    std::unordered_map<std::string, std::pair<const float*, int64_t>> sd;
    for (int i = 0; i < n; ++i) {
        if (!names[i] || !ptrs[i]) return fail(h, DPK_E_INVALID, "dpk_load_weights: null entry");
        std::string k = names[i];
        if (k.rfind("module.", 0) == 0) k = k.substr(7);
        sd[k] = {ptrs[i], numels[i]};
    }
    std::string missing;
    auto get = [&](const std::string& k, int64_t numel) -> const float* {
        auto it = sd.find(k);
        if (it == sd.end()) {
            missing = "missing key " + k;
            return nullptr;
        }
        if (it->second.second != numel) {
            missing = "size mismatch for " + k;
            return nullptr;
        }
        return it->second.first;
    };
#define GET(var, key, numel)                                             \
    const float* var = get(key, numel);                                  \
    if (!var) return fail(h, DPK_E_WEIGHTS, "dpk_load_weights: " + missing);

    float* A = h->h_arena.data();
    for (int l = 0; l < NL; ++l) {
        float* Lw = A + (size_t)l * LAYER_FLOATS;
        const std::string at = "atten_layers." + std::to_string(l) + ".";
        const std::string gc = "gconv_layers." + std::to_string(l) + ".";
        GET(wq, at + "self_attn.linears.0.weight", D * D);
        GET(wk, at + "self_attn.linears.1.weight", D * D);
        GET(wv, at + "self_attn.linears.2.weight", D * D);
        GET(wo, at + "self_attn.linears.3.weight", D * D);
        GET(bq, at + "self_attn.linears.0.bias", D);
        GET(bk, at + "self_attn.linears.1.bias", D);
        GET(bv, at + "self_attn.linears.2.bias", D);
        GET(bo, at + "self_attn.linears.3.bias", D);
        GET(ahat, at + "feed_forward.A_hat", J * J);
        GET(f1w, at + "feed_forward.gconv1.fc.weight", D2 * D);
        GET(f1b, at + "feed_forward.gconv1.fc.bias", D2);
        GET(f2w, at + "feed_forward.gconv2.fc.weight", D * D2);
        GET(f2b, at + "feed_forward.gconv2.fc.bias", D);
        GET(n0a, at + "sublayer.0.norm.a_2", D);
        GET(n0b, at + "sublayer.0.norm.b_2", D);
        GET(n1a, at + "sublayer.1.norm.a_2", D);
        GET(n1b, at + "sublayer.1.norm.b_2", D);
        GET(c1w, gc + "gconv1.gconv.weight", 3 * D * D);
        GET(c1b, gc + "gconv1.gconv.bias", D);
        GET(c2w, gc + "gconv2.gconv.weight", 3 * D * D);
        GET(c2b, gc + "gconv2.gconv.bias", D);
        GET(tpw, gc + "temb_proj.weight", D * E);
        GET(tpb, gc + "temb_proj.bias", D);
        // nn.Linear weight is (out, in): W_eff[k][n] = weight[n][k]
        pack_blocks(Lw + OFF_QKV, D, D3, KB_D, 18, [&](int k, int n) {
            const float* w = n < D ? wq : (n < 2 * D ? wk : wv);
            return w[(n % D) * D + k];
        });
        pack_blocks(Lw + OFF_O, D, D, KB_D, 6, [&](int k, int n) { return wo[n * D + k]; });
        pack_blocks(Lw + OFF_FC1, D, D2, KB_D, 12, [&](int k, int n) { return f1w[n * D + k]; });
        pack_blocks(Lw + OFF_FC2, D2, D, KB_D2, 6, [&](int k, int n) { return f2w[n * D2 + k]; });
        // ChebConv weight (3,1,in,out): row k = order*in + c of the stacked [X|T1X|T2X]
        pack_blocks(Lw + OFF_C1, D3, D, KB_D3, 6, [&](int k, int n) { return c1w[(k / D) * D * D + (k % D) * D + n]; });
        pack_blocks(Lw + OFF_C2, D3, D, KB_D3, 6, [&](int k, int n) { return c2w[(k / D) * D * D + (k % D) * D + n]; });
        for (int c = 0; c < D; ++c) {
            Lw[OFF_BQKV + c] = bq[c];
            Lw[OFF_BQKV + D + c] = bk[c];
            Lw[OFF_BQKV + 2 * D + c] = bv[c];
            Lw[OFF_BO + c] = bo[c];
            Lw[OFF_BFC2 + c] = f2b[c];
            Lw[OFF_BC1 + c] = c1b[c];
            Lw[OFF_BC2 + c] = c2b[c];
            Lw[OFF_LN0A + c] = n0a[c];
            Lw[OFF_LN0B + c] = n0b[c];
            Lw[OFF_LN1A + c] = n1a[c];
            Lw[OFF_LN1B + c] = n1b[c];
        }
        for (int c = 0; c < D2; ++c) Lw[OFF_BFC1 + c] = f1b[c];
        graph_lap(ahat, Lw + OFF_LG);
        // temb_proj: transposed [in=384][out=96]
        float* T = h->h_temb.data();
        for (int o = 0; o < D; ++o) {
            for (int k = 0; k < E; ++k) T[TOFF_WP + (size_t)l * E * D + k * D + o] = tpw[o * E + k];
            T[TOFF_BP + l * D + o] = tpb[o];
        }
    }
    GET(wi, "gconv_input.weight", 3 * CIN * D);
    GET(bi, "gconv_input.bias", D);
    GET(wout, "gconv_output.weight", 3 * D * COUT);
    GET(bout, "gconv_output.bias", COUT);
    GET(d0w, "temb.dense.0.weight", E * D);
    GET(d0b, "temb.dense.0.bias", E);
    GET(d1w, "temb.dense.1.weight", E * E);
    GET(d1b, "temb.dense.1.bias", E);
#undef GET
    pack_blocks(A + OFF_WIN, 3 * CIN, D, 1, 6, [&](int k, int n) { return wi[(k / CIN) * CIN * D + (k % CIN) * D + n]; });
    pack_blocks(A + OFF_WOUT, D3, COUT, KB_D3, 1,
                [&](int k, int n) { return wout[(k / D) * D * COUT + (k % D) * COUT + n]; });
    for (int c = 0; c < D; ++c) A[OFF_BIN + c] = bi[c];
    for (int c = 0; c < 16; ++c) A[OFF_BOUT + c] = c < COUT ? bout[c] : 0.f;
    float* T = h->h_temb.data();
    for (int o = 0; o < E; ++o) {
        for (int k = 0; k < D; ++k) T[TOFF_W0 + k * E + o] = d0w[o * D + k];
        for (int k = 0; k < E; ++k) T[TOFF_W1 + k * E + o] = d1w[o * E + k];
        T[TOFF_B0 + o] = d0b[o];
        T[TOFF_B1 + o] = d1b[o];
    }
    h->have_weights = true;
    return upload(h);
}

int dpk_set_schedule(dpk_handle* h, const float* abar, int n_alpha, const int* seq, int K, float eta) {
    if (!h || !abar || !seq || K <= 0 || n_alpha < 2) return fail(h, DPK_E_INVALID, "dpk_set_schedule: bad args");
    std::vector<float> c((size_t)K * 6);
    // execution order: i over reversed(seq), j over reversed([-1] + seq[:-1]) (utils_diff.py:49-52)
    for (int s = 0; s < K; ++s) {
        const int t = seq[K - 1 - s];
        const int tn = (K - 2 - s) >= 0 ? seq[K - 2 - s] : -1;
        if (t + 1 < 0 || t + 1 >= n_alpha || tn + 1 < 0 || tn + 1 >= n_alpha)
            return fail(h, DPK_E_INVALID, "dpk_set_schedule: timestep outside alpha table (index t+1)");
        const float at = abar[t + 1], an = abar[tn + 1];
        const float one = 1.0f;
        volatile float s1a = sqrtf(one - at);
        volatile float sa = sqrtf(at);
        volatile float san = sqrtf(an);
        volatile float r = at / an;
        volatile float u = one - r;
        volatile float v = one - an;
        volatile float w = u * v;
        volatile float inner = w / (one - at);
        volatile float c1 = eta * sqrtf(inner);
        volatile float c1sq = c1 * c1;
        volatile float c2 = sqrtf((one - an) - c1sq);
        c[s * 6 + 0] = s1a;
        c[s * 6 + 1] = sa;
        c[s * 6 + 2] = san;
        c[s * 6 + 3] = c1;
        c[s * 6 + 4] = c2;
        c[s * 6 + 5] = (float)t;
    }
    HIPCHK(h, hipSetDevice(h->device));
    if (h->coef && h->K < K) {
        HIPCHK(h, hipFree(h->coef));
        h->coef = nullptr;
    }
    if (!h->coef) HIPCHK(h, hipMalloc(&h->coef, (size_t)std::max(K, 1) * 6 * 4));
    HIPCHK(h, hipMemcpy(h->coef, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    h->h_coef = c;
    h->K = K;
    h->eta = eta;
    h->have_sched = true;
    return DPK_OK;
}

static int ensure_tproj(dpk_handle* h, int slots) {
    if (h->tproj_cap >= slots) return DPK_OK;
    if (h->tproj) HIPCHK(h, hipFree(h->tproj));
    h->tproj = nullptr;
    HIPCHK(h, hipMalloc(&h->tproj, (size_t)slots * NL * D * 4));
    h->tproj_cap = slots;
    return DPK_OK;
}

static int check_ready(dpk_handle* h) {
    if (!h->have_graph) return fail(h, DPK_E_STATE, "graph (adjacency) not set");
    if (!h->have_weights) return fail(h, DPK_E_STATE, "weights not loaded");
    return DPK_OK;
}

int dpk_eps(dpk_handle* h, const float* x, const float* t, float* eps, int N, void* stream) {
    if (!h) return DPK_E_INVALID;
    if (N < 0 || (N > 0 && (!x || !t || !eps))) return fail(h, DPK_E_INVALID, "dpk_eps: bad args");
    int rc = check_ready(h);
    if (rc) return rc;
    if (N == 0) return DPK_OK;
    HIPCHK(h, hipSetDevice(h->device));
    rc = ensure_tproj(h, N);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(temb_kernel, dim3(N), dim3(256), 0, st, h->temb, t, 1, h->tproj);
    HIPCHK(h, hipGetLastError());
    SampleArgs a{};
    a.arena = h->arena;
    a.coef = h->coef;     // unused in eps mode
    a.tproj = h->tproj;
    a.x_in = x;
    a.x_out = eps;
    a.N = N;
    a.K = 1;
    a.mask = h->mask;
    std::pair<hipEvent_t, hipEvent_t> ev;
    if (h->profiling && prof_begin(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_eps: event record");
    hipLaunchKernelGGL(sample_kernel<true>, dim3((N + P - 1) / P), dim3(NT), 0, st, a);
    HIPCHK(h, hipGetLastError());
    if (h->profiling && prof_end(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_eps: event record");
    return DPK_OK;
}

int dpk_sample(dpk_handle* h, const float* x, float* out, float* xs, float* x0s, int N, uint64_t seed,
               void* stream) {
    if (!h) return DPK_E_INVALID;
    if (N < 0 || (N > 0 && (!x || !out))) return fail(h, DPK_E_INVALID, "dpk_sample: bad args");
    int rc = check_ready(h);
    if (rc) return rc;
    if (!h->have_sched) return fail(h, DPK_E_STATE, "schedule not set");
    if (N == 0) return DPK_OK;
    HIPCHK(h, hipSetDevice(h->device));
    rc = ensure_tproj(h, h->K);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (xs) HIPCHK(h, hipMemcpyAsync(xs, x, (size_t)N * PE * 4, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(temb_kernel, dim3(h->K), dim3(256), 0, st, h->temb, h->coef + 5, 6, h->tproj);
    HIPCHK(h, hipGetLastError());
    SampleArgs a{};
    a.arena = h->arena;
    a.coef = h->coef;
    a.tproj = h->tproj;
    a.x_in = x;
    a.x_out = out;
    a.xs = xs;
    a.x0s = x0s;
    a.N = N;
    a.K = h->K;
    a.mask = h->mask;
    a.eta = h->eta;
    a.seed = seed;
    std::pair<hipEvent_t, hipEvent_t> ev;
    if (h->profiling && prof_begin(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_sample: event record");
    hipLaunchKernelGGL(sample_kernel<false>, dim3((N + P - 1) / P), dim3(NT), 0, st, a);
    HIPCHK(h, hipGetLastError());
    if (h->profiling && prof_end(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_sample: event record");
    return DPK_OK;
}

int dpk_profile(dpk_handle* h, int enable) {
    if (!h) return DPK_E_INVALID;
    h->profiling = enable != 0;
    return DPK_OK;
}

int dpk_profile_read(dpk_handle* h, float* ms, int cap, int* count) {
    if (!h || (cap > 0 && !ms)) return fail(h, DPK_E_INVALID, "dpk_profile_read: bad args");
    HIPCHK(h, hipSetDevice(h->device));
    int n = 0;
    for (auto& e : h->ev_used) {
        HIPCHK(h, hipEventSynchronize(e.second));
        float t = 0.f;
        HIPCHK(h, hipEventElapsedTime(&t, e.first, e.second));
        if (n < cap) ms[n] = t;
        ++n;
        h->ev_free.push_back(e);
    }
    h->ev_used.clear();
    if (count) *count = n;
    return DPK_OK;
}

int dpk_ddim_update(dpk_handle* h, const float* xt, const float* et, float* xn, float* x0, int64_t n, int step,
                    uint64_t seed, void* stream) {
    if (!h) return DPK_E_INVALID;
    if (n < 0 || (n > 0 && (!xt || !et || !xn))) return fail(h, DPK_E_INVALID, "dpk_ddim_update: bad args");
    if (!h->have_sched) return fail(h, DPK_E_STATE, "schedule not set");
    if (step < 0 || step >= h->K) return fail(h, DPK_E_INVALID, "dpk_ddim_update: step out of range");
    if (n == 0) return DPK_OK;
    HIPCHK(h, hipSetDevice(h->device));
    const long long nb = (n + 255) / 256;
    hipLaunchKernelGGL(ddim_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, xt, et, xn, x0, (long long)n,
                       h->coef + step * 6, step, h->eta, (unsigned long long)seed);
    HIPCHK(h, hipGetLastError());
    return DPK_OK;
}

}  // extern "C"
