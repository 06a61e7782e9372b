// Probe: what a non-MFMA instruction costs when it sits between v_mfma_f32_16x16x4_f32 issues
// (one wave per SIMD, 256 workgroups of 4 waves, one per CU).  Each body is 128 independent
// MFMAs over 8 accumulators plus fillers, written as one inline-asm block so the order is exact.
// Reports cycles per body against the 128 x 32 = 4096-cycle MFMA issue bound.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_filler_probe.hip -o build/mfma_filler_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define MF(i) "v_mfma_f32_16x16x4_f32 %" #i ", %14, %15, %" #i "\n"
#define MF8 MF(0) MF(1) MF(2) MF(3) MF(4) MF(5) MF(6) MF(7)

// filler strings (operands: %8/%9 load destinations, %10/%11 packed pair, %12 scratch VGPR, %13 scratch
// SGPR, %16 rsrc, %17 voff, %18 soff, %19 lds addr, %20 spill-lane VGPR, %21 scratch VGPR)
#define F_NONE ""
#define F_BL "buffer_load_dwordx4 %8, %17, %16, %18 offen\n"
#define F_BLIMM "buffer_load_dwordx4 %8, %17, %16, 0 offen offset:1024\n"
#define F_RDL_BL "v_readlane_b32 %13, %20, 0\ns_nop 4\nbuffer_load_dwordx4 %8, %17, %16, %13 offen\n"
#define F_RDL "v_readlane_b32 %13, %20, 0\n"
#define F_DSR "ds_read_b128 %9, %19\n"
#define F_SALU "s_add_u32 %13, %13, 1\n"
#define F_VADD "v_add_f32 %12, %12, %21\n"
#define F_PKADD "v_pk_add_f32 %10, %10, %11\n"
#define F_NOP4 "s_nop 4\n"
#define F_WAIT "s_waitcnt vmcnt(8)\n"
#define F_ACCRD "v_accvgpr_read_b32 %12, a0\n"

// body: 16 groups of 8 MFMAs; G = filler after every group, M = filler after every MFMA
#define GRP(G) MF8 G
#define BODY_G(G) GRP(G) GRP(G) GRP(G) GRP(G) GRP(G) GRP(G) GRP(G) GRP(G) GRP(G) GRP(G) GRP(G) GRP(G) MF8 MF8 MF8 MF8
#define MFM(i, M) MF(i) M
#define MF8M(M) MFM(0, M) MFM(1, M) MFM(2, M) MFM(3, M) MFM(4, M) MFM(5, M) MFM(6, M) MFM(7, M)
#define BODY_M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8M(M) MF8 MF8 MF8 MF8
#define TAIL "s_waitcnt vmcnt(0) lgkmcnt(0)\ns_nop 15\ns_nop 15\n"

#define KERNEL(NAME, BODY)                                                                                        \
    __global__ void __launch_bounds__(256, 1) NAME(float* buf, long long* cyc, int iters) {                       \
        __shared__ f32x4 lds[256];                                                                                \
        lds[threadIdx.x] = f32x4{1.f, 2.f, 3.f, 4.f};                                                             \
        __syncthreads();                                                                                          \
        f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;                   \
        f32x4 l0, l1;                                                                                             \
        f32x2 l2 = {0.f, 0.f}, l3 = {1.f, 1.f};                                                                   \
        float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f, va = 0.f, vb = 1.f;                        \
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 1 << 20, 0x00020000); \
        const int voff = (threadIdx.x & 63) * 16;                                                                 \
        int soff = 2048;                                                                                          \
        const unsigned ldsa = (unsigned)(size_t)(&lds[threadIdx.x & 63]);                                        \
        const int spill = 4096;                                                                                   \
        int stmp = 0;                                                                                             \
        long long t0 = __builtin_amdgcn_s_memtime();                                                              \
        for (int it = 0; it < iters; ++it) {                                                                      \
            asm volatile(BODY TAIL                                                                                \
                         : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7),       \
                           "=&v"(l0), "=&v"(l1), "+v"(l2), "+v"(l3), "+v"(va), "+s"(stmp)                        \
                         : "v"(a), "v"(b), "s"(rsrc), "v"(voff), "s"(soff), "v"(ldsa), "v"(spill), "v"(vb)       \
                         : "memory");                                                                            \
        }                                                                                                         \
        long long t1 = __builtin_amdgcn_s_memtime();                                                              \
        float s = c0[0] + c1[1] + c2[2] + c3[3] + c4[0] + c5[1] + c6[2] + c7[3] + l2[0] + va + (float)stmp;       \
        buf[(1 << 18) + blockIdx.x * 256 + threadIdx.x] = s;                                                      \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                                          \
    }

KERNEL(k_none, BODY_G(F_NONE))
KERNEL(k_bl_g, BODY_G(F_BL))
KERNEL(k_blimm_g, BODY_G(F_BLIMM))
KERNEL(k_rdlbl_g, BODY_G(F_RDL_BL))
KERNEL(k_rdl_g, BODY_G(F_RDL))
KERNEL(k_nop4_g, BODY_G(F_NOP4))
KERNEL(k_dsr_g, BODY_G(F_DSR))
KERNEL(k_wait_g, BODY_G(F_BL F_WAIT))
KERNEL(k_salu_m, BODY_M(F_SALU))
KERNEL(k_vadd_m, BODY_M(F_VADD))
KERNEL(k_pkadd_m, BODY_M(F_PKADD))
KERNEL(k_vadd2_m, BODY_M(F_VADD F_VADD))
KERNEL(k_accrd_m, BODY_M(F_ACCRD))
KERNEL(k_bl_m, BODY_M(F_BLIMM))
KERNEL(k_dsr_m, BODY_M(F_DSR))

int main() {
    float* d;
    long long* cyc;
    hipMalloc(&d, 4 << 20);
    hipMemset(d, 0, 4 << 20);
    hipMalloc(&cyc, 256 * 8);
    const int iters = 400;
    double base = 0;
    struct K { const char* n; void (*k)(float*, long long*, int); int nf; };
    K ks[] = {{"none", k_none, 0},      {"bl/8", k_bl_g, 12},       {"blimm/8", k_blimm_g, 12}, {"rdl+bl/8", k_rdlbl_g, 12},
              {"rdl/8", k_rdl_g, 12},   {"nop4/8", k_nop4_g, 12},   {"dsr/8", k_dsr_g, 12},     {"bl+wait/8", k_wait_g, 12},
              {"salu/1", k_salu_m, 96}, {"vadd/1", k_vadd_m, 96},   {"pkadd/1", k_pkadd_m, 96}, {"vadd2/1", k_vadd2_m, 96},
              {"accrd/1", k_accrd_m, 96}, {"bl/1", k_bl_m, 96},     {"dsr/1", k_dsr_m, 96}};
    for (auto& k : ks) {
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k.k, dim3(256), dim3(256), 0, 0, d, cyc, iters);
        hipDeviceSynchronize();
        long long c[256];
        hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < 256; ++i) s += c[i];
        const double per = s / 256 / iters;
        if (k.nf == 0) base = per;
        printf("%-10s %8.1f cyc/body (128 MFMA; bound 4096)  fillers %3d  %+7.2f cyc per filler\n", k.n, per, k.nf,
               k.nf ? (per - base) / k.nf : 0.0);
    }
    return 0;
}
