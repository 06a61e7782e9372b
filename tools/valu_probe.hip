// Probe: issue cost (cycles per instruction, one wave per SIMD) of the VALU forms the
// sampler's VALU phases use: v_fmac_f32, v_pk_fma_f32, v_fmac_f32_dpp row_newbcast,
// v_add_f32_dpp quad_perm / row_ror, and ds_read_b128 broadcast reads.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o build/valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int IT = 256;

template <int MODE>
__global__ void __launch_bounds__(256, 1) probe(float* out, long long* cyc) {
    __shared__ f32x4 lds[1024];
    const int t = threadIdx.x;
    for (int i = t; i < 1024; i += 256) lds[i] = f32x4{i * 1e-3f, 1.f, 2.f, 3.f};
    __syncthreads();
    float a[16];
    f32x2 p[16];
    for (int i = 0; i < 16; ++i) {
        a[i] = t * 1e-3f + i;
        p[i] = f32x2{a[i], a[i] + 1.f};
    }
    float x = t * 0.5f, y = t * 0.25f;
    f32x2 x2 = {x, y};
    f32x4 acc4 = {0, 0, 0, 0};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < IT; ++it) {
        if constexpr (MODE == 0) {   // 16 independent v_fmac_f32
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i]) : "v"(x), "v"(y));
        } else if constexpr (MODE == 1) {   // 16 independent v_pk_fma_f32
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(x2), "v"(x2));
        } else if constexpr (MODE == 2) {   // 16 independent v_fmac_f32_dpp row_newbcast
#pragma unroll
            for (int i = 0; i < 16; ++i)
                asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(x), "v"(y));
        } else if constexpr (MODE == 3) {   // 16 independent v_add_f32_dpp quad_perm
#pragma unroll
            for (int i = 0; i < 16; ++i)
                asm volatile("v_add_f32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(x));
        } else if constexpr (MODE == 4) {   // 16 ds_read_b128, 4 distinct addresses per wave (broadcast)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const f32x4 v = lds[((t >> 4) & 3) * 64 + i * 4 + (it & 3)];
                acc4 += v;
            }
        } else if constexpr (MODE == 5) {   // 16 ds_read_b128, 64 distinct consecutive addresses
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const f32x4 v = lds[(t & 63) + (i & 3) * 64 + (it & 3) * 256];
                acc4 += v;
            }
        } else if constexpr (MODE == 6) {   // 16 independent v_mul_f32 + 16 v_pk_mul (mixed)
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p[i]) : "v"(x2));
        } else if constexpr (MODE == 7) {   // v_exp_f32
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = acc4[0] + acc4[1] + acc4[2] + acc4[3];
    for (int i = 0; i < 16; ++i) s += a[i] + p[i][0] + p[i][1];
    out[blockIdx.x * 256 + t] = s;
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
static void run(const char* name, float* out, long long* cyc) {
    hipLaunchKernelGGL((probe<MODE>), dim3(256), dim3(256), 0, 0, out, cyc);
    hipLaunchKernelGGL((probe<MODE>), dim3(256), dim3(256), 0, 0, out, cyc);
    hipDeviceSynchronize();
    long long c[256];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 256; ++i) s += c[i];
    // s_memtime counts at the shader clock / 1 on gfx950 (see phase_trace's implied-clock check)
    printf("%-34s %6.2f memtime-cycles per instruction per wave\n", name, s / 256 / (IT * 16.0));
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&cyc, 256 * 8);
    run<0>("v_fmac_f32", out, cyc);
    run<1>("v_pk_fma_f32", out, cyc);
    run<2>("v_fmac_f32_dpp row_newbcast", out, cyc);
    run<3>("v_add_f32_dpp quad_perm", out, cyc);
    run<4>("ds_read_b128 4 addr (+v_pk_add x2)", out, cyc);
    run<5>("ds_read_b128 64 addr (+v_pk_add x2)", out, cyc);
    run<6>("v_pk_mul_f32", out, cyc);
    run<7>("v_exp_f32", out, cyc);
    return 0;
}
