#include <hip/hip_runtime.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
// 1: 16x16x4 f32 -> builtin permlane32 swap
__global__ void k1(float* o, const float* in) {
    int l = threadIdx.x;
    f32x4 c = {0,0,0,0};
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(in[l], in[l+64], c, 0, 0, 0);
    auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, c[0]), __builtin_bit_cast(unsigned, c[1]), false, false);
    o[l] = __builtin_bit_cast(float, r[0]) - 2.0f * __builtin_bit_cast(float, r[1]);
}
// 2: 4x4x4_16b bf16 -> builtin swap
__global__ void k2(float* o, const bf16x4* in) {
    int l = threadIdx.x;
    f32x4 c = {0,0,0,0};
    c = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(__builtin_bit_cast(s16x4, in[l]), __builtin_bit_cast(s16x4, in[l+64]), c, 0, 0, 0);
    auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, c[0]), __builtin_bit_cast(unsigned, c[1]), false, false);
    o[l] = __builtin_bit_cast(float, r[0]) - 2.0f * __builtin_bit_cast(float, r[1]);
}
// 3: 16x16x32 bf16 -> builtin swap
__global__ void k3(float* o, const bf16x8* in) {
    int l = threadIdx.x;
    f32x4 c = {0,0,0,0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(in[l], in[l+64], c, 0, 0, 0);
    auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, c[0]), __builtin_bit_cast(unsigned, c[1]), false, false);
    o[l] = __builtin_bit_cast(float, r[0]) - 2.0f * __builtin_bit_cast(float, r[1]);
}
// 4: 4x4x1 f32 -> v_add
__global__ void k4(float* o, const float* in) {
    int l = threadIdx.x;
    f32x4 c = {0,0,0,0};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(in[l], in[l+64], c, 0, 0, 0);
    o[l] = c[0] + c[1];
}
// 5: 4x4x1 f32 -> swap
__global__ void k5(float* o, const float* in) {
    int l = threadIdx.x;
    f32x4 c = {0,0,0,0};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(in[l], in[l+64], c, 0, 0, 0);
    auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, c[0]), __builtin_bit_cast(unsigned, c[1]), false, false);
    o[l] = __builtin_bit_cast(float, r[0]) - 2.0f * __builtin_bit_cast(float, r[1]);
}
// 6: 16x16x4 f32 -> v_add
__global__ void k6(float* o, const float* in) {
    int l = threadIdx.x;
    f32x4 c = {0,0,0,0};
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(in[l], in[l+64], c, 0, 0, 0);
    o[l] = c[0] + c[1];
}
// 7: 16x16x32 f16 -> v_add
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__global__ void k7(float* o, const f16x8* in) {
    int l = threadIdx.x;
    f32x4 c = {0,0,0,0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(in[l], in[l+64], c, 0, 0, 0);
    o[l] = c[0] + c[1];
}
// 8: 16x16x16 bf16 -> v_add
__global__ void k8(float* o, const bf16x4* in) {
    int l = threadIdx.x;
    f32x4 c = {0,0,0,0};
    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, in[l]), __builtin_bit_cast(s16x4, in[l+64]), c, 0, 0, 0);
    o[l] = c[0] + c[1];
}
