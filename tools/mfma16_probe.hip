// Probe: operand layouts of v_mfma_f32_16x16x32_f16 and v_mfma_f32_4x4x4_16b_f16 as the
// split-fp16 GEMM path assumes them, checked against a CPU product.
//   16x16x32: lane l holds A[row l&15][k 8*(l>>4)+i] and B[k 8*(l>>4)+i][col l&15], i=0..7;
//             D reg r of lane l = C[row 4*(l>>4)+r][col l&15].
//   4x4x4_16b: block b = l>>2; lane l holds A_b[row l&3][k 0..3] and B_b[k 0..3][col l&3];
//             D reg r of lane l = C_b[row r][col l&3].
// Also checks the 3-term split product hi*hi + hi*lo + lo*hi against fp64.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k16(const float* A, const float* B, float* C, float* C3) {   // A 16x32, B 32x16 row-major
    const int l = threadIdx.x;
    f16x8 a, b, ah, al, bh, bl;
    for (int i = 0; i < 8; ++i) {
        const int k = 8 * (l >> 4) + i;
        const float av = A[(l & 15) * 32 + k], bv = B[k * 16 + (l & 15)];
        a[i] = (_Float16)av;
        b[i] = (_Float16)bv;
        ah[i] = (_Float16)av;
        al[i] = (_Float16)(av - (float)ah[i]);
        bh[i] = (_Float16)bv;
        bl[i] = (_Float16)(bv - (float)bh[i]);
    }
    f32x4 c = {0, 0, 0, 0}, c3 = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c3, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c3, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c3, 0, 0, 0);
    for (int r = 0; r < 4; ++r) {
        C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
        C3[(4 * (l >> 4) + r) * 16 + (l & 15)] = c3[r];
    }
}

__global__ void k4(const float* A, const float* B, float* C) {   // 16 blocks: A_b 4x4, B_b 4x4
    const int l = threadIdx.x, b = l >> 2;
    f16x4 a, bb;
    for (int kk = 0; kk < 4; ++kk) {
        a[kk] = (_Float16)A[b * 16 + (l & 3) * 4 + kk];    // A_b[row l&3][k]
        bb[kk] = (_Float16)B[b * 16 + kk * 4 + (l & 3)];   // B_b[k][col l&3]
    }
    f32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_4x4x4f16(a, bb, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[b * 16 + r * 4 + (l & 3)] = c[r];
}

int main() {
    float hA[512], hB[512], hC[256], hC3[256];
    srand(1);
    for (int i = 0; i < 512; ++i) {
        hA[i] = (float)((rand() % 2001) - 1000) / 997.0f;
        hB[i] = (float)((rand() % 2001) - 1000) / 991.0f;
    }
    float *dA, *dB, *dC, *dC3;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dC, 1024); hipMalloc(&dC3, 1024);
    hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC, dC3);
    hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    hipMemcpy(hC3, dC3, 1024, hipMemcpyDeviceToHost);
    double e1 = 0, e3 = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s16 = 0, s = 0;
            for (int k = 0; k < 32; ++k) {
                s16 += (double)(float)(_Float16)hA[i * 32 + k] * (double)(float)(_Float16)hB[k * 16 + j];
                s += (double)hA[i * 32 + k] * hB[k * 16 + j];
            }
            e1 = fmax(e1, fabs(s16 - hC[i * 16 + j]));
            e3 = fmax(e3, fabs(s - hC3[i * 16 + j]) / (fabs(s) + 1e-3));
        }
    printf("16x16x32 f16 layout: max |err| vs fp16-rounded product %.3g (expect ~1e-6)\n", e1);
    printf("16x16x32 3-term split: max rel err vs fp64 %.3g (expect <~1e-6)\n", e3);
    hipLaunchKernelGGL(k4, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    double e4 = 0;
    for (int b = 0; b < 16; ++b)
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double s = 0;
                for (int k = 0; k < 4; ++k)
                    s += (double)(float)(_Float16)hA[b * 16 + i * 4 + k] * (double)(float)(_Float16)hB[b * 16 + k * 4 + j];
                e4 = fmax(e4, fabs(s - hC[b * 16 + i * 4 + j]));
            }
    printf("4x4x4_16b f16 layout: max |err| %.3g (expect ~1e-7)\n", e4);
    return 0;
}
