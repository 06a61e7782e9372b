// dpk_metrics.hip — per-frame evaluation of the sampler output on the GPU.
//
// test_hyber (runners/diffpose_frame.py:382-387) averages the test_times hypotheses,
// takes the xyz channels, subtracts the root joint from prediction and target, and
// scores every frame with MPJPE (common/loss.py:7-13; per frame as in
// common/utils.py:103-127) and P-MPJPE, the error after the similarity transform
// (scale, rotation, translation) that best aligns the prediction to the target
// (common/loss.py:25-64, per frame common/utils.py:155-187).  The reference runs the latter on
// the host in float32 numpy, after a device->host copy of the batch.
//
// Here one thread owns one frame and does everything in registers, in fp64.  Rotation: Horn's
// closed form.  The rotation maximising sum_j x_j.(Q y_j) is the quaternion eigenvector of the
// largest eigenvalue of a symmetric 4x4 built from S = Y0^T X0.  That eigenvalue equals the
// reference's sign-corrected singular-value trace s1 + s2 + sign(det R) s3, so reflections
// are excluded exactly as in the SVD formulation.  The 4x4 eigenproblem is solved with cyclic
// Jacobi sweeps.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "diffpose_kernels.h"

namespace dpk_metrics {

constexpr int J = 17;
constexpr int PE = J * 5;

__device__ void jacobi4(double A[4][4], double V[4][4]) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) V[i][j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 16; ++sweep) {
        double off = 0.0, diag = 0.0;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                if (i != j) off += A[i][j] * A[i][j];
                else diag += A[i][j] * A[i][j];
            }
        if (off <= 1e-30 * diag || off == 0.0) break;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                const double apq = A[p][q];
                if (apq == 0.0) continue;
                const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 4; ++k) {       // A <- A J
                    const double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 4; ++k) {       // A <- J^T A
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 4; ++k) {       // V <- V J
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
}

// one thread per frame
__global__ void __launch_bounds__(64) metrics_kernel(const float* __restrict__ out, const float* __restrict__ tgt,
                                                     int F, int H, int root_mode, double* __restrict__ p1,
                                                     double* __restrict__ p2, float* __restrict__ xyz_out) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    float y[J][3], x[J][3];
    // hypothesis mean in fp32, sum over h then / H (torch.mean over dim 0, diffpose_frame.py:382)
    for (int j = 0; j < J; ++j)
        for (int c = 0; c < 3; ++c) {
            float s = 0.f;
            for (int h = 0; h < H; ++h) s += out[((size_t)h * F + f) * PE + j * 5 + 2 + c];
            y[j][c] = H == 1 ? s : s / (float)H;
            x[j][c] = tgt[(size_t)f * J * 3 + j * 3 + c];
        }
    // root handling of prediction and target (diffpose_frame.py:384-385); mode 0 = the aliased
    // in-place subtraction's CPU-torch result (root row zeroed only)
    if (root_mode == 0) {
        for (int c = 0; c < 3; ++c) y[0][c] = x[0][c] = 0.f;
    } else if (root_mode == 1) {
        for (int j = J - 1; j >= 0; --j)
            for (int c = 0; c < 3; ++c) {
                y[j][c] -= y[0][c];
                x[j][c] -= x[0][c];
            }
    }
    if (xyz_out)
        for (int j = 0; j < J; ++j)
            for (int c = 0; c < 3; ++c) xyz_out[(size_t)f * J * 3 + j * 3 + c] = y[j][c];
    // MPJPE
    double e1 = 0.0;
    for (int j = 0; j < J; ++j) {
        const double d0 = (double)y[j][0] - x[j][0], d1 = (double)y[j][1] - x[j][1], d2 = (double)y[j][2] - x[j][2];
        e1 += sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    }
    p1[f] = e1 / J;
    // P-MPJPE
    double mx[3] = {0, 0, 0}, my[3] = {0, 0, 0};
    for (int j = 0; j < J; ++j)
        for (int c = 0; c < 3; ++c) {
            mx[c] += x[j][c];
            my[c] += y[j][c];
        }
    for (int c = 0; c < 3; ++c) {
        mx[c] /= J;
        my[c] /= J;
    }
    double nx = 0.0, ny = 0.0;
    for (int j = 0; j < J; ++j)
        for (int c = 0; c < 3; ++c) {
            const double a = x[j][c] - mx[c], b = y[j][c] - my[c];
            nx += a * a;
            ny += b * b;
        }
    nx = sqrt(nx);
    ny = sqrt(ny);
    double S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};   // S[a][b] = sum_j Y0[j][a] X0[j][b]
    for (int j = 0; j < J; ++j)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) S[a][b] += ((y[j][a] - my[a]) / ny) * ((x[j][b] - mx[b]) / nx);
    double N[4][4] = {
        {S[0][0] + S[1][1] + S[2][2], S[1][2] - S[2][1], S[2][0] - S[0][2], S[0][1] - S[1][0]},
        {S[1][2] - S[2][1], S[0][0] - S[1][1] - S[2][2], S[0][1] + S[1][0], S[2][0] + S[0][2]},
        {S[2][0] - S[0][2], S[0][1] + S[1][0], -S[0][0] + S[1][1] - S[2][2], S[1][2] + S[2][1]},
        {S[0][1] - S[1][0], S[2][0] + S[0][2], S[1][2] + S[2][1], -S[0][0] - S[1][1] + S[2][2]}};
    double V[4][4];
    jacobi4(N, V);
    int k = 0;
    for (int i = 1; i < 4; ++i)
        if (N[i][i] > N[k][k]) k = i;
    const double lam = N[k][k];
    double q0 = V[0][k], qx = V[1][k], qy = V[2][k], qz = V[3][k];
    const double qn = sqrt(q0 * q0 + qx * qx + qy * qy + qz * qz);
    q0 /= qn;
    qx /= qn;
    qy /= qn;
    qz /= qn;
    const double Q[3][3] = {{q0 * q0 + qx * qx - qy * qy - qz * qz, 2 * (qx * qy - q0 * qz), 2 * (qx * qz + q0 * qy)},
                            {2 * (qy * qx + q0 * qz), q0 * q0 - qx * qx + qy * qy - qz * qz, 2 * (qy * qz - q0 * qx)},
                            {2 * (qz * qx - q0 * qy), 2 * (qz * qy + q0 * qx), q0 * q0 - qx * qx - qy * qy + qz * qz}};
    const double sc = lam * nx / ny;                        // scale a = tr * |X0| / |Y0|
    double t[3];
    for (int a = 0; a < 3; ++a)
        t[a] = mx[a] - sc * (Q[a][0] * my[0] + Q[a][1] * my[1] + Q[a][2] * my[2]);
    double e2 = 0.0;
    for (int j = 0; j < J; ++j) {
        double ss = 0.0;
        for (int a = 0; a < 3; ++a) {
            const double al = sc * (Q[a][0] * y[j][0] + Q[a][1] * y[j][1] + Q[a][2] * y[j][2]) + t[a];
            const double d = al - x[j][a];
            ss += d * d;
        }
        e2 += sqrt(ss);
    }
    p2[f] = e2 / J;
}

}  // namespace dpk_metrics

extern "C" int dpk_pose_metrics(const float* out_uvxyz, const float* targets, int F, int H, int root_mode,
                                double* p1, double* p2, float* xyz, void* stream) {
    if (F < 0 || H < 1 || root_mode < 0 || root_mode > 2) return DPK_E_INVALID;
    if (F == 0) return DPK_OK;
    if (!out_uvxyz || !targets || !p1 || !p2) return DPK_E_INVALID;
    hipLaunchKernelGGL(dpk_metrics::metrics_kernel, dim3((F + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                       out_uvxyz, targets, F, H, root_mode, p1, p2, xyz);
    return hipGetLastError() == hipSuccess ? DPK_OK : DPK_E_HIP;
}
