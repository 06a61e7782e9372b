// dpk_gmm.hip — GMM 2D-keypoint sampling of the evaluation/training input pipeline on the GPU
// (SURVEY §8 f3).
//
// PoseGenerator_gmm.__getitem__ (common/generators.py:24-53) picks, for every joint of a frame,
// one of the kernel_n Gaussian components of its 2D detection with
// np.random.choice(kernel_n, 1, p=weights) and emits
//     uvxyz       = [mu_u, mu_v, x, y, z]          (x, y, z root-relative, generators.py:19)
//     noise_scale = [var_u, var_v, 1, 1, 1]
// The reference does this per frame in Python inside DataLoader workers.  Here one thread owns one
// (frame, joint): it re-implements numpy's legacy RandomState.choice selection in fp64 —
// weights converted to double, cdf = sequential cumsum, cdf /= cdf[-1], index =
// searchsorted(cdf, u, side='right') — so, given the same uniform draw u, the component is the one
// numpy picks, bit for bit.  numpy's argument checks are kept as status flags (negative weight;
// Kahan sum of the weights off 1 by more than atol), which the host turns into the same ValueError.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "diffpose_kernels.h"

namespace dpk_gmm {

constexpr int J = 17;
constexpr int KMAX = 64;   // components per joint accepted by the kernel

// uniform double in [0, 1) with 53 random bits from a counter (seeded mode; not numpy's stream)
__device__ __forceinline__ double counter_uniform(uint64_t seed, uint64_t ctr) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (ctr + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// T: the dtype of the caller's arrays (float32, or float64 as numpy would hold them).  The choice
// runs on double(p) either way (numpy converts p to double); with float64 arrays the root-relative
// subtraction happens in double and only the outputs are rounded to float32, as the reference's
// `.float()` at generators.py:46-50 does.
template <typename T>
__global__ void gmm_sample_kernel(const T* __restrict__ gmm, const T* __restrict__ poses3d, int n_src,
                                  int kn, const int64_t* __restrict__ index, int F, const double* __restrict__ u,
                                  uint64_t seed, double atol, float* __restrict__ uvxyz,
                                  float* __restrict__ noise_scale, int* __restrict__ status) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= F * J) return;
    const int f = gid / J, j = gid - f * J;
    int64_t src = index ? index[f] : f;
    src %= n_src;                                    // generators.py:26-29 (index wraps)
    if (src < 0) src += n_src;
    const T* row = gmm + ((size_t)src * J + j) * (size_t)kn * 5;
    // np.random.choice argument checks (mtrand.pyx): p >= 0, |kahan_sum(p) - 1| <= atol
    int flags = 0;
    double ksum = (double)row[0], c = 0.0;
    if (row[0] < T(0)) flags |= 1;
    for (int k = 1; k < kn; ++k) {
        const double pk = (double)row[k * 5];
        if (pk < 0.0) flags |= 1;
        const double y = pk - c;
        const double t = ksum + y;
        c = (t - ksum) - y;
        ksum = t;
    }
    if (fabs(ksum - 1.0) > atol) flags |= 2;
    if (flags) atomicOr(status, flags);
    // cdf = p.cumsum(); cdf /= cdf[-1]; idx = cdf.searchsorted(uniform, side='right')
    double cdf[KMAX];
    double acc = 0.0;
    for (int k = 0; k < kn; ++k) {
        acc += (double)row[k * 5];
        cdf[k] = acc;
    }
    const double last = cdf[kn - 1];
    const double uu = u ? u[gid] : counter_uniform(seed, (uint64_t)gid);
    int idx = 0;
    for (int k = 0; k < kn; ++k) idx += (cdf[k] / last <= uu) ? 1 : 0;   // cdf is non-decreasing
    if (idx > kn - 1) idx = kn - 1;      // only reachable with invalid weights (flagged above)
    const T* comp = row + idx * 5;
    const T* p3 = poses3d + (size_t)src * J * 3;
    float* o = uvxyz + (size_t)gid * 5;
    float* s = noise_scale + (size_t)gid * 5;
    o[0] = (float)comp[1];
    o[1] = (float)comp[2];
    s[0] = (float)comp[3];
    s[1] = (float)comp[4];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        o[2 + d] = (float)(p3[j * 3 + d] - p3[d]);  // root-relative in the arrays' dtype, then .float()
        s[2 + d] = 1.0f;
    }
}

}  // namespace dpk_gmm

template <typename T>
static int gmm_launch(const T* gmm_dev, const T* poses3d_dev, int n_src, int kernel_n, const int64_t* index_dev, int F,
                      const double* u_dev, uint64_t seed, double atol, float* uvxyz_dev, float* noise_scale_dev,
                      int* status_dev, void* stream) {
    if (F < 0 || n_src <= 0 || kernel_n < 1 || kernel_n > dpk_gmm::KMAX) return DPK_E_INVALID;
    if (F == 0) return DPK_OK;
    if (!gmm_dev || !poses3d_dev || !uvxyz_dev || !noise_scale_dev || !status_dev) return DPK_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(status_dev, 0, sizeof(int), st) != hipSuccess) return DPK_E_HIP;
    const int n = F * dpk_gmm::J, nt = 256;
    hipLaunchKernelGGL(dpk_gmm::gmm_sample_kernel<T>, dim3((n + nt - 1) / nt), dim3(nt), 0, st, gmm_dev, poses3d_dev,
                       n_src, kernel_n, index_dev, F, u_dev, seed, atol, uvxyz_dev, noise_scale_dev, status_dev);
    return hipGetLastError() == hipSuccess ? DPK_OK : DPK_E_HIP;
}

extern "C" int dpk_gmm_sample(const float* gmm_dev, const float* poses3d_dev, int n_src, int kernel_n,
                              const int64_t* index_dev, int F, const double* u_dev, uint64_t seed, double atol,
                              float* uvxyz_dev, float* noise_scale_dev, int* status_dev, void* stream) {
    return gmm_launch(gmm_dev, poses3d_dev, n_src, kernel_n, index_dev, F, u_dev, seed, atol, uvxyz_dev,
                      noise_scale_dev, status_dev, stream);
}

extern "C" int dpk_gmm_sample_f64(const double* gmm_dev, const double* poses3d_dev, int n_src, int kernel_n,
                                  const int64_t* index_dev, int F, const double* u_dev, uint64_t seed, double atol,
                                  float* uvxyz_dev, float* noise_scale_dev, int* status_dev, void* stream) {
    return gmm_launch(gmm_dev, poses3d_dev, n_src, kernel_n, index_dev, F, u_dev, seed, atol, uvxyz_dev,
                      noise_scale_dev, status_dev, stream);
}
