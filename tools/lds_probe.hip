// Does a kernel get more than 64 KB of dynamic LDS on gfx950?  (tools/lds_probe.hip)
// Build: hipcc --offload-arch=gfx950 -O2 tools/lds_probe.hip -o build/lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) fill(float* out, int n) {
    extern __shared__ float sm[];
    for (int i = threadIdx.x; i < n; i += 256) sm[i] = (float)i;
    __syncthreads();
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) s += sm[n - 1 - i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    float* d;
    if (hipMalloc(&d, 1024 * 256 * 4) != hipSuccess) return 1;
    for (int kb : {32, 64, 96, 128, 156}) {
        const size_t bytes = (size_t)kb * 1024;
        hipError_t a = hipFuncSetAttribute((const void*)fill, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), bytes, 0, d, (int)(bytes / 4));
        hipError_t l = hipGetLastError();
        hipError_t s = hipDeviceSynchronize();
        float h[256];
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        double tot = 0;
        for (float v : h) tot += v;
        const double n = bytes / 4, want = n * (n - 1) / 2;
        printf("%3d KB: setattr %s, launch %s, sync %s, block-0 sum %.0f (want %.0f)\n", kb, hipGetErrorString(a),
               hipGetErrorString(l), hipGetErrorString(s), tot, want);
    }
    return 0;
}
