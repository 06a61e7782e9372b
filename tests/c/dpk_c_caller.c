/* dpk_c_caller.c — a plain-C caller of libdpk.so through include/diffpose_kernels.h only (no Python,
 * no torch): the C binding INTEGRATION.md §4 describes, run end to end.
 *
 *   dpk_c_caller WEIGHTS.bin N K OUT.bin
 *
 * WEIGHTS.bin (written by tests/test_c_caller.py): int32 count, then per state_dict entry
 * int32 name_len, name bytes, int64 numel, numel float32.  The program builds the H36M adjacency
 * (runners/diffpose_frame.py:120-124, models/GraFormer.py:32-44), the linear beta schedule's
 * alpha_bar table (common/utils_diff.py:7-43) and the uniform skip seq over T'=50 (K steps,
 * runners/diffpose_frame.py:310-317), draws N deterministic poses, runs dpk_sample under tail
 * plans 2 and 0 and writes: int32 N, the N*17*5 inputs, the plan-2 outputs, then int32 equal
 * (plan 2 == plan 0 bitwise).  Exit 0 on success.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "diffpose_kernels.h"

/* the six HIP runtime entry points this caller needs (C linkage in libamdhip64), declared here so
 * that a plain C compiler needs no HIP headers */
typedef void* hipStream_t;
enum { hipSuccess = 0, hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2 };
extern int hipMalloc(void** p, size_t size);
extern int hipFree(void* p);
extern int hipMemcpy(void* dst, const void* src, size_t size, int kind);
extern int hipStreamCreate(hipStream_t* s);
extern int hipStreamSynchronize(hipStream_t s);
extern int hipStreamDestroy(hipStream_t s);

#define CHECK(x)                                                                  \
    do {                                                                          \
        int rc_ = (x);                                                            \
        if (rc_ != 0) {                                                           \
            fprintf(stderr, "%s failed: %d %s\n", #x, rc_, h ? dpk_last_error(h) : ""); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

static const int EDGES[16][2] = {{0, 1}, {1, 2}, {2, 3}, {0, 4}, {4, 5}, {5, 6}, {0, 7}, {7, 8},
                                 {8, 9}, {9, 10}, {8, 11}, {11, 12}, {12, 13}, {8, 14}, {14, 15}, {15, 16}};

int main(int argc, char** argv) {
    dpk_handle* h = NULL;
    if (argc != 5) {
        fprintf(stderr, "usage: %s WEIGHTS.bin N K OUT.bin\n", argv[0]);
        return 2;
    }
    const int N = atoi(argv[2]), K = atoi(argv[3]);
    if (N < 1 || K < 1 || K > 50) return 2;

    /* state_dict */
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 3;
    int32_t count = 0;
    if (fread(&count, 4, 1, f) != 1 || count <= 0) return 3;
    char** names = (char**)calloc((size_t)count, sizeof(char*));
    float** data = (float**)calloc((size_t)count, sizeof(float*));
    int64_t* numels = (int64_t*)calloc((size_t)count, sizeof(int64_t));
    for (int i = 0; i < count; ++i) {
        int32_t len = 0;
        if (fread(&len, 4, 1, f) != 1 || len <= 0 || len > 256) return 3;
        names[i] = (char*)calloc((size_t)len + 1, 1);
        if (fread(names[i], 1, (size_t)len, f) != (size_t)len) return 3;
        if (fread(&numels[i], 8, 1, f) != 1 || numels[i] <= 0) return 3;
        data[i] = (float*)malloc((size_t)numels[i] * 4);
        if (fread(data[i], 4, (size_t)numels[i], f) != (size_t)numels[i]) return 3;
    }
    fclose(f);

    /* GCNdiff(adj, config): hid 96, 5 layers, 4 heads, 17 joints, coords [5,5] */
    dpk_config cfg = {96, 5, 4, 17, 5, 5, 0};
    CHECK(dpk_create(&cfg, &h));
    float adj[17 * 17];
    memset(adj, 0, sizeof(adj));
    for (int e = 0; e < 16; ++e) {
        adj[EDGES[e][0] * 17 + EDGES[e][1]] = 1.f;
        adj[EDGES[e][1] * 17 + EDGES[e][0]] = 1.f;
    }
    for (int i = 0; i < 17; ++i) {
        adj[i * 17 + i] += 1.f;
        float s = 0.f;
        for (int j = 0; j < 17; ++j) s += adj[i * 17 + j];
        const float r = 1.f / s;
        for (int j = 0; j < 17; ++j) adj[i * 17 + j] *= r;
    }
    CHECK(dpk_set_graph(h, adj));
    CHECK(dpk_load_weights(h, (const char* const*)names, (const float* const*)data, numels, count));

    /* schedule: betas = linspace(1e-4, 1e-3, 51) in double, alpha_bar = cumprod(1 - cat(0, betas)) in fp32
     * accumulated in double (torch's CPU cumprod), seq = range(0, 50, 50 / K) */
    float abar[52];
    double acc = 1.0;
    abar[0] = 1.f;
    for (int t = 0; t < 51; ++t) {
        const float beta = (float)(1e-4 + (1e-3 - 1e-4) * (double)t / 50.0);
        acc *= (double)(1.0f - beta);
        abar[t + 1] = (float)acc;
    }
    int seq[50];
    const int skip = 50 / K;
    for (int s = 0; s < K; ++s) seq[s] = s * skip;
    CHECK(dpk_set_schedule(h, abar, 52, seq, K, 0.f));

    /* inputs: deterministic uvxyz-like values in [-0.5, 0.5] */
    const size_t n = (size_t)N * 17 * 5;
    float* hx = (float*)malloc(n * 4);
    uint32_t st = 12345u;
    for (size_t i = 0; i < n; ++i) {
        st = st * 1664525u + 1013904223u;
        hx[i] = (float)(st >> 8) / 16777216.0f - 0.5f;
    }
    float *dx = NULL, *d2 = NULL, *d0 = NULL;
    if (hipMalloc((void**)&dx, n * 4) != hipSuccess || hipMalloc((void**)&d2, n * 4) != hipSuccess ||
        hipMalloc((void**)&d0, n * 4) != hipSuccess)
        return 4;
    if (hipMemcpy(dx, hx, n * 4, hipMemcpyHostToDevice) != hipSuccess) return 4;
    hipStream_t stream;
    if (hipStreamCreate(&stream) != hipSuccess) return 4;
    CHECK(dpk_set_tail_plan(h, 2));
    CHECK(dpk_sample(h, dx, d2, NULL, NULL, N, 0, (void*)stream));
    CHECK(dpk_set_tail_plan(h, 0));
    CHECK(dpk_sample(h, dx, d0, NULL, NULL, N, 0, (void*)stream));
    if (hipStreamSynchronize(stream) != hipSuccess) return 4;
    float* o2 = (float*)malloc(n * 4);
    float* o0 = (float*)malloc(n * 4);
    if (hipMemcpy(o2, d2, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(o0, d0, n * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 4;
    const int32_t equal = memcmp(o2, o0, n * 4) == 0;

    FILE* g = fopen(argv[4], "wb");
    if (!g) return 5;
    const int32_t nn = N;
    fwrite(&nn, 4, 1, g);
    fwrite(hx, 4, n, g);
    fwrite(o2, 4, n, g);
    fwrite(&equal, 4, 1, g);
    fclose(g);

    dpk_destroy(h);
    (void)hipFree(dx);
    (void)hipFree(d2);
    (void)hipFree(d0);
    (void)hipStreamDestroy(stream);
    for (int i = 0; i < count; ++i) {
        free(names[i]);
        free(data[i]);
    }
    free(names);
    free(data);
    free(numels);
    free(hx);
    free(o2);
    free(o0);
    printf("dpk_c_caller: N=%d K=%d plan2==plan0 %s\n", N, K, equal ? "bitwise" : "DIFFERENT");
    return equal ? 0 : 6;
}
