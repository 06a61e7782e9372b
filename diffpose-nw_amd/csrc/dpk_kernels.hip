// dpk_kernels.hip — MI355X (gfx950, CDNA4) DDIM sampler for DiffPose's GCNdiff denoiser.
//
// One persistent kernel runs the whole K-step reverse-diffusion loop of the reference
// (common/utils_diff.py:46-68) for a tile of P=4 poses per workgroup: every step's
// GCNdiff forward (models/gcndiff.py:101-113) and the DDIM update happen in LDS, so the
// only HBM traffic is the (N,17,5) input, the output and the weights (L2/MALL-resident).
//
// Tile geometry: 4 poses = 68 rows of 96 features; Linear/ChebConv
// GEMMs run on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32 fma chains) over 4 row tiles
// of 16 (each wave: 2 row tiles x half the columns), the 4 leftover rows on the VALU inside
// the same k-loop.  LayerNorm, 17-joint attention and the 17x17 graph products are VALU
// work between workgroup barriers.  Weights are repacked at load time into MFMA
// B-fragment order: one 1 KiB coalesced float4-per-lane load per (16 cols x 16 k) block.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "diffpose_kernels.h"

// Timing-only ablation builds (tools/ablate.py): bit set = phase skipped.  Outputs of such
// a build are wrong by construction; the shipped library is built with DPK_ABLATE=0.
#ifndef DPK_ABLATE
#define DPK_ABLATE 0
#endif
#define DPK_RUN(bit) ((DPK_ABLATE & (bit)) == 0)
// Phase tracing builds (tools/phase_trace.py): lane 0 of every wave stamps s_memtime before and
// after each workgroup barrier of one chosen DDIM step.
#ifndef DPK_TRACE
#define DPK_TRACE 0
#endif
// GEMM phase stamps: tools/gemm_probe.hip defines its own; trace builds stamp into the trace
// buffer (end of k-loop, end of epilogue); empty in the library
#if DPK_TRACE
namespace dpk {
__shared__ unsigned long long* tr_row[8];   // per-wave stamp row of the traced step (null: off)
__shared__ int tr_ix[8];
__device__ __forceinline__ void tr_stamp() {
    const int w = threadIdx.x >> 6;
    if (tr_row[w] && (threadIdx.x & 63) == 0 && tr_ix[w] < 256) tr_row[w][tr_ix[w]] = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0 && tr_row[w]) tr_ix[w] += 1;
}
}  // namespace dpk
#ifndef DPK_GEMM_HOOK
#define DPK_GEMM_HOOK(tag)                       \
    do {                                         \
        if ((tag) != 0) {                        \
            __builtin_amdgcn_sched_barrier(0);   \
            dpk::tr_stamp();                     \
            __builtin_amdgcn_sched_barrier(0);   \
        }                                        \
    } while (0)
#endif
#endif
#ifndef DPK_GEMM_HOOK
#define DPK_GEMM_HOOK(tag)
#endif


// Launch arguments of the sampler kernel, shared by both tile sizes (dpk_sampler.inc).
namespace dpk_shared {
struct SampleArgs {
    const float* arena;   // packed weights
    const float* coef;    // [K][6] = sqrt(1-at), sqrt(at), sqrt(an), c1, c2, t
    const float* tproj;   // [slots][NL][D] temb_proj(swish(temb)) per step (sample) / per pose (eps); zeros (pose)
    const float* x_in;    // [N][17][5]  (pose: [N][17][2] uv)
    float* x_out;         // [N][17][5]  final x (sample) or eps (eps mode); pose: [N][17][3] xyz or null
    float* xs;            // [K+1][N][17][5] or null
    float* x0s;           // [K][N][17][5]   or null
    float* uvxyz;         // pose: [H][N][17][5] cat(uv, root-processed xyz), repeated H times; or null
    int N;
    int K;
    int H;                // pose: test_times
    int root_mode;        // pose: 0 reference in-place quirk (root zeroed), 1 root-relative, 2 raw
    unsigned mask;        // 17-bit key mask
    const unsigned* pmask;  // per-pose 17-bit key masks [N] (dpk_set_pose_masks), or null: `mask` for all
    float eta;
    unsigned long long seed;
    int pose_off;         // first pose of this launch (a batch split over two launches, see launch_sampler)
    int num_layers;       // GraAttenLayer + _ResChebGC_diff pairs run (config num_layer, 1..NL)
    // Step-split last round (sample mode, launch_sampler): the last split_n tiles run their K steps
    // as two halves on two workgroups.  Blocks [0, split_n) run steps [0, split_k) of tiles
    // split_full + b and publish x_t through x_out and flags[b]; blocks [split_n, split_n + split_full)
    // run whole tiles; the last split_n blocks wait for their tile's flag and run [split_k, K).
    int split_n;
    int split_k;
    int split_full;
    unsigned* flags;      // [split_n] handoff words: 0 between launches, (token << 2) | state during one
    unsigned token;       // nonzero, per launch (30 bits)
    // (round 4; after the round-3 fields so their kernel-argument offsets, and the code built around
    // them, stay as they were)
    const float* noise;   // [K][N][17][5] caller noise for c1*z (the reference's per-step randn_like), or null
    int* split_stats;     // device counter: second halves that recomputed their first half's steps
    int split_dbg;        // dpk_debug_split: 0 normal; 1 first halves start late; 2 no idle wait
#if DPK_TRACE
    unsigned long long* trace;   // [blocks][NW][TRACE_SLOTS]
    int trace_step;
#endif
};
}  // namespace dpk_shared

#define DPK_P 4
namespace dpk {
#include "dpk_sampler.inc"
}  // namespace dpk
#undef DPK_P
#define DPK_P 2
namespace dpk2 {
#include "dpk_sampler.inc"
}  // namespace dpk2
// The persistent sampler at a wider model (round 5): hid 128 / 8 heads (d_k 16), 2-pose tiles (4-pose
// tiles of 128-wide rows do not fit 160 KB of LDS), fp32 GEMMs; run by the generic-shape path for that
// shape instead of its per-op launches (dpk_generic.inc, GenFused)
#undef DPK_P
#define DPK_P 2
#undef DPK_D
#undef DPK_NH
#define DPK_D 128
#define DPK_NH 8
namespace dpkw {
#include "dpk_sampler.inc"
}  // namespace dpkw
#undef DPK_NH
#undef DPK_D
#undef DPK_P
// ... at hid 128 / 4 heads (d_k 32), 2-pose tiles
#define DPK_P 2
#define DPK_D 128
#define DPK_NH 4
namespace dpkw4 {
#include "dpk_sampler.inc"
}  // namespace dpkw4
#undef DPK_NH
#undef DPK_D
#undef DPK_P
// ... and at hid 64 / 2 heads (d_k 32; the generic-shape tests' width) and hid 64 / 4 heads (d_k 16), 4-pose
// tiles (129 KB of LDS)
#define DPK_P 4
#define DPK_D 64
#define DPK_NH 2
namespace dpkn {
#include "dpk_sampler.inc"
}  // namespace dpkn
#undef DPK_NH
#define DPK_NH 4
namespace dpkn4 {
#include "dpk_sampler.inc"
}  // namespace dpkn4
#undef DPK_NH
#undef DPK_D
#undef DPK_P

namespace dpk {

// ---------------------------------------------------------------------------------------
// Elementwise DDIM update for externally computed eps; z from the caller's draws of this step
// (`noise`, n floats) or counter-based.
__global__ void __launch_bounds__(256) ddim_kernel(const float* __restrict__ xt, const float* __restrict__ et,
                                                   float* __restrict__ xn, float* __restrict__ x0o, long long n,
                                                   const float* __restrict__ cf, int step, float eta,
                                                   unsigned long long seed, const float* __restrict__ noise) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float z = noise ? noise[i] : (eta != 0.f ? normal_noise(seed, step, i) : 0.f);
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

// One DDIM schedule on the device, immutable once built: the step scalars coef [K][6] and the
// per-step timestep projections tps [K][NL][D] = temb_proj_l(swish(temb(t_s))) (they depend only
// on the weights and the schedule; SURVEY a7: batch-invariant).  dpk_set_schedule builds a new one
// instead of rewriting the old, so a launch still in flight (or a captured graph) keeps reading
// the schedule it was launched with; the old one is freed once every stream that used it has
// passed its last launch (an event per stream), or never if a graph was captured with it.
struct Sched {
    uint64_t serial = 0;           // unique per schedule built (keys the generic path's loop graphs)
    float* buf = nullptr;          // device: coef, then tps (16-byte aligned)
    float* coef = nullptr;
    float* tps = nullptr;
    int K = 0;
    float eta = 0.f;
    std::vector<float> h_coef;
    uint64_t tps_gen = 0;          // weights generation tps was computed from (0: not yet)
    int pins = 0;                  // captured graphs that read it (CapRes): kept while any is alive
    std::vector<std::pair<hipStream_t, hipEvent_t>> uses;   // last launch on each stream
};

// dpk_eps's per-pose projections [N][NL][D].  Uncaptured calls use one buffer per caller stream:
// two dpk_eps calls on different streams never share one, and calls on the same stream are ordered
// by the stream, so a buffer can grow (after a sync of its stream) without racing anyone.  A
// captured call becomes a graph node that keeps the buffer's address for the graph's life and may
// replay on any stream, concurrently with other graphs: it takes a buffer of its own, the handle's
// spare (allocated by the uncaptured calls, since nothing can be allocated inside a capture), and
// that buffer is pinned until dpk_destroy.
struct EpsBuf {
    hipStream_t st = nullptr;
    float* p = nullptr;
    int cap = 0;
};

// What the launches captured in one stream capture (one hipGraph) read by address: the schedules
// they were captured with, dpk_eps projection buffers (one per capturing stream: the captured
// launches of one stream are sequential graph nodes and share it) and step-split flag slots (one
// per capturing stream likewise).  A HIP user object retained by the capture's graph drops the
// graph's reference when the graph and its executable instances are destroyed (host callback, no
// HIP calls); the handle's next uncaptured call then waits for the device once and recycles the
// resources.  Where the runtime cannot retain one, they are kept until dpk_destroy.
struct CapRes {
    unsigned long long id = 0;                 // capture sequence id (hipStreamGetCaptureInfo_v2)
    std::atomic<int> refs{1};                  // the handle's reference (+1 while a graph holds one)
    std::atomic<bool> released{false};
    bool tracked = false;                      // a graph retains our user object
    std::vector<Sched*> scheds;
    std::vector<EpsBuf> eps;                   // per capturing stream
    std::vector<std::pair<hipStream_t, int>> slots;   // flag slot per capturing stream
    // generic-shape path: the activation scratch of each capturing stream (taken from the model's
    // spare, which uncaptured generic calls size; dpk_generic.inc gen_scratch_cap)
    struct GenBuf {
        hipStream_t st;
        float* p;
        size_t cap;   // floats
    };
    std::vector<GenBuf> gen;
};
static void cap_release_cb(void* p) {
    CapRes* c = static_cast<CapRes*>(p);
    c->released.store(true);
    if (c->refs.fetch_sub(1) == 1) delete c;
}

struct GenModel;   // dpk_generic.inc: the forward for model shapes other than the compiled one
struct dpk_handle;
static void gen_spare_put(dpk_handle* h, float* p, size_t cap);   // dpk_generic.inc

struct dpk_handle {
    int device = 0;
    GenModel* gen = nullptr;       // non-null: this handle's shape runs on the generic path
    int n_pts = J;                 // joints of the handle's model
    int kind = 0;                  // 0: GCNdiff (coords 5->5), 1: GCNpose (coords 2->3)
    int num_layers = NL;           // config num_layer (1..NL): layers the kernels run
    int n_cu = 256;                // compute units of the device (workgroups per round)
    int tail_plan = 2;             // dpk_set_tail_plan: 0 4-pose tiles, 1 2-pose tail round, 2 step split
    unsigned* flags = nullptr;     // device: FLAG_SLOTS x n_cu step-split handoff words (zero between launches),
                                   // then the split fallback counter
    std::vector<int> slot_free;    // flag slots no launch holds
    std::vector<std::pair<int, hipEvent_t>> slot_busy;   // uncaptured launches: slot until its event completes
    std::vector<hipEvent_t> slot_ev;   // idle events for slot_busy
    int split_dbg = 0;             // dpk_debug_split mode
    unsigned token = 0;            // per-launch handoff token (30 bits, never 0)
    std::vector<CapRes*> caps;     // resources of captured launches (per capture)
    std::string err;
    float* arena = nullptr;        // device: packed weights + graph constants
    float* temb = nullptr;         // device: timestep-MLP weights
    float* tproj_zero = nullptr;   // device: [NL][D] zeros (GCNpose: no timestep projection)
    hipStream_t aux = nullptr;     // handle-internal stream for schedule construction
    uint64_t weights_gen = 0;      // bumped by every weight/graph upload
    Sched* sched = nullptr;        // current schedule
    std::vector<Sched*> retired;   // replaced schedules not yet known to be unused
    std::vector<EpsBuf> eps_bufs;  // per stream (uncaptured dpk_eps)
    EpsBuf eps_spare;              // unused buffer for the next capture's dpk_eps (no stream)
    std::vector<float> h_arena;    // host staging of the arena
    char* arena16 = nullptr;       // device: split-fp16 GEMM weights (gemm mode 1)
    std::vector<uint16_t> h_arena16;
    char* arenabf = nullptr;       // device: bf16 GEMM weights (gemm mode 2), same layout
    std::vector<uint16_t> h_arenabf;
    int gemm_mode = 0;             // 0: fp32 MFMA, 1: 3x fp16-split MFMA, 2: bf16 MFMA (dpk_set_gemm_mode)
    bool w16_ok = true;            // loaded weights fit the split-fp16 packing (|w| < 1015)
    std::vector<float> h_temb;
    bool have_graph = false, have_weights = false;
    unsigned mask = (1u << J) - 1u;
    const unsigned* pmask = nullptr;   // dpk_set_pose_masks: caller-owned device array
    int pmask_n = 0;
    std::vector<float> h_adj;
    bool profiling = false;
    bool sparse_graph = false;     // adjacency matches the compiled H36M Chebyshev pattern
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used, ev_free;
#if DPK_TRACE
    unsigned long long* trace = nullptr;
    size_t trace_len = 0;
    int trace_step = -1;
#endif
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

// Host fp32 -> bf16, round to nearest even (finite inputs).
static inline uint16_t bf16_rne(float v) {
    uint32_t u = __builtin_bit_cast(uint32_t, v);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
static inline float bf16_to_f32(uint16_t b) { return __builtin_bit_cast(float, (uint32_t)b << 16); }

// Split W_eff * W16_SCALE into 16x16x32 B fragments for the half-width-operand GEMMs (gemmh_pass):
// lane l holds column n = ct*16 + (l&15) at the 8 k of its lane group g = l>>4 in the order
// 4g..4g+3, 16+4g..16+4g+3 of the 32-block (the A fragments' order: two fp32 16x16x4 fragments).
// BF = false (gemm mode 1, f16x3): blocks [NC][KB32][hi 1 KiB | lo 1 KiB], hi = fp16(v) (RNE),
//   lo = fp16(v - hi) (v - hi is exact in fp32, Sterbenz);
// BF = true (gemm mode 2, bf16): blocks [NC][KB32][1 KiB] of bf16(v) (RNE).
template <bool BF = false, class F>
static float pack16(uint16_t* dst, int Kreal, int Nreal, int KB32, int NC, F w) {
    constexpr size_t blk = BF ? 512 : 1024;      // uint16 per block
    float wmax = 0.f;
    for (int ct = 0; ct < NC; ++ct)
        for (int kb = 0; kb < KB32; ++kb)
            for (int lane = 0; lane < 64; ++lane)
                for (int i = 0; i < 8; ++i) {
                    const int g = lane >> 4;
                    const int k = kb * 32 + (i < 4 ? 4 * g + i : 16 + 4 * g + (i - 4));
                    const int n = ct * 16 + (lane & 15);
                    const float v = (k < Kreal && n < Nreal) ? w(k, n) * W16_SCALE : 0.f;
                    wmax = fmaxf(wmax, fabsf(v));
                    const size_t base = (size_t)(ct * KB32 + kb) * blk;
                    if constexpr (BF) {
                        dst[base + lane * 8 + i] = bf16_rne(v);
                    } else {
                        const _Float16 hi = (_Float16)v;
                        const _Float16 lo = (_Float16)(v - (float)hi);
                        dst[base + lane * 8 + i] = __builtin_bit_cast(uint16_t, hi);
                        dst[base + 512 + lane * 8 + i] = __builtin_bit_cast(uint16_t, lo);
                    }
                }
    return wmax;
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

// Is `st` capturing a graph right now?  (Launches then become graph nodes: nothing may be
// allocated or freed, and the schedule they read must outlive the graph.)
static int capturing(dpk_handle* h, hipStream_t st, bool* cap) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIPCHK(h, hipStreamIsCapturing(st, &cs));
    *cap = cs != hipStreamCaptureStatusNone;
    return DPK_OK;
}

static void sched_free(Sched* s) {
    if (s->buf) (void)hipFree(s->buf);
    for (auto& u : s->uses) (void)hipEventDestroy(u.second);
    delete s;
}

// Free the retired schedules whose every recorded use has completed (never one a live graph reads).
static void sched_sweep(dpk_handle* h) {
    std::vector<Sched*> keep;
    for (Sched* s : h->retired) {
        bool done = s->pins == 0;
        for (auto& u : s->uses) done = done && hipEventQuery(u.second) == hipSuccess;
        if (done) sched_free(s);
        else keep.push_back(s);
    }
    h->retired.swap(keep);
}

// The CapRes of the capture `st` is recording into (created on its first captured launch).
static int cap_get(dpk_handle* h, hipStream_t st, CapRes** out) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    HIPCHK(h, hipStreamGetCaptureInfo_v2(st, &cs, &id, &graph, nullptr, nullptr));
    for (CapRes* c : h->caps)
        if (c->id == id) {
            *out = c;
            return DPK_OK;
        }
    CapRes* c = new CapRes();
    c->id = id;
    // hand the graph a user object that releases the resources with it (DPK_CAPTURE_RELEASE=0: keep them
    // until dpk_destroy instead)
    const char* env = getenv("DPK_CAPTURE_RELEASE");
    if (graph && !(env && atoi(env) == 0)) {
        c->refs.fetch_add(1);              // the graph's reference (dropped by cap_release_cb)
        hipUserObject_t obj = nullptr;
        if (hipUserObjectCreate(&obj, c, cap_release_cb, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
            c->refs.fetch_sub(1);
            (void)hipGetLastError();
        } else if (hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipUserObjectRelease(obj, 1);   // runs the callback: drops the graph's reference
        } else {
            c->tracked = true;
        }
    }
    h->caps.push_back(c);
    *out = c;
    return DPK_OK;
}

static void slot_put(dpk_handle* h, int slot) { h->slot_free.push_back(slot); }

// Wait for the device in relaxed capture mode: a thread capturing in global mode (torch.cuda.graph's
// default) would otherwise see this potentially unsafe call invalidate its capture.  false (error
// cleared) if the runtime refuses the sync, e.g. while a stream of the device is capturing.
static bool drain_relaxed() {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    const bool exch = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
    const hipError_t se = hipDeviceSynchronize();
    if (exch) (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (se != hipSuccess) (void)hipGetLastError();
    return se == hipSuccess;
}

// Uncaptured calls only: recycle the resources of captures whose graphs are gone.  No drain: the release
// callback runs when the graph's executable is destroyed, and on this runtime destroying an executable
// waits for its launches in flight (tools/probe_user_object_release.py: deleting a CUDAGraph 0.1 ms after
// its 175 ms replay was enqueued returned when the replay had finished, and `released` was never seen
// set while it ran), so nothing the capture reads is still in use.  A drain here, even in relaxed capture
// mode, invalidates another thread's global-mode capture on this runtime (round 4 without the relaxed
// mode, advisor r04; round 6 with it, ADVICE r05: test_sweep_while_another_thread_captures failed with
// hipErrorStreamCaptureInvalidated), so the recycling relies on that blocking destruction.
static void cap_sweep(dpk_handle* h) {
    bool any = false;
    for (CapRes* c : h->caps) any = any || (c->tracked && c->released.load());
    if (!any) return;
    std::vector<CapRes*> keep;
    for (CapRes* c : h->caps) {
        if (!(c->tracked && c->released.load())) {
            keep.push_back(c);
            continue;
        }
        for (Sched* s : c->scheds) --s->pins;
        for (auto& e : c->eps) {
            if (!h->eps_spare.p || h->eps_spare.cap < e.cap) {
                if (h->eps_spare.p) (void)hipFree(h->eps_spare.p);
                h->eps_spare = EpsBuf{nullptr, e.p, e.cap};
            } else {
                (void)hipFree(e.p);
            }
        }
        for (auto& s : c->slots) slot_put(h, s.second);
        for (auto& gb : c->gen) gen_spare_put(h, gb.p, gb.cap);
        if (c->refs.fetch_sub(1) == 1) delete c;
    }
    h->caps.swap(keep);
    sched_sweep(h);
}

// After enqueuing a launch that reads `s` on `st`: pin it to the capture if the launch was
// captured, else record its completion on that stream.
static int sched_note_use(dpk_handle* h, Sched* s, hipStream_t st, bool cap) {
    if (cap) {
        CapRes* c = nullptr;
        const int rc = cap_get(h, st, &c);
        if (rc) return rc;
        if (std::find(c->scheds.begin(), c->scheds.end(), s) == c->scheds.end()) {
            c->scheds.push_back(s);
            ++s->pins;
        }
        return DPK_OK;
    }
    hipEvent_t ev = nullptr;
    for (auto& u : s->uses)
        if (u.first == st) ev = u.second;
    if (!ev) {
        HIPCHK(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        s->uses.push_back({st, ev});
    }
    HIPCHK(h, hipEventRecord(ev, st));
    return DPK_OK;
}

// tps of `s` from the current weights, on the handle's own stream; returns once they are written
static int sched_compute_tps(dpk_handle* h, Sched* s) {
    hipLaunchKernelGGL(temb_kernel, dim3(s->K), dim3(256), 0, h->aux, h->temb, s->coef + 5, 6, s->tps);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->aux));
    s->tps_gen = h->weights_gen;
    return DPK_OK;
}

static int upload(dpk_handle* h) {
    HIPCHK(h, hipSetDevice(h->device));
    // launches already enqueued on any stream may still read the arena: overwrite it only after
    // the device has drained (weights and graphs are loaded rarely; the launches stay async)
    HIPCHK(h, hipDeviceSynchronize());
    // every uncaptured launch has completed: the retired schedules only they used go now, so the
    // projections below are recomputed for the current schedule and the graph-pinned ones only
    sched_sweep(h);
    if (!h->arena) HIPCHK(h, hipMalloc(&h->arena, (size_t)ARENA_FLOATS * 4));
    if (!h->arena16) HIPCHK(h, hipMalloc(&h->arena16, (size_t)ARENA16_BYTES));
    HIPCHK(h, hipMemcpy(h->arena16, h->h_arena16.data(), (size_t)ARENA16_BYTES, hipMemcpyHostToDevice));
    if (!h->arenabf) HIPCHK(h, hipMalloc(&h->arenabf, (size_t)ARENAB_BYTES));
    HIPCHK(h, hipMemcpy(h->arenabf, h->h_arenabf.data(), (size_t)ARENAB_BYTES, hipMemcpyHostToDevice));
    if (!h->temb) HIPCHK(h, hipMalloc(&h->temb, (size_t)TEMB_FLOATS * 4));
    HIPCHK(h, hipMemcpy(h->arena, h->h_arena.data(), (size_t)ARENA_FLOATS * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->temb, h->h_temb.data(), (size_t)TEMB_FLOATS * 4, hipMemcpyHostToDevice));
    ++h->weights_gen;
    if (!h->have_weights || h->kind != 0) return DPK_OK;
    // every live schedule (current, retired, pinned by a graph) follows the new weights
    if (h->sched) {
        const int rc = sched_compute_tps(h, h->sched);
        if (rc) return rc;
    }
    for (Sched* s : h->retired) {
        const int rc = sched_compute_tps(h, s);
        if (rc) return rc;
    }
    return DPK_OK;
}

// Flag slots of step-split launches (launch_sampler).  No two launches that may overlap share a slot:
// an uncaptured launch holds one until an event recorded behind it has completed (checked at the
// next launch), a captured one for the life of its graph (shared by the captured launches of one
// stream, which are sequential graph nodes; every launch leaves its words at 0).  -1 when all are
// held (the caller then runs the 2-pose tail plan).
constexpr int FLAG_SLOTS = 64;
static int split_slot(dpk_handle* h, hipStream_t st, bool cap) {
    if (!h->flags) return -1;
    if (cap) {
        CapRes* c = nullptr;
        if (cap_get(h, st, &c)) return -1;
        for (auto& s : c->slots)
            if (s.first == st) return s.second;
        if (h->slot_free.empty()) return -1;
        const int slot = h->slot_free.back();
        h->slot_free.pop_back();
        c->slots.push_back({st, slot});
        return slot;
    }
    std::vector<std::pair<int, hipEvent_t>> busy;
    for (auto& b : h->slot_busy) {
        if (hipEventQuery(b.second) == hipSuccess) {
            h->slot_free.push_back(b.first);
            h->slot_ev.push_back(b.second);
        } else {
            busy.push_back(b);
        }
    }
    (void)hipGetLastError();          // hipEventQuery's hipErrorNotReady
    h->slot_busy.swap(busy);
    if (h->slot_free.empty()) return -1;
    const int slot = h->slot_free.back();
    h->slot_free.pop_back();
    return slot;
}
// after an uncaptured launch that used `slot` on `st`
static int split_slot_hold(dpk_handle* h, int slot, hipStream_t st) {
    hipEvent_t ev = nullptr;
    if (!h->slot_ev.empty()) {
        ev = h->slot_ev.back();
        h->slot_ev.pop_back();
    } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        h->slot_free.push_back(slot);    // the launch is enqueued; a later launch reusing the slot is
        HIPCHK(h, hipStreamSynchronize(st));   // safe once this one has finished
        return DPK_OK;
    }
    h->slot_busy.push_back({slot, ev});
    HIPCHK(h, hipEventRecord(ev, st));
    return DPK_OK;
}

// One launch of the sampler kernel with tile size PT (4: dpk, 2: dpk2) for the handle's graph
// pattern and GEMM mode.
template <int MODE, int PT>
static void launch_tiles(dpk_handle* h, int blocks, size_t shmem, hipStream_t st, const SampleArgs& a) {
    const int gm = h->gemm_mode;
    const char* a16 = gm == 2 ? h->arenabf : h->arena16;
    const dim3 grid(blocks), block(NT);
#define DPK_LAUNCH3(NS, SP, NZ)                                                                                   \
    do {                                                                                                        \
        if (gm == 1) hipLaunchKernelGGL((NS::sample_kernel<MODE, SP, 1, NZ>), grid, block, shmem, st, a, h->arena, a16); \
        else if (gm == 2) hipLaunchKernelGGL((NS::sample_kernel<MODE, SP, 2, NZ>), grid, block, shmem, st, a, h->arena, a16); \
        else hipLaunchKernelGGL((NS::sample_kernel<MODE, SP, 0, NZ>), grid, block, shmem, st, a, h->arena, a16);  \
    } while (0)
#define DPK_LAUNCH(NS)                                                                                          \
    do {                                                                                                        \
        if constexpr (MODE == M_SAMPLE) {                                                                       \
            if (a.noise) {      /* the caller's draws (ZM = 1) */                                               \
                if (h->sparse_graph) DPK_LAUNCH3(NS, true, 1);                                                  \
                else DPK_LAUNCH3(NS, false, 1);                                                                 \
                break;                                                                                          \
            }                                                                                                   \
        }                                                                                                       \
        if (h->sparse_graph) DPK_LAUNCH3(NS, true, 0);                                                          \
        else DPK_LAUNCH3(NS, false, 0);                                                                         \
    } while (0)
    if constexpr (PT == 4) DPK_LAUNCH(dpk);
    else DPK_LAUNCH(dpk2);
#undef DPK_LAUNCH
#undef DPK_LAUNCH3
}

// The sampler over a.N poses.  One 4-pose workgroup per CU per round; a partial last round of r
// tiles would cost a whole round.  Plan 2 (sample mode, at least one full round before it,
// r <= n_cu / 2): each of those tiles runs steps [0, K/2) and [K/2, K) on two workgroups, one
// launch of full + 2r blocks ordered [first halves | full tiles | second halves].  The dispatcher
// starts blocks in order as CUs free up, so the first halves run beside the first full round and
// the second halves after the last one: the tail costs half a round, and a second half only ever
// waits for a block numbered below it (no deadlock for any CU count).  E.g. config 5's 2,560
// poses per GPU = 640 tiles: 2.5 round times instead of 3.  Every tile runs the same per-step
// arithmetic, so the outputs are bitwise those of plan 0.
// Plan 1 (and plan 2 where it does not apply): when the last round would leave at least half the
// CUs idle (at most 2 poses per CU remain) those poses run as 2-pose workgroups (dpk2, about 0.6
// of a 4-pose tile's time), one per CU, in a second launch after the full rounds.  Each
// workgroup's result depends only on its own poses.
template <int MODE>
static int launch_sampler(dpk_handle* h, hipStream_t st, SampleArgs a, bool cap) {
    const int N = a.N;
    const int round4 = P * h->n_cu;
    if constexpr (MODE == M_SAMPLE) {
        const int tiles = (N + P - 1) / P, q = tiles / h->n_cu, r = tiles % h->n_cu;
        if (h->tail_plan == 2 && a.K >= 2 && q >= 1 && r > 0 && 2 * r <= h->n_cu) {
            const int slot = split_slot(h, st, cap);
            if (slot >= 0) {
                a.pose_off = 0;
                a.split_n = r;
                a.split_k = a.K / 2;
                a.split_full = q * h->n_cu;
                a.flags = h->flags + (size_t)slot * h->n_cu;
                a.split_stats = reinterpret_cast<int*>(h->flags + (size_t)FLAG_SLOTS * h->n_cu);
                a.split_dbg = h->split_dbg;
                h->token = (h->token + 1) & 0x3fffffffu;
                if (h->token == 0) h->token = 1;
                a.token = h->token;
                launch_tiles<MODE, P>(h, q * h->n_cu + 2 * r, 0, st, a);
                HIPCHK(h, hipGetLastError());
                return cap ? DPK_OK : split_slot_hold(h, slot, st);
            }
        }
    }
    int n4 = N;
    const int rem = N % round4;
    if (h->tail_plan >= 1 && rem != 0 && rem <= 2 * h->n_cu) n4 = N - rem;
    if (n4 > 0) {
        a.pose_off = 0;
        launch_tiles<MODE, P>(h, (n4 + P - 1) / P, 0, st, a);
    }
    if (n4 < N) {
        // pad the 2-pose kernel's LDS past half a CU's so the dispatcher places one per CU
        constexpr int P2 = dpk2::P;
        constexpr size_t half = 160 * 1024 / 2, lds2 = (size_t)dpk2::SM_FLOATS * 4;
        constexpr size_t pad = lds2 > half ? 0 : half - lds2 + 256;
        a.pose_off = n4;
        launch_tiles<MODE, P2>(h, (N - n4 + P2 - 1) / P2, pad, st, a);
    }
    HIPCHK(h, hipGetLastError());
    return DPK_OK;
}

#include "dpk_generic.inc"

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
    // the compiled shape runs the persistent sampler; any other (hid_dim a multiple of n_head,
    // n_pts <= 32, any num_layer) the generic path (dpk_generic.inc); DPK_FORCE_GENERIC=1 sends the
    // compiled shape there too (tests compare the two)
    const char* fg = getenv("DPK_FORCE_GENERIC");
    const bool pose_io = cfg->coords_in == CIN_POSE && cfg->coords_out == COUT_POSE;
    const bool compiled = cfg->hid_dim == D && cfg->num_layers >= 1 && cfg->num_layers <= NL && cfg->n_head == NH &&
                          cfg->n_pts == J && (pose_io || (cfg->coords_in == CIN && cfg->coords_out == COUT)) &&
                          !(fg && atoi(fg) != 0);
    if (cfg->hid_dim < 2 || cfg->n_head < 1 || cfg->hid_dim % cfg->n_head != 0 || cfg->num_layers < 1 ||
        cfg->n_pts < 2 || cfg->n_pts > dpkg::GJ_MAX || cfg->coords_in < 1 || cfg->coords_out < 1)
        return DPK_E_UNSUPPORTED;
    // GCNpose: coords 2 -> 3; GCNdiff: x and eps share a shape (coords in == out)
    int kind;
    if (pose_io) kind = 1;
    else if (cfg->coords_in == cfg->coords_out) kind = 0;
    else return DPK_E_UNSUPPORTED;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || cfg->device < 0 || cfg->device >= ndev) return DPK_E_HIP;
    dpk_handle* h = new dpk_handle();
    h->device = cfg->device;
    h->kind = kind;
    h->num_layers = cfg->num_layers;
    h->n_pts = cfg->n_pts;
    h->mask = cfg->n_pts >= 32 ? ~0u : (1u << cfg->n_pts) - 1u;   // every key attends (all-ones src_mask)
    if (!compiled)
        h->gen = gen_new(cfg->hid_dim, cfg->n_head, cfg->n_pts, cfg->num_layers, cfg->coords_in, cfg->coords_out, kind);
    if (hipSetDevice(h->device) != hipSuccess ||
        hipStreamCreateWithFlags(&h->aux, hipStreamNonBlocking) != hipSuccess ||
        hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess) {
        if (h->aux) (void)hipStreamDestroy(h->aux);
        gen_free(h->gen);
        delete h;
        return DPK_E_HIP;
    }
    h->n_cu = std::max(h->n_cu, 1);
    // DPK_TAIL_SPLIT=0/1/2: the initial tail plan (A/B timing); trace builds stamp per block id
    if (const char* ts = getenv("DPK_TAIL_SPLIT")) h->tail_plan = std::min(std::max(atoi(ts), 0), 2);
    if (DPK_TRACE) h->tail_plan = 0;
    // FLAG_SLOTS x n_cu handoff words + the fallback counter
    const size_t flag_bytes = ((size_t)FLAG_SLOTS * h->n_cu + 4) * 4;
    for (int s = FLAG_SLOTS - 1; s >= 0; --s) h->slot_free.push_back(s);
    if (hipMalloc(&h->flags, flag_bytes) != hipSuccess || hipMemset(h->flags, 0, flag_bytes) != hipSuccess) {
        if (h->flags) (void)hipFree(h->flags);
        (void)hipStreamDestroy(h->aux);
        gen_free(h->gen);
        delete h;
        return DPK_E_HIP;
    }
    h->h_arena.assign(ARENA_FLOATS, 0.f);
    h->h_arena16.assign(ARENA16_BYTES / 2, 0);
    h->h_arenabf.assign(ARENAB_BYTES / 2, 0);
    h->h_temb.assign(TEMB_FLOATS, 0.f);
    *out = h;
    return DPK_OK;
}

void dpk_destroy(dpk_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->arena) (void)hipFree(h->arena);
    if (h->arena16) (void)hipFree(h->arena16);
    if (h->arenabf) (void)hipFree(h->arenabf);
    if (h->temb) (void)hipFree(h->temb);
    if (h->tproj_zero) (void)hipFree(h->tproj_zero);
    if (h->flags) (void)hipFree(h->flags);
    gen_free(h->gen);
    // hipFree waits for the device, so in-flight launches finish before their buffers go
    if (h->sched) sched_free(h->sched);
    for (Sched* s : h->retired) sched_free(s);
    for (auto& b : h->eps_bufs)
        if (b.p) (void)hipFree(b.p);
    if (h->eps_spare.p) (void)hipFree(h->eps_spare.p);
    for (CapRes* c : h->caps) {
        for (auto& e : c->eps) (void)hipFree(e.p);
        for (auto& gb : c->gen) (void)hipFree(gb.p);
        // a graph still alive keeps the CapRes object (its callback touches only that)
        if (c->refs.fetch_sub(1) == 1) delete c;
    }
    for (auto& b : h->slot_busy) (void)hipEventDestroy(b.second);
    for (hipEvent_t e : h->slot_ev) (void)hipEventDestroy(e);
    if (h->aux) (void)hipStreamDestroy(h->aux);
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
    if (h->gen) {
        gen_set_graph(h->gen, adj);
        h->have_graph = true;
        return h->have_weights ? gen_upload(h, h->gen) : DPK_OK;
    }
    float T1[J * J], T2[J * J];
    cheb_terms(adj, T1, T2);
    for (int i = 0; i < J * J; ++i) {
        h->h_arena[OFF_CHEB + i] = T1[i];
        h->h_arena[OFF_CHEB + J * J + i] = T2[i];
    }
    // sparse path iff every nonzero of T1/T2 lies inside the compiled H36M pattern
    bool fits = true;
    for (int i = 0; i < J; ++i)
        for (int j = 0; j < J; ++j) {
            bool in1 = false, in2 = false;
            for (int k = 0; k < SPAT.n1[i]; ++k) in1 = in1 || SPAT.c1[i][k] == j;
            for (int k = 0; k < SPAT.n2[i]; ++k) in2 = in2 || SPAT.c2[i][k] == j;
            if ((!in1 && T1[i * J + j] != 0.f) || (!in2 && T2[i * J + j] != 0.f)) fits = false;
        }
    for (int i = 0; i < J; ++i) {
        for (int k = 0; k < SPAT.n1[i]; ++k) h->h_arena[OFF_CHEBS + SPAT.o1[i] + k] = T1[i * J + SPAT.c1[i][k]];
        for (int k = 0; k < SPAT.n2[i]; ++k)
            h->h_arena[OFF_CHEBS + SPAT.nnz1 + SPAT.o2[i] + k] = T2[i * J + SPAT.c2[i][k]];
    }
    // padded rows of the same values for the output ChebConv (OFF_CHEBT): (value bits, row offset j'*LD2)
    for (int i = 0; i < J; ++i) {
        float* row = &h->h_arena[OFF_CHEBT + (size_t)i * (SPT1 + SPT2) * 2];
        for (int k = 0; k < SPT1 + SPT2; ++k) {
            const bool t1 = k < SPT1;
            const int kk = t1 ? k : k - SPT1;
            const int n = t1 ? SPAT.n1[i] : SPAT.n2[i];
            const int col = kk < n ? (t1 ? SPAT.c1[i][kk] : SPAT.c2[i][kk]) : i;
            row[2 * k] = kk < n ? (t1 ? T1 : T2)[i * J + col] : 0.f;
            const int32_t off = col * LD2;
            memcpy(&row[2 * k + 1], &off, 4);
        }
    }
    h->sparse_graph = fits;
    h->h_adj.assign(adj, adj + J * J);
    h->have_graph = true;
    if (h->have_weights) return upload(h);
    return DPK_OK;
}

int dpk_set_mask(dpk_handle* h, const uint8_t* m) {
    if (!h || !m) return fail(h, DPK_E_INVALID, "dpk_set_mask: null argument");
    unsigned bits = 0;
    for (int j = 0; j < h->n_pts; ++j)
        if (m[j]) bits |= 1u << j;
    h->mask = bits;
    return DPK_OK;
}

int dpk_set_pose_masks(dpk_handle* h, const uint32_t* bits_dev, int n) {
    if (!h) return DPK_E_INVALID;
    if (bits_dev && n <= 0) return fail(h, DPK_E_INVALID, "dpk_set_pose_masks: n must be positive");
    h->pmask = reinterpret_cast<const unsigned*>(bits_dev);
    h->pmask_n = bits_dev ? n : 0;
    return DPK_OK;
}

// per-pose masks cover the launch's N poses (models/GraFormer.py:107-108 broadcasts [N,1,17])
static int check_pose_masks(dpk_handle* h, int N, const char* who) {
    if (h->pmask && N > h->pmask_n)
        return fail(h, DPK_E_INVALID, std::string(who) + ": " + std::to_string(N) + " poses but dpk_set_pose_masks covers " +
                                          std::to_string(h->pmask_n));
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
    if (h->gen) {
        if (!gen_load(h->gen, get)) return fail(h, DPK_E_WEIGHTS, "dpk_load_weights: " + missing);
        h->have_weights = true;
        return gen_upload(h, h->gen);
    }
#define GET(var, key, numel)                                             \
    const float* var = get(key, numel);                                  \
    if (!var) return fail(h, DPK_E_WEIGHTS, "dpk_load_weights: " + missing);

    const bool pose = h->kind == 1;
    const int cin = pose ? CIN_POSE : CIN, cout = pose ? COUT_POSE : COUT;
    float* A = h->h_arena.data();
    float w16max = 0.f;             // largest |64 w| of the split-fp16 GEMM weights
    for (int l = 0; l < h->num_layers; ++l) {
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
        const float* tpw = nullptr;
        const float* tpb = nullptr;
        if (!pose) {     // GCNpose's _ResChebGC has no temb_proj (models/ChebConv.py:154-165)
            GET(tpw_, gc + "temb_proj.weight", D * E);
            GET(tpb_, gc + "temb_proj.bias", D);
            tpw = tpw_;
            tpb = tpb_;
        }
        // nn.Linear weight is (out, in): W_eff[k][n] = weight[n][k]
        auto wqkv = [&](int k, int n) {
            const float* w = n < D ? wq : (n < 2 * D ? wk : wv);
            return w[(n % D) * D + k];
        };
        // QKV GEMM with LN0's affine folded in (the LN phase writes (x - mean) / (std + eps)):
        // W' = diag(a) W, bias c = b W + b_qkv (summed in double)
        pack_blocks(Lw + OFF_QKV, D, D3, KB_D, 18, [&](int k, int n) { return n0a[k] * wqkv(k, n); });
        for (int n = 0; n < D3; ++n) {
            double cs = 0.0;
            for (int k = 0; k < D; ++k) cs += (double)n0b[k] * (double)wqkv(k, n);
            const float bqkv = n < D ? bq[n] : (n < 2 * D ? bk[n - D] : bv[n - 2 * D]);
            Lw[OFF_CQKV + n] = (float)(cs + (double)bqkv);
        }
        pack_blocks(Lw + OFF_O, D, D, KB_D, 6, [&](int k, int n) { return wo[n * D + k]; });
        pack_blocks(Lw + OFF_FC1, D, D2, KB_D, 12, [&](int k, int n) { return f1w[n * D + k]; });
        pack_blocks(Lw + OFF_FC2, D2, D, KB_D2, 6, [&](int k, int n) { return f2w[n * D2 + k]; });
        // ChebConv weight (3,1,in,out): the GEMMs read [x | T1x | T2x] (x from its own buffer,
        // cheb_prep XSKIP), the reference's row order
        pack_blocks(Lw + OFF_C1, D3, D, KB_D3, 6, [&](int k, int n) { return c1w[k * D + n]; });
        pack_blocks(Lw + OFF_C2, D3, D, KB_D3, 6, [&](int k, int n) { return c2w[k * D + n]; });
        // the half-width-operand GEMMs (modes 1, 2) read the fp32 mode's operands: LN0 folded into QKV
        // (bias OFF_CQKV), the Chebyshev GEMMs' [x | T1x | T2x] in the reference's row order
        auto wqkv_f = [&](int k, int n) { return n0a[k] * wqkv(k, n); };
        auto wo_f = [&](int k, int n) { return wo[n * D + k]; };
        auto f1_f = [&](int k, int n) { return f1w[n * D + k]; };
        auto f2_f = [&](int k, int n) { return f2w[n * D2 + k]; };
        auto c1_f = [&](int k, int n) { return c1w[k * D + n]; };
        auto c2_f = [&](int k, int n) { return c2w[k * D + n]; };
        uint16_t* L16 = h->h_arena16.data() + (size_t)l * LAYER16_BYTES / 2;
        w16max = fmaxf(w16max, pack16(L16 + O16_QKV / 2, D, D3, KB32_D, 18, wqkv_f));
        w16max = fmaxf(w16max, pack16(L16 + O16_O / 2, D, D, KB32_D, 6, wo_f));
        w16max = fmaxf(w16max, pack16(L16 + O16_FC1 / 2, D, D2, KB32_D, 12, f1_f));
        w16max = fmaxf(w16max, pack16(L16 + O16_FC2 / 2, D2, D, KB32_D2, 6, f2_f));
        w16max = fmaxf(w16max, pack16(L16 + O16_C1 / 2, D3, D, KB32_D3, 6, c1_f));
        w16max = fmaxf(w16max, pack16(L16 + O16_C2 / 2, D3, D, KB32_D3, 6, c2_f));
        uint16_t* Lb = h->h_arenabf.data() + (size_t)l * LAYER16_BYTES / 4;     // bf16 blocks: half the bytes
        (void)pack16<true>(Lb + O16_QKV / 4, D, D3, KB32_D, 18, wqkv_f);
        (void)pack16<true>(Lb + O16_O / 4, D, D, KB32_D, 6, wo_f);
        (void)pack16<true>(Lb + O16_FC1 / 4, D, D2, KB32_D, 12, f1_f);
        (void)pack16<true>(Lb + O16_FC2 / 4, D2, D, KB32_D2, 6, f2_f);
        (void)pack16<true>(Lb + O16_C1 / 4, D3, D, KB32_D3, 6, c1_f);
        (void)pack16<true>(Lb + O16_C2 / 4, D3, D, KB32_D3, 6, c2_f);
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
        for (int s = 0; s < 5; ++s)
            for (int ln = 0; ln < 64; ++ln) {
                const int i = 4 * s + (ln >> 4);
                Lw[OFF_LGF + s * 64 + ln] = i < J ? Lw[OFF_LG + (ln & 15) * J + i] : 0.f;
                Lw[OFF_LGF + (5 + s) * 64 + ln] = i < J ? Lw[OFF_LG + 16 * J + i] : 0.f;
            }
        // temb_proj: transposed [in=384][out=96]
        if (!pose) {
            float* T = h->h_temb.data();
            for (int o = 0; o < D; ++o) {
                for (int k = 0; k < E; ++k) T[TOFF_WP + (size_t)l * E * D + k * D + o] = tpw[o * E + k];
                T[TOFF_BP + l * D + o] = tpb[o];
            }
        }
    }
    // fp16 hi parts must stay finite: |64 w| below the largest fp16 (65504), with margin
    h->w16_ok = w16max < 65000.f;
    GET(wi, "gconv_input.weight", 3 * cin * D);
    GET(bi, "gconv_input.bias", D);
    GET(wout, "gconv_output.weight", 3 * D * cout);
    GET(bout, "gconv_output.bias", cout);
    // input rows k = order*5 + channel of the 5-channel tile; GCNpose's channels 2-4 are zero
    pack_blocks(A + OFF_WIN, 3 * CIN, D, 1, 6, [&](int k, int n) {
        const int o = k / CIN, c = k % CIN;
        return c < cin ? wi[o * cin * D + c * D + n] : 0.f;
    });
    // output ChebConv as Y = x [W0 | W1 | W2] (96 -> 3*cout columns), out = Y0 + T1 Y1 + T2 Y2 in the kernel
    pack_blocks(A + OFF_WOUT, D, 3 * cout, KB_D, 1,
                [&](int k, int n) { return wout[((n / cout) * D + k) * cout + n % cout]; });
    for (int c = 0; c < D; ++c) A[OFF_BIN + c] = bi[c];
    for (int c = 0; c < 16; ++c) A[OFF_BOUT + c] = c < cout ? bout[c] : 0.f;
    if (!pose) {         // GCNpose carries temb.dense too (gcnpose.py:94-98) but never uses it
        GET(d0w, "temb.dense.0.weight", E * D);
        GET(d0b, "temb.dense.0.bias", E);
        GET(d1w, "temb.dense.1.weight", E * E);
        GET(d1b, "temb.dense.1.bias", E);
        float* T = h->h_temb.data();
        for (int o = 0; o < E; ++o) {
            for (int k = 0; k < D; ++k) T[TOFF_W0 + k * E + o] = d0w[o * D + k];
            for (int k = 0; k < E; ++k) T[TOFF_W1 + k * E + o] = d1w[o * E + k];
            T[TOFF_B0 + o] = d0b[o];
            T[TOFF_B1 + o] = d1b[o];
        }
    }
#undef GET
    h->have_weights = true;
    int rc = upload(h);
    if (rc || !pose) return rc;
    // the pose backbone adds no timestep projection: a zero row per layer (E_CHEB1 adds +0)
    if (!h->tproj_zero) {
        HIPCHK(h, hipMalloc(&h->tproj_zero, (size_t)NL * D * 4));
        HIPCHK(h, hipMemset(h->tproj_zero, 0, (size_t)NL * D * 4));
    }
    return DPK_OK;
}

int dpk_set_schedule(dpk_handle* h, const float* abar, int n_alpha, const int* seq, int K, float eta) {
    if (!h || !abar || !seq || K <= 0 || n_alpha < 2) return fail(h, DPK_E_INVALID, "dpk_set_schedule: bad args");
    if (h->kind != 0) return fail(h, DPK_E_STATE, "GCNpose handle (coords 2->3) has no diffusion schedule");
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
    sched_sweep(h);
    // an identical schedule keeps its device buffers (and every graph captured with them)
    if (h->sched && h->sched->K == K && h->sched->eta == eta && h->sched->h_coef == c) return DPK_OK;
    Sched* s = new Sched();
    static uint64_t sched_serial = 0;
    s->serial = ++sched_serial;
    const size_t tps_off = ((size_t)K * 6 + 3) / 4 * 4;
    hipError_t e = hipMalloc(&s->buf, (tps_off + (size_t)K * NL * D) * 4);
    if (e != hipSuccess) {
        delete s;
        return fail(h, DPK_E_HIP, std::string("dpk_set_schedule: hipMalloc: ") + hipGetErrorString(e) +
                                      " (a schedule cannot be built while a graph is being captured)");
    }
    s->coef = s->buf;
    s->tps = s->buf + tps_off;
    s->K = K;
    s->eta = eta;
    s->h_coef = c;
    // a fresh buffer no launch has seen: the copy cannot race any stream
    e = hipMemcpyAsync(s->coef, c.data(), c.size() * 4, hipMemcpyHostToDevice, h->aux);
    if (e == hipSuccess) e = hipStreamSynchronize(h->aux);
    if (e != hipSuccess) {
        sched_free(s);
        return fail(h, DPK_E_HIP, std::string("dpk_set_schedule: coef upload: ") + hipGetErrorString(e));
    }
    if (h->have_weights && !h->gen) {   // the generic path computes its projections per call
        const int rc = sched_compute_tps(h, s);
        if (rc) {
            sched_free(s);
            return rc;
        }
    }
    if (h->sched) h->retired.push_back(h->sched);
    h->sched = s;
    sched_sweep(h);
    return DPK_OK;
}


static int check_ready(dpk_handle* h, int kind = 0) {
    if (h->kind != kind)
        return fail(h, DPK_E_STATE, kind ? "GCNdiff handle: dpk_pose needs a GCNpose handle (coords 2->3)"
                                         : "GCNpose handle (coords 2->3): use dpk_pose");
    if (!h->have_graph) return fail(h, DPK_E_STATE, "graph (adjacency) not set");
    if (!h->have_weights) return fail(h, DPK_E_STATE, "weights not loaded");
    if (h->gen && h->gemm_mode != 0)
        return fail(h, DPK_E_UNSUPPORTED, "generic-shape path (model shape other than hid 96 / 4 heads / 17 joints): "
                                          "fp32 GEMMs only (gemm mode 0)");
    if (h->gemm_mode == 1 && !h->w16_ok)
        return fail(h, DPK_E_UNSUPPORTED, "gemm mode 1 (3x fp16): a GEMM weight has |w| >= 1015, outside the split-fp16 "
                                          "packing range; use gemm mode 0 (fp32)");
    return DPK_OK;
}

int dpk_eps(dpk_handle* h, const float* x, const float* t, float* eps, int N, void* stream) {
    if (!h) return DPK_E_INVALID;
    if (N < 0 || (N > 0 && (!x || !t || !eps))) return fail(h, DPK_E_INVALID, "dpk_eps: bad args");
    int rc = check_ready(h);
    if (rc) return rc;
    if (N == 0) return DPK_OK;
    if ((rc = check_pose_masks(h, N, "dpk_eps"))) return rc;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    bool cap = false;
    rc = capturing(h, st, &cap);
    if (rc) return rc;
    if (h->gen) return gen_eps(h, x, t, eps, N, st, cap);
    float* proj = nullptr;
    if (cap) {
        // graph nodes keep this buffer: the capture's own for this stream (its captured dpk_eps calls
        // are sequential nodes and share it), taken from the spare that uncaptured calls size
        CapRes* c = nullptr;
        if ((rc = cap_get(h, st, &c))) return rc;
        EpsBuf* mine = nullptr;
        for (auto& e : c->eps)
            if (e.st == st) mine = &e;
        if (!mine) {
            if (h->eps_spare.cap < N)
                return fail(h, DPK_E_STATE, "dpk_eps: a captured call needs a projection buffer of " +
                                                std::to_string(N) + " poses, and the spare holds " +
                                                std::to_string(h->eps_spare.cap) +
                                                "; make an uncaptured dpk_eps call of >= N poses before the capture");
            c->eps.push_back(EpsBuf{st, h->eps_spare.p, h->eps_spare.cap});
            h->eps_spare = EpsBuf{};
            mine = &c->eps.back();
        } else if (mine->cap < N) {
            return fail(h, DPK_E_STATE, "dpk_eps: the captured calls of one stream share the buffer of the capture's "
                                        "first call (" + std::to_string(mine->cap) + " poses); this one has " +
                                        std::to_string(N) + "; warm up with the largest N before capturing");
        }
        proj = mine->p;
    } else {
        cap_sweep(h);
        EpsBuf* buf = nullptr;
        for (auto& b : h->eps_bufs)
            if (b.st == st) buf = &b;
        if (!buf) {
            h->eps_bufs.push_back(EpsBuf{st, nullptr, 0});
            buf = &h->eps_bufs.back();
        }
        if (buf->cap < N) {
            // earlier dpk_eps calls on this stream may still read the old buffer
            HIPCHK(h, hipStreamSynchronize(st));
            if (buf->p) HIPCHK(h, hipFree(buf->p));
            buf->p = nullptr;
            buf->cap = 0;
            const int cap_new = std::max(N, 64);
            HIPCHK(h, hipMalloc(&buf->p, (size_t)cap_new * NL * D * 4));
            buf->cap = cap_new;
        }
        proj = buf->p;
        // keep a spare of at least N poses for a later capture (no launch has seen it: no race)
        if (h->eps_spare.cap < N) {
            if (h->eps_spare.p) HIPCHK(h, hipFree(h->eps_spare.p));
            h->eps_spare = EpsBuf{};
            const int cap_new = std::max(N, 64);
            HIPCHK(h, hipMalloc(&h->eps_spare.p, (size_t)cap_new * NL * D * 4));
            h->eps_spare.cap = cap_new;
        }
    }
    hipLaunchKernelGGL(temb_kernel, dim3(N), dim3(256), 0, st, h->temb, t, 1, proj);
    HIPCHK(h, hipGetLastError());
    SampleArgs a{};
    a.arena = h->arena;
    a.coef = nullptr;     // unused in eps mode
    a.tproj = proj;
    a.x_in = x;
    a.x_out = eps;
    a.N = N;
    a.K = 1;
    a.mask = h->mask;
    a.pmask = h->pmask;
    a.num_layers = h->num_layers;
    const bool prof = h->profiling && !cap;
    std::pair<hipEvent_t, hipEvent_t> ev;
    if (prof && prof_begin(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_eps: event record");
    if ((rc = launch_sampler<M_EPS>(h, st, a, cap))) return rc;
    if (prof && prof_end(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_eps: event record");
    return DPK_OK;
}

int dpk_sample(dpk_handle* h, const float* x, float* out, float* xs, float* x0s, int N, uint64_t seed,
               void* stream) {
    return dpk_sample_noise(h, x, out, xs, x0s, N, seed, nullptr, stream);
}

int dpk_sample_noise(dpk_handle* h, const float* x, float* out, float* xs, float* x0s, int N, uint64_t seed,
                     const float* noise, void* stream) {
    if (!h) return DPK_E_INVALID;
    if (N < 0 || (N > 0 && (!x || !out))) return fail(h, DPK_E_INVALID, "dpk_sample: bad args");
    int rc = check_ready(h);
    if (rc) return rc;
    Sched* sc = h->sched;
    if (!sc) return fail(h, DPK_E_STATE, "schedule not set");
    if (N == 0) return DPK_OK;
    if (!h->gen && sc->tps_gen != h->weights_gen)
        return fail(h, DPK_E_STATE, "dpk_sample: schedule projections are stale");
    if ((rc = check_pose_masks(h, N, "dpk_sample"))) return rc;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    bool cap = false;
    rc = capturing(h, st, &cap);
    if (rc) return rc;
    if (!cap) {
        cap_sweep(h);
        sched_sweep(h);
    }
    if (h->gen) return gen_sample(h, sc, x, out, xs, x0s, N, seed, noise, st, cap);
    if (xs) HIPCHK(h, hipMemcpyAsync(xs, x, (size_t)N * PE * 4, hipMemcpyDeviceToDevice, st));
    SampleArgs a{};
    a.noise = noise;
    a.arena = h->arena;
    a.coef = sc->coef;
    a.tproj = sc->tps;
    a.x_in = x;
    a.x_out = out;
    a.xs = xs;
    a.x0s = x0s;
    a.N = N;
    a.K = sc->K;
    a.mask = h->mask;
    a.pmask = h->pmask;
    a.eta = sc->eta;
    a.seed = seed;
    a.num_layers = h->num_layers;
#if DPK_TRACE
    if (h->trace_step >= 0) {
        const size_t len = (size_t)((N + P - 1) / P) * NW * TRACE_SLOTS;
        if (h->trace_len < len) {
            if (h->trace) HIPCHK(h, hipFree(h->trace));
            HIPCHK(h, hipMalloc(&h->trace, len * 8));
            h->trace_len = len;
        }
        HIPCHK(h, hipMemsetAsync(h->trace, 0, len * 8, st));
    }
    a.trace = h->trace_step >= 0 ? h->trace : nullptr;
    a.trace_step = h->trace_step;
#endif
    const bool prof = h->profiling && !cap;
    std::pair<hipEvent_t, hipEvent_t> ev;
    if (prof && prof_begin(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_sample: event record");
    if ((rc = launch_sampler<M_SAMPLE>(h, st, a, cap))) return rc;
    if (prof && prof_end(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_sample: event record");
    return sched_note_use(h, sc, st, cap);
}

int dpk_pose(dpk_handle* h, const float* x2d, float* xyz, float* uvxyz, int N, int H, int root_mode,
             void* stream) {
    if (!h) return DPK_E_INVALID;
    if (N < 0 || H < 1 || root_mode < 0 || root_mode > 2 || (N > 0 && (!x2d || (!xyz && !uvxyz))))
        return fail(h, DPK_E_INVALID, "dpk_pose: bad args");
    int rc = check_ready(h, 1);
    if (rc) return rc;
    if (N == 0) return DPK_OK;
    if ((rc = check_pose_masks(h, N, "dpk_pose"))) return rc;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    bool cap = false;
    rc = capturing(h, st, &cap);
    if (rc) return rc;
    if (h->gen) return gen_pose(h, x2d, xyz, uvxyz, N, H, root_mode, st, cap);
    SampleArgs a{};
    a.arena = h->arena;
    a.num_layers = h->num_layers;
    a.tproj = h->tproj_zero;   // zeros
    a.x_in = x2d;
    a.x_out = xyz;
    a.uvxyz = uvxyz;
    a.N = N;
    a.K = 1;
    a.H = H;
    a.root_mode = root_mode;
    a.mask = h->mask;
    a.pmask = h->pmask;
    const bool prof = h->profiling && !cap;
    std::pair<hipEvent_t, hipEvent_t> ev;
    if (prof && prof_begin(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_pose: event record");
    if ((rc = launch_sampler<M_POSE>(h, st, a, cap))) return rc;
    if (prof && prof_end(h, st, ev)) return fail(h, DPK_E_HIP, "dpk_pose: event record");
    return DPK_OK;
}

int dpk_set_gemm_mode(dpk_handle* h, int mode) {
    if (!h) return DPK_E_INVALID;
    if (mode < 0 || mode > 2)
        return fail(h, DPK_E_INVALID, "dpk_set_gemm_mode: mode must be 0 (fp32), 1 (3xfp16) or 2 (bf16)");
    h->gemm_mode = mode;
    return DPK_OK;
}

int dpk_set_tail_plan(dpk_handle* h, int plan) {
    if (!h) return DPK_E_INVALID;
    if (plan < 0 || plan > 2) return fail(h, DPK_E_INVALID, "dpk_set_tail_plan: plan must be 0, 1 or 2");
    h->tail_plan = DPK_TRACE ? 0 : plan;
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
    return dpk_ddim_update_noise(h, xt, et, xn, x0, n, step, seed, nullptr, stream);
}

int dpk_ddim_update_noise(dpk_handle* h, const float* xt, const float* et, float* xn, float* x0, int64_t n,
                          int step, uint64_t seed, const float* noise, void* stream) {
    if (!h) return DPK_E_INVALID;
    if (n < 0 || (n > 0 && (!xt || !et || !xn))) return fail(h, DPK_E_INVALID, "dpk_ddim_update: bad args");
    Sched* sc = h->sched;
    if (!sc) return fail(h, DPK_E_STATE, "schedule not set");
    if (step < 0 || step >= sc->K) return fail(h, DPK_E_INVALID, "dpk_ddim_update: step out of range");
    if (n == 0) return DPK_OK;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    bool cap = false;
    int rc = capturing(h, st, &cap);
    if (rc) return rc;
    if (!cap) cap_sweep(h);
    const long long nb = (n + 255) / 256;
    hipLaunchKernelGGL(ddim_kernel, dim3((unsigned)nb), dim3(256), 0, st, xt, et, xn, x0, (long long)n,
                       sc->coef + step * 6, step, sc->eta, (unsigned long long)seed, noise);
    HIPCHK(h, hipGetLastError());
    return sched_note_use(h, sc, st, cap);
}

int dpk_debug_split(dpk_handle* h, int mode, int* fallbacks) {
    if (!h) return DPK_E_INVALID;
    if (mode < 0 || mode > 2) return fail(h, DPK_E_INVALID, "dpk_debug_split: mode must be 0, 1 or 2");
    h->split_dbg = mode;
    if (fallbacks) {
        HIPCHK(h, hipSetDevice(h->device));
        HIPCHK(h, hipDeviceSynchronize());
        int* ctr = reinterpret_cast<int*>(h->flags + (size_t)FLAG_SLOTS * h->n_cu);
        HIPCHK(h, hipMemcpy(fallbacks, ctr, 4, hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemset(ctr, 0, 4));
    }
    return DPK_OK;
}

int dpk_debug_resources(dpk_handle* h, int* out, int n) {
    if (!h || (n > 0 && !out)) return DPK_E_INVALID;
    int released = 0, tracked = 0, retired = (int)h->retired.size();
    for (CapRes* c : h->caps) {
        tracked += c->tracked ? 1 : 0;
        released += (c->tracked && c->released.load()) ? 1 : 0;
    }
    const int v[8] = {(int)h->caps.size(), tracked, released, (int)h->slot_free.size(), retired,
                      h->eps_spare.cap, gen_graph_count(h->gen), gen_spare_kib(h->gen)};
    for (int i = 0; i < n && i < 8; ++i) out[i] = v[i];
    return DPK_OK;
}

#if DPK_TRACE
// trace builds only (not part of the C ABI): choose the traced step; copy the stamps out
int dpk_debug_trace(dpk_handle* h, int step, unsigned long long* out, long long cap) {
    if (!h) return DPK_E_INVALID;
    h->trace_step = step;
    if (!out || !h->trace) return DPK_OK;
    HIPCHK(h, hipDeviceSynchronize());
    HIPCHK(h, hipMemcpy(out, h->trace, std::min((size_t)cap, h->trace_len) * 8, hipMemcpyDeviceToHost));
    return (int)std::min((size_t)cap, h->trace_len);
}
#endif

}  // extern "C"
