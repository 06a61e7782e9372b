/*
 * diffpose_kernels.h — C ABI of the MI355X-native DiffPose DDIM sampler (libdpk.so).
 *
 * Drop-in boundary for the reference hot path (reference at nwicakson/diffpose-nw):
 *   - the denoiser callable  GCNdiff.forward(x, mask, t, cemd) -> eps      models/gcndiff.py:101-113
 *     (called once per step at common/utils_diff.py:58)
 *   - the DDIM reverse loop  generalized_steps(x, src_mask, seq, model, b, eta)
 *                                                                           common/utils_diff.py:46-68
 *   - its caller             Diffpose.test_hyber                           runners/diffpose_frame.py:345-370
 * The reference has no FFI of its own (pure PyTorch); these entry points are what a
 * ctypes binding of that seam needs.  INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - All tensor pointers are caller-owned DEVICE memory (fp32, row-major, contiguous)
 *     on the device the handle was created for; work is enqueued on `stream`
 *     (a hipStream_t, NULL = default stream) and is asynchronous.
 *   - Poses are (N, 17, 5) uvxyz: N poses x 17 joints x 5 channels.
 *   - Return value 0 = OK, negative = error (DPK_E_*); dpk_last_error() has the text.
 *   - A handle is bound to one device and is not thread-safe: one handle per rank/thread.
 *   - Stream order: launches (dpk_sample / dpk_eps / dpk_pose / dpk_ddim_update) may be in
 *     flight on several streams at once.  dpk_set_schedule never rewrites a schedule a launch
 *     may still read: it builds a new one, and the old one is freed only after every stream
 *     that used it has passed its last launch.  Uncaptured dpk_eps calls keep their per-pose
 *     timestep projections in a buffer per caller stream.  dpk_load_weights / dpk_set_graph
 *     wait for the device to drain before overwriting the weights (configuration calls).
 *   - Graph capture (hipStreamBeginCapture / torch.cuda.graph): dpk_sample, dpk_eps, dpk_pose
 *     and dpk_ddim_update may be captured.  A captured launch reads the schedule current at
 *     capture time for the graph's whole life (a later dpk_set_schedule builds a new one and
 *     leaves the captured one in place); weights reloaded later are seen by replays.  It also
 *     keeps the key mask it was captured with: the dpk_set_mask bits by value, and the
 *     dpk_set_pose_masks array by address (that array must stay allocated and unchanged while
 *     the graph may replay).  Nothing is allocated inside a captured call.  What the launches of
 *     one capture read by address (their schedules, one dpk_eps projection buffer and one
 *     step-split flag slot per capturing stream, shared by that stream's captured calls) belongs
 *     to the capture: a user object retained by the captured graph releases it when the graph and
 *     its executable instances are destroyed, and the handle's next uncaptured call recycles it
 *     (after one device-wide wait).  The first captured dpk_eps of a capture takes the handle's
 *     spare projection buffer, which every uncaptured dpk_eps of at least N poses sizes: make one
 *     with the capture's largest N before it (else DPK_E_STATE).  Replays of one executable graph
 *     must not overlap each other (HIP orders launches of the same graph exec), and neither may
 *     two executable instances of one captured graph (they share its projection buffer and flag
 *     slot): capture again for a second concurrent instance.
 */
#ifndef DIFFPOSE_KERNELS_H
#define DIFFPOSE_KERNELS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPK_OK              0
#define DPK_E_INVALID      -1   /* bad argument (null pointer, N<0, size mismatch)       */
#define DPK_E_UNSUPPORTED  -2   /* model dims / mode neither path supports               */
#define DPK_E_HIP          -3   /* HIP runtime error                                     */
#define DPK_E_STATE        -4   /* weights / graph / schedule not set yet                */
#define DPK_E_WEIGHTS      -5   /* unknown, missing or mis-sized state_dict entry        */

typedef struct dpk_handle dpk_handle;

/* Model hyper-parameters (configs/human36m_diffpose_uvxyz_*.yml model: section,
 * emd_dim = 4*hid_dim per models/gcndiff.py:68).  The persistent sampler is compiled for
 * hid_dim 96, n_head 4, n_pts 17 and coords_dim [5,5] (GCNdiff, the denoiser) or [2,3]
 * (GCNpose, the 2D->3D front-end; runners/diffpose_frame.py:138), with num_layers (the
 * config's num_layer, models/gcndiff.py:63-90) a run-time value in 1..5 (the reference's
 * configs all use 5); other shapes run the generic-shape path (dpk_create). */
typedef struct {
    int hid_dim;
    int num_layers;
    int n_head;
    int n_pts;
    int coords_in;
    int coords_out;
    int device;        /* HIP device ordinal */
} dpk_config;

/* Library version (major*10000 + minor*100 + patch). */
int dpk_version(void);

/* Create a handle on cfg->device.  Replaces GCNdiff(adj, config) construction
 * (models/gcndiff.py:55-99; runners/diffpose_frame.py:118-127).  The shape every reference config
 * uses (hid_dim 96, n_head 4, n_pts 17, num_layer 1..5, coords [5,5] or GCNpose's [2,3]) runs the
 * persistent sampler; any other shape with hid_dim a multiple of n_head, n_pts <= 32 and coords
 * in == out (or [2,3]) runs the generic-shape path: the same model as per-op HIP kernels, or, for GCNdiff
 * at hid_dim 128 / n_head 8 or 4 and hid_dim 64 / n_head 2 or 4 on 17 joints (num_layer <= 5, coords [5,5]), the
 * persistent sampler compiled at that width (round 5); fp32 GEMMs only (dpk_set_gemm_mode 1/2 then fail
 * with DPK_E_UNSUPPORTED), per-stream scratch grown on demand; under a caller's stream capture the
 * launches are recorded into the caller's graph from a capture-owned scratch (round 5; the first capture
 * of a size needs one uncaptured call of at least that size, else DPK_E_STATE).  Other shapes:
 * DPK_E_UNSUPPORTED. */
int dpk_create(const dpk_config* cfg, dpk_handle** out);

/* Dense n_pts x n_pts adjacency as passed to GCNdiff(adj, ...) (row-normalised,
 * models/GraFormer.py:32-44).  Derives the Chebyshev terms T0..T2 of its
 * normalised Laplacian once (models/ChebConv.py:90-130), instead of per call. */
int dpk_set_graph(dpk_handle* h, const float* adj_host);

/* Load a GCNdiff state_dict (keys as in models/gcndiff.py, with or without the
 * DataParallel "module." prefix; runners/diffpose_frame.py:130-132).  Copies the n
 * host arrays, repacks GEMM weights into MFMA fragment order and precomputes each
 * layer's GraphNet Laplacian (models/GraFormer.py:174-178).  All keys required. */
int dpk_load_weights(dpk_handle* h, const char* const* names, const float* const* host_ptrs,
                     const int64_t* numels, int n);

/* Attention key mask, n_pts bytes (nonzero = attend).  Default all ones, the
 * reference's src_mask (runners/diffpose_frame.py:39-40); zero entries take the
 * masked_fill(-1e9) path of models/GraFormer.py:107-108. */
int dpk_set_mask(dpk_handle* h, const uint8_t* mask_host);

/* Per-pose key masks: the reference's masked_fill broadcasts a [N,1,n_pts] mask
 * over heads and queries (models/GraFormer.py:107-108, mask.unsqueeze(1)).
 * bits_dev: n uint32 words in device memory, bit j of word i = key j of pose i
 * attends.  Owned by the caller and read by every later dpk_eps / dpk_sample /
 * dpk_pose launch (pose i of the launch uses word i; a launch of more than n
 * poses fails with DPK_E_INVALID) until replaced; NULL returns to the
 * dpk_set_mask mask for all poses.  The launches read the array asynchronously, on
 * their streams: free or rewrite it only after they have completed (and never while
 * a graph captured with it may replay). */
int dpk_set_pose_masks(dpk_handle* h, const uint32_t* bits_dev, int n);

/* DDIM schedule.  alpha_bar: fp32 table (1-cat([0],betas)).cumprod(0), n_alpha = T+1
 * entries (compute_alpha, common/utils_diff.py:40-43); seq: K timesteps in
 * ascending order as built by test_hyber (runners/diffpose_frame.py:310-317);
 * eta as in common/utils_diff.py:61-63.  Step scalars are evaluated in fp32 in
 * the reference's operation order.  Host-synchronous: builds a new device schedule
 * (step scalars + per-step timestep projections, on a handle-internal stream) unless
 * the schedule is unchanged; see "Stream order" above.  Not callable while a graph is
 * being captured. */
int dpk_set_schedule(dpk_handle* h, const float* alpha_bar, int n_alpha, const int* seq, int K, float eta);

/* One denoiser evaluation eps = GCNdiff(x, mask, t) for N poses with a
 * per-pose timestep t_dev[N] (float, as model(xt, mask, t.float(), 0)). */
int dpk_eps(dpk_handle* h, const float* x_dev, const float* t_dev, float* eps_dev, int N, void* stream);

/* The whole K-step reverse loop of generalized_steps for N poses in ONE
 * persistent kernel (the per-step timestep projections come with the schedule).
 *   x_dev   [N,17,5] input x (= xs[0])
 *   out_dev [N,17,5] final sample xs[-1]
 *   xs_dev  [K+1,N,17,5] or NULL: full trajectory xs (xs[0] copied from x_dev)
 *   x0s_dev [K,N,17,5]   or NULL: x0_preds
 *   seed: noise stream for eta > 0 (counter-based, not torch.randn_like). */
int dpk_sample(dpk_handle* h, const float* x_dev, float* out_dev, float* xs_dev, float* x0s_dev,
               int N, uint64_t seed, void* stream);

/* dpk_sample with the caller's noise for eta > 0: noise_dev [K,N,17,5] fp32 device, slice k the
 * draw z of the k-th executed step (t = seq[K-1-k]) in x' = sqrt(an)*x0 + c1*z + c2*et — what the
 * reference draws as torch.randn_like(x) once per step (common/utils_diff.py:65), so a caller that
 * draws the same K tensors reproduces the reference's eta > 0 trajectory.  NULL = counter-based
 * noise from `seed` (dpk_sample).  Read asynchronously on `stream`. */
int dpk_sample_noise(dpk_handle* h, const float* x_dev, float* out_dev, float* xs_dev, float* x0s_dev,
                     int N, uint64_t seed, const float* noise_dev, void* stream);

/* One DDIM update for an externally computed eps (generic model callables):
 * the per-element body of common/utils_diff.py:59-65 for schedule step `step`
 * (0 = first executed step, t = seq[K-1]).  x0_out may be NULL. */
int dpk_ddim_update(dpk_handle* h, const float* xt_dev, const float* eps_dev, float* xnext_dev,
                    float* x0_dev, int64_t n_elems, int step, uint64_t seed, void* stream);

/* dpk_ddim_update with this step's draw z (noise_dev [n_elems] fp32 device; NULL = counter-based). */
int dpk_ddim_update_noise(dpk_handle* h, const float* xt_dev, const float* eps_dev, float* xnext_dev,
                          float* x0_dev, int64_t n_elems, int step, uint64_t seed, const float* noise_dev,
                          void* stream);

/* GCNpose front-end (models/gcnpose.py:55-113) for a handle created with coords_in 2,
 * coords_out 3 (create_pose_model, runners/diffpose_frame.py:134-154), fused with the
 * sampler-input assembly of test_hyber (runners/diffpose_frame.py:337-342):
 *   x2d_dev   [N,17,2]  input_2d
 *   xyz_dev   [N,17,3]  model_pose(input_2d) as returned by the model, or NULL
 *   uvxyz_dev [H,N,17,5] cat(input_2d, root-processed xyz).repeat(H,1,1), or NULL
 *   root_mode 0: what the reference's in-place `xyz[:, :, :] -= xyz[:, :1, :]` yields on CPU
 *                torch (aliasing: only the root row is zeroed; pinned by golden g5)
 *             1: true root-relative (xyz - xyz[:, :1]);  2: no root subtraction
 * The key mask of dpk_set_mask applies (GCNpose.forward(x, mask)).  At least one of
 * xyz_dev / uvxyz_dev must be non-NULL. */
int dpk_pose(dpk_handle* h, const float* x2d_dev, float* xyz_dev, float* uvxyz_dev, int N, int H,
             int root_mode, void* stream);

/* Per-frame evaluation of the sampler output (test_hyber, runners/diffpose_frame.py:382-387),
 * handle-free, one thread per frame, fp64:
 *   out_uvxyz_dev [H,F,17,5] sampler output (hypothesis-major, as generalized_steps returns it)
 *   targets_dev   [F,17,3]   targets_3d
 *   root_mode     as in dpk_pose, applied to prediction and target
 *   p1_dev [F] (double)      MPJPE of each frame (metres; common/utils.py:103-127 per frame)
 *   p2_dev [F] (double)      P-MPJPE of each frame, after the best similarity transform
 *                            (common/loss.py:25-64 / common/utils.py:155-187)
 *   xyz_dev [F,17,3] or NULL the hypothesis-mean, root-processed xyz (output_xyz)
 * Returns DPK_OK, DPK_E_INVALID or DPK_E_HIP (no handle, so no dpk_last_error text). */
int dpk_pose_metrics(const float* out_uvxyz_dev, const float* targets_dev, int F, int H, int root_mode,
                     double* p1_dev, double* p2_dev, float* xyz_dev, void* stream);

/* GMM 2D-keypoint sampling of the input pipeline: replaces
 * PoseGenerator_gmm.__getitem__ (common/generators.py:24-53) for a whole batch.
 *   gmm_dev      [n_src,17,kernel_n,5] fp32  per joint: [w, mu_u, mu_v, var_u, var_v] x kernel_n
 *   poses3d_dev  [n_src,17,3] fp32           3D poses (made root-relative here, generators.py:19)
 *   index_dev    [F] int64 or NULL           source frame of each output (taken modulo n_src, as
 *                                            generators.py:26-29); NULL = 0..F-1
 *   u_dev        [F,17] fp64 or NULL         the uniform draw np.random.choice consumes for each
 *                                            joint (RandomState.random_sample, in frame-then-joint
 *                                            order); NULL = counter-based uniforms from `seed`
 *   atol                                     numpy's tolerance on sum(w) = 1 (sqrt(eps) of the
 *                                            weights' dtype: 3.4526698e-4 for float32)
 *   uvxyz_dev, noise_scale_dev  [F,17,5] fp32 outputs (uvxyz = [mu_u, mu_v, xyz - xyz_root],
 *                                            noise_scale = [var_u, var_v, 1, 1, 1])
 *   status_dev   one int (device)            0, or an OR of 1 (a negative weight) and 2 (weights
 *                                            not summing to 1 within atol): numpy's ValueErrors
 * Component selection is numpy's RandomState.choice(kernel_n, 1, p) bit for bit given u.
 * Returns DPK_OK, DPK_E_INVALID (kernel_n outside 1..64, bad pointers) or DPK_E_HIP. */
int dpk_gmm_sample(const float* gmm_dev, const float* poses3d_dev, int n_src, int kernel_n,
                   const int64_t* index_dev, int F, const double* u_dev, uint64_t seed, double atol,
                   float* uvxyz_dev, float* noise_scale_dev, int* status_dev, void* stream);

/* The same for float64 arrays (numpy data kept in double): weights and poses are read as
 * double, the root-relative subtraction runs in double and the outputs are rounded to float32 —
 * the reference's order (generators.py:19 on the float64 array, .float() at :46-50). */
int dpk_gmm_sample_f64(const double* gmm_dev, const double* poses3d_dev, int n_src, int kernel_n,
                       const int64_t* index_dev, int F, const double* u_dev, uint64_t seed, double atol,
                       float* uvxyz_dev, float* noise_scale_dev, int* status_dev, void* stream);

/* GEMM arithmetic of the sampler's transformer/ResChebGC GEMMs (not part of the reference
 * interface; the reference computes everything in fp32 on its device):
 *   mode 0 (default): fp32 MFMA (v_mfma_f32_16x16x4_f32), fp32 accumulate;
 *   mode 1: 3-term fp16 split (a = a_hi + a_lo, w*64 = w_hi + w_lo; a_hi w_hi + a_hi w_lo +
 *           a_lo w_hi on v_mfma_f32_16x16x32_f16, fp32 accumulate), ~fp32-accurate products;
 *   mode 2: bf16 (a and w rounded to bf16, one v_mfma_f32_16x16x32_bf16 product, fp32
 *           accumulate; since round 5 also attention's score and P.V products, and the GraphNet
 *           products from bf16 activations against L_g as a bf16 hi + lo pair): a reduced-precision
 *           mode for the tolerance study of BASELINE config 3.
 * The input/output ChebConvs, LayerNorm, the softmax and the DDIM update stay fp32 in all modes, and
 * so do attention and the GraphNet products in modes 0 and 1.
 * Applies to later dpk_sample / dpk_eps / dpk_pose calls on this handle.  Range: mode 1 needs
 * every GEMM weight |w| < 1015 (else those calls return DPK_E_UNSUPPORTED) and GEMM inputs
 * (LayerNorm/attention/graph/Chebyshev outputs) below 65504 in magnitude; an overflow there
 * shows as non-finite outputs. */
int dpk_set_gemm_mode(dpk_handle* h, int mode);

/* How dpk_sample balances a partial last round of tiles (4 poses per workgroup, one workgroup
 * per CU per round; not part of the reference interface, which has no tiles):
 *   plan 0: the last round in 4-pose tiles like the others;
 *   plan 1: when it holds at most 2 poses per CU, one round of 2-pose tiles (about 0.6 of a
 *           round);
 *   plan 2 (default): when at least one full round precedes it and it holds at most half a
 *           round of tiles, each of its tiles runs its K steps as two halves on two CUs (the
 *           first half's x_t handed over through `out` and a device flag), so the last round
 *           costs about half a round; otherwise plan 1.
 * Plans 0 and 2 give bitwise the same outputs (the same tiles, the same per-step arithmetic);
 * plan 1 agrees within fp32 rounding (other rows on the 4-row tail path).  The plan-2 handoff
 * assumes no dispatch order: a second half whose first half has not started after a few ms runs
 * the whole tile itself (correct output, only slower; dpk_debug_split counts these), and a first
 * half that then starts leaves without writing.  Plan 2 needs one of 64 flag slots per handle: an
 * uncaptured call holds one until its launch has completed, a capture one per capturing stream
 * for the graph's life; a call that finds none free runs plan 1.  dpk_eps and dpk_pose (one step)
 * use plan 1 for plan 2.  The environment variable DPK_TAIL_SPLIT sets a new handle's plan. */
int dpk_set_tail_plan(dpk_handle* h, int plan);

/* Launch timing of the sampler kernel itself: with enable != 0, every dpk_sample /
 * dpk_eps brackets its sampler-kernel launch with a pair of HIP events on the
 * caller's stream.  dpk_profile_read waits for the recorded events and returns up to
 * `cap` elapsed times in ms (oldest first), then clears them. */
int dpk_profile(dpk_handle* h, int enable);
int dpk_profile_read(dpk_handle* h, float* ms_out, int cap, int* count);

/* Test hooks (not part of the reference interface).
 * dpk_debug_split: mode 0 normal; 1: step-split first halves start ~100 ms late and second halves
 * do not wait for an unstarted first half, so every split tile takes the recompute path; 2: second
 * halves do not wait for an unstarted first half.  With `fallbacks` non-NULL, waits for the device
 * and returns (then clears) the number of second halves that ran their tile's first-half steps.
 * dpk_debug_resources: out[0..7] = captures holding resources, captures whose graph holds our
 * user object, captures released (graph gone, not yet recycled), free flag slots, retired
 * schedules, spare dpk_eps capacity (poses); generic-shape handles also: K-step loops recorded as
 * hipGraphs (out[6]) and the spare capture scratch in KiB (out[7]). */
int dpk_debug_split(dpk_handle* h, int mode, int* fallbacks);
int dpk_debug_resources(dpk_handle* h, int* out, int n);

/* Poses per workgroup of the sampler kernel and its static LDS bytes (for docs/bench). */
int dpk_kernel_geometry(int* poses_per_workgroup, int* threads_per_workgroup, int* lds_bytes);

const char* dpk_last_error(const dpk_handle* h);
void dpk_destroy(dpk_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* DIFFPOSE_KERNELS_H */
