"""GPU parity: the HIP sampler (through the C ABI) vs the reference's golden vectors and
the golden-pinned CPU oracle.

Tolerances (fp32 everywhere; the HIP path reorders fp32 sums — MFMA k-order, fused
Chebyshev GEMM, double-accumulated LayerNorm statistics — so it is not bitwise).  Round 4 set
them from what the kernel achieves (every check reports its delta through
``conftest.record_delta``; the GPU run's log is kept under profiles/):
  * single denoiser call: |eps - eps_ref| <= 5e-6 (|eps| ~ 1);
  * trajectories: |x - x_ref| <= 5e-6 elementwise;
  * north-star bar: |MPJPE_hip - MPJPE_ref| <= 1e-4 mm at B=1024, K=50.
The reference's own fp32-vs-fp64 gap on these inputs is 1.6e-5 mm / 1.2e-6 per element.
"""
import numpy as np
import pytest
import torch

from conftest import record_delta

from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict
from diffpose_amd.data import synthetic_batch
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd import utils_diff

pytestmark = pytest.mark.gpu

EPS_TOL = 5e-6
TRAJ_TOL = 5e-6
MPJPE_TOL_MM = 1e-4


def _betas(T):
    return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                              num_diffusion_timesteps=T)).float()


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict())
    return m


@pytest.fixture(scope="module")
def mask():
    return torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0")


def _maxdiff(a, b):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if torch.is_tensor(b) else np.asarray(b, np.float64)
    assert a.shape == b.shape
    return float(np.abs(a - b).max())


def _mpjpe_mm(out, targets):
    o = out.detach().cpu().double() if torch.is_tensor(out) else torch.from_numpy(np.asarray(out)).double()
    xyz = o[:, :, 2:]
    xyz = xyz - xyz[:, :1, :]
    t = torch.from_numpy(np.asarray(targets)).double()
    return float(torch.mean(torch.norm(xyz - t, dim=-1)) * 1000.0)


def test_eps_vs_golden(model, mask, golden):
    g = golden("g2_modules.npz")
    x = torch.from_numpy(g["x"]).cuda()
    t = torch.from_numpy(g["t"]).cuda()
    eps = model(x, mask, t, 0)
    assert record_delta(_maxdiff(eps, g["eps"]), EPS_TOL)
    m2 = torch.from_numpy(g["mask2"]).cuda()
    eps2 = model(x, m2, t, 0)
    assert record_delta(_maxdiff(eps2, g["eps_masked"]), EPS_TOL)
    eps3 = model(x, mask, t, 0)                      # mask restored
    assert record_delta(_maxdiff(eps3, g["eps"]), EPS_TOL)


def test_trajectory_vs_golden(model, mask, golden):
    g = golden("g3_traj_n64_k10.npz")
    x = torch.from_numpy(g["x"]).cuda()
    xs, x0s = utils_diff.generalized_steps(x, mask, [int(s) for s in g["seq"]], model, _betas(51).cuda(), eta=0.0)
    assert xs[0] is x and len(xs) == 11 and len(x0s) == 10
    assert record_delta(_maxdiff(torch.stack(xs), g["xs"]), TRAJ_TOL)
    assert record_delta(_maxdiff(torch.stack(x0s), g["x0s"]), TRAJ_TOL)
    assert record_delta(abs(_mpjpe_mm(xs[-1], g["targets"]) - float(g["mpjpe_mm"])), MPJPE_TOL_MM)


@pytest.mark.parametrize("name", ["g4_final_n16_k50.npz", "g4_final_n16_k100_T101.npz", "g4_final_n8_quad.npz"])
def test_final_vs_golden(model, mask, golden, name):
    g = golden(name)
    x = torch.from_numpy(g["x"]).cuda()
    out = model.sample(x, [int(s) for s in g["seq"]], _betas(int(g["T"])), mask=mask)
    assert record_delta(_maxdiff(out, g["out"]), TRAJ_TOL)
    assert record_delta(abs(_mpjpe_mm(out, g["targets"]) - _mpjpe_mm(g["out"], g["targets"])), MPJPE_TOL_MM)


def test_bench_config_vs_oracle(model, mask):
    """B=1024, K=50 (the BASELINE metric's config) against the golden-pinned CPU oracle."""
    from oracle import gcndiff_oracle as O

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    x, tgt = synthetic_batch(1024, seed=19960903)
    seq = make_seq("uniform", 50, 50)
    out = model.sample(torch.from_numpy(x).cuda(), seq, _betas(51), mask=mask)
    P = O.params_to_torch(synthetic_state_dict())
    adj = O.adjacency()
    xs, _ = O.generalized_steps(torch.from_numpy(x), torch.ones(1, 1, 17, dtype=torch.bool), seq,
                                lambda a, m, t: O.gcndiff_forward(P, adj, a, m, t), _betas(51))
    ref = xs[-1]
    assert record_delta(_maxdiff(out, ref), TRAJ_TOL)
    assert record_delta(abs(_mpjpe_mm(out, tgt) - _mpjpe_mm(ref, tgt)), MPJPE_TOL_MM)


def test_generic_callable_path(model, mask):
    """generalized_steps with a non-HIP model callable: host loop + HIP DDIM update."""
    x, _ = synthetic_batch(32, seed=3)
    x = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    ref_xs, ref_x0s = utils_diff.generalized_steps(x, mask, seq, model, _betas(51).cuda())
    gen_xs, gen_x0s = utils_diff.generalized_steps(x, mask, seq, lambda a, m, t, c: model(a, m, t, c), _betas(51).cuda())
    assert _maxdiff(torch.stack(gen_xs), torch.stack(ref_xs)) <= 1e-6
    assert _maxdiff(torch.stack(gen_x0s), torch.stack(ref_x0s)) <= 1e-6
    # the schedule-only DDIM handle is created once per device and reused: a second call (another
    # schedule) allocates no new handle, and the first call's results come back unchanged after it
    h1 = utils_diff.schedule_handle(x.device)
    n_handles = len(utils_diff._sched_cache())
    seq2 = make_seq("uniform", 50, 5)
    utils_diff.generalized_steps(x, mask, seq2, lambda a, m, t, c: model(a, m, t, c), _betas(51).cuda())
    again_xs, _ = utils_diff.generalized_steps(x, mask, seq, lambda a, m, t, c: model(a, m, t, c), _betas(51).cuda())
    assert utils_diff.schedule_handle(x.device) is h1 and len(utils_diff._sched_cache()) == n_handles
    assert h1._h.value == utils_diff.schedule_handle(x.device)._h.value
    assert torch.equal(torch.stack(again_xs), torch.stack(gen_xs))
    # the cache is per thread; another thread gets its own handle, and
    # clear_schedule_handles() closes the calling thread's handles
    import threading
    other = []
    th = threading.Thread(target=lambda: other.append(utils_diff.schedule_handle(x.device)._h.value))
    th.start()
    th.join()
    assert other and other[0] != h1._h.value
    assert utils_diff.clear_schedule_handles() == n_handles and h1._h is None
    assert utils_diff.schedule_handle(x.device) is not h1


@pytest.mark.parametrize("n", [1, 3, 5, 67])
def test_ragged_batches_are_batch_invariant(model, mask, n):
    """Partial workgroups: every pose's result is independent of its batch neighbours (bitwise)."""
    x, _ = synthetic_batch(256, seed=11)
    x = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    full = model.sample(x, seq, _betas(51), mask=mask)
    part = model.sample(x[:n].contiguous(), seq, _betas(51), mask=mask)
    assert torch.equal(part, full[:n])


def test_empty_batch(model, mask):
    x = torch.empty(0, 17, 5, device="cuda:0")
    out = model.sample(x, [0, 12], _betas(51), mask=mask)
    assert out.shape == (0, 17, 5)
    eps = model(x, mask, torch.empty(0, device="cuda:0"), 0)
    assert eps.shape == (0, 17, 5)


def test_large_batch_property(model, mask):
    """H=20 hypotheses x 1024 frames (config 5 shape): identical hypotheses stay identical,
    and each frame equals the B=1024 run bit for bit (size-independent check)."""
    x, _ = synthetic_batch(1024, seed=19960903)
    xt = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 50)
    base = model.sample(xt, seq, _betas(51), mask=mask)
    big = model.sample(xt.repeat(20, 1, 1).contiguous(), seq, _betas(51), mask=mask)
    assert torch.equal(big.view(20, 1024, 17, 5), base.unsqueeze(0).expand(20, -1, -1, -1))


def test_tail_round_plans(model, mask):
    """Config 5's per-GPU share (2,560 poses = 640 4-pose tiles = 2.5 rounds on 256 CUs).
    Plan "step_split" (default): the last 128 tiles run steps [0, 5) and [5, 10) on two CUs,
    x_t handed over through the output buffer; bitwise equal to plan "four" (every tile in
    4-pose tiles), trajectories and eta > 0 noise included.  Plan "two_pose": 2 full rounds + one
    round of 2-pose tiles, each part bitwise what its poses give alone, within rounding of the
    others (the tiles put different joints on the 4-row tail path).  Tail poses vs the oracle."""
    from oracle import gcndiff_oracle as O

    x, _ = synthetic_batch(2560, seed=23)
    xt = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    try:
        out = model.sample(xt, seq, _betas(51), mask=mask)
        model.set_tail_plan("four")
        out4 = model.sample(xt, seq, _betas(51), mask=mask)
        assert torch.equal(out, out4)
        xs4, x0s4 = model.sample(xt, seq, _betas(51), eta=0.5, seed=5, mask=mask, trajectory=True)
        model.set_tail_plan("step_split")
        xs2, x0s2 = model.sample(xt, seq, _betas(51), eta=0.5, seed=5, mask=mask, trajectory=True)
        assert torch.equal(xs2, xs4) and torch.equal(x0s2, x0s4)
        model.set_tail_plan("two_pose")
        out1 = model.sample(xt, seq, _betas(51), mask=mask)
        head = model.sample(xt[:2048].contiguous(), seq, _betas(51), mask=mask)
        tail = model.sample(xt[2048:].contiguous(), seq, _betas(51), mask=mask)
        assert torch.equal(out1[:2048], head) and torch.equal(out1[2048:], tail)
        assert torch.equal(out4[:2048], head)
        assert record_delta(_maxdiff(out1, out), TRAJ_TOL)
    finally:
        model.set_tail_plan("step_split")
    P, adj = O.params_to_torch(synthetic_state_dict()), O.adjacency()
    sel = torch.tensor([2048, 2049, 2050, 2051, 2558, 2559])
    xs, _ = O.generalized_steps(torch.from_numpy(x)[sel], torch.ones(1, 1, 17, dtype=torch.bool), seq,
                                lambda a_, m_, t_: O.gcndiff_forward(P, adj, a_, m_, t_), _betas(51))
    assert record_delta(_maxdiff(out[sel.cuda()], xs[-1]), TRAJ_TOL)


@pytest.mark.parametrize("n,k", [(1101, 25), (1100, 2), (2048 + 4 * 128, 50), (1025, 10), (1536, 10),
                                 (2048 + 4 * 128 + 3, 10)])
def test_step_split_matches_four_pose_plan(model, mask, n, k):
    """Step split at other shapes: a ragged last tile (1,101 poses: 276 tiles, the last holding one
    pose), an odd K (halves of 12 and 13 steps), K=2 (one step per half), config 5's share at K=50,
    a single split tile holding one pose (1,025), half a round (1,536) and a ragged 2.5 rounds.
    Bitwise equal to plan "four"; a repeated call (flags reset by every second half) too."""
    x, _ = synthetic_batch(n, seed=29)
    xt = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, k)
    try:
        model.set_tail_plan("four")
        ref = model.sample(xt, seq, _betas(51), mask=mask)
        model.set_tail_plan("step_split")
        for _ in range(2):
            assert torch.equal(model.sample(xt, seq, _betas(51), mask=mask), ref)
    finally:
        model.set_tail_plan("step_split")


def test_step_split_quad_schedule(model, mask):
    """The step split under the quad skip (duplicate t values, runners/diffpose_frame.py:314-317)
    with eta > 0: bitwise equal to plan "four" (the schedule and the noise keys are per step)."""
    x, _ = synthetic_batch(1536, seed=31)
    xt = torch.from_numpy(x).cuda()
    seq = make_seq("quad", 50, 20)
    try:
        model.set_tail_plan("four")
        ref = model.sample(xt, seq, _betas(51), eta=0.3, seed=11, mask=mask)
        model.set_tail_plan("step_split")
        assert torch.equal(model.sample(xt, seq, _betas(51), eta=0.3, seed=11, mask=mask), ref)
    finally:
        model.set_tail_plan("step_split")


def test_eta_reference_noise_vs_golden(model, mask, golden):
    """eta > 0 pinned to the reference (golden g11: the reference's generalized_steps under
    torch.manual_seed, common/utils_diff.py:65 drawing randn_like once per step).  The HIP sampler
    given those K draws (dpk_sample_noise) follows the reference trajectory within the fp32 bars;
    ``generalized_steps(noise="torch-cpu")`` under the same seed draws the same tensors (bitwise the
    explicit run); the host-loop path (generic callable + dpk_ddim_update_noise) matches too; and
    K=50 at eta=1 stays within the MPJPE bar."""
    g = golden("g11_eta.npz")
    x = torch.from_numpy(g["x"]).cuda()
    seq10 = [int(s) for s in g["seq10"]]
    eta = float(g["eta10"])
    noise = torch.from_numpy(g["noise10"]).cuda()
    xs, x0s = model.sample(x, seq10, _betas(51), eta=eta, mask=mask, trajectory=True, noise=noise)
    assert record_delta(_maxdiff(xs, g["xs10"]), TRAJ_TOL)
    assert record_delta(_maxdiff(x0s, g["x0s10"]), TRAJ_TOL)
    assert record_delta(abs(_mpjpe_mm(xs[-1], g["targets"]) - _mpjpe_mm(g["xs10"][-1], g["targets"])), MPJPE_TOL_MM)
    torch.manual_seed(int(g["seed10"]))
    xs_t, _ = utils_diff.generalized_steps(x, mask, seq10, model, _betas(51), eta=eta, noise="torch-cpu")
    assert torch.equal(xs_t[-1], xs[-1])
    fwd = lambda a_, m_, t_, c_: model(a_, m_, t_, c_)   # noqa: E731  (a plain callable: host loop)
    xs_h, _ = utils_diff.generalized_steps(x, mask, seq10, fwd, _betas(51), eta=eta, noise=noise)
    assert record_delta(_maxdiff(torch.stack(xs_h), g["xs10"]), TRAJ_TOL)
    seq50 = [int(s) for s in g["seq50"]]
    out50 = model.sample(x, seq50, _betas(51), eta=float(g["eta50"]), mask=mask,
                         noise=torch.from_numpy(g["noise50"]).cuda())
    assert record_delta(_maxdiff(out50, g["out50"]), TRAJ_TOL)
    assert record_delta(abs(_mpjpe_mm(out50, g["targets"]) - _mpjpe_mm(g["out50"], g["targets"])), MPJPE_TOL_MM)
    with pytest.raises(ValueError):
        model.sample(x, seq10, _betas(51), eta=eta, mask=mask, noise=noise[:5])
    model.set_schedule(seq10, _betas(51), eta=0.0)


def test_step_split_with_noise_and_fallback(model, mask):
    """Caller noise through the step split (1,100 poses: 19 split tiles after one full round) is
    bitwise plan "four"'s.  The handoff's fallback (dpk_debug_split 1: first halves start ~100 ms
    late and second halves do not wait for an unstarted one) makes every second half run its whole
    tile from x_in: same bits, and the library counts 19 fallbacks; mode 2 (no idle wait, first
    halves on time) may take either path per tile, same bits.  A first half that starts after its
    second half gave up writes nothing (the outputs would differ otherwise)."""
    x, _ = synthetic_batch(1100, seed=37)
    xt = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    noise = torch.randn((10,) + tuple(xt.shape), generator=torch.Generator().manual_seed(4)).cuda()
    try:
        model.set_tail_plan("four")
        ref = model.sample(xt, seq, _betas(51), eta=0.7, mask=mask, noise=noise)
        ref0 = model.sample(xt, seq, _betas(51), mask=mask)
        model.set_tail_plan("step_split")
        assert model.debug_split(0, read=True) >= 0          # clear the counter
        assert torch.equal(model.sample(xt, seq, _betas(51), eta=0.7, mask=mask, noise=noise), ref)
        assert model.debug_split(0, read=True) == 0
        model.debug_split(1)
        assert torch.equal(model.sample(xt, seq, _betas(51), eta=0.7, mask=mask, noise=noise), ref)
        assert torch.equal(model.sample(xt, seq, _betas(51), mask=mask), ref0)
        n_fb = model.debug_split(2, read=True)
        print(f"\nstep split fallback (mode 1): {n_fb} of 2 x 19 second halves recomputed")
        assert n_fb == 2 * 19
        assert torch.equal(model.sample(xt, seq, _betas(51), mask=mask), ref0)
        assert 0 <= model.debug_split(0, read=True) <= 19
        assert torch.equal(model.sample(xt, seq, _betas(51), mask=mask), ref0)   # back to normal: flags clean
        assert model.debug_split(0, read=True) == 0
        # the 2-pose tail round (second launch at pose offset 1,024) reads the same noise rows
        model.set_tail_plan("two_pose")
        out1 = model.sample(xt, seq, _betas(51), eta=0.7, mask=mask, noise=noise)
        assert torch.equal(out1[:1024], ref[:1024])
        assert record_delta(_maxdiff(out1, ref), TRAJ_TOL)
    finally:
        model.debug_split(0)
        model.set_tail_plan("step_split")
        model.set_schedule(seq, _betas(51), eta=0.0)


def test_step_split_slots_recycled_across_streams(model, mask):
    """Flag slots are held per launch, not per stream: 80 short-lived HIP streams (more than the 64
    slots; destroyed after use, so addresses recur) each run a step-split launch; every one runs plan 2 (bitwise plan "four") and all 64
    slots are free again once the launches have completed."""
    x, _ = synthetic_batch(1100, seed=41)
    xt = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 2)
    try:
        model.set_tail_plan("four")
        ref = model.sample(xt, seq, _betas(51), mask=mask)
        model.set_tail_plan("step_split")
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        torch.cuda.synchronize()
        outs = []
        for _ in range(80):                    # raw HIP streams (torch's own come from a pool of 32)
            h = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(h)) == 0
            es = torch.cuda.ExternalStream(h.value)
            o = torch.empty_like(xt)                # allocated on torch's stream, written on es
            torch.cuda.synchronize()
            with torch.cuda.stream(es):
                model.sample(xt, seq, _betas(51), mask=mask, out=o)
            es.synchronize()
            outs.append(o)
            assert hip.hipStreamDestroy(h) == 0     # a later stream may reuse the address
        torch.cuda.synchronize()
        assert all(torch.equal(o, ref) for o in outs)
        model.sample(xt, seq, _betas(51), mask=mask)      # sweeps the completed launches
        torch.cuda.synchronize()
        assert model.debug_resources()["free_slots"] >= 63
    finally:
        model.set_tail_plan("step_split")


def test_eta_noise_statistics(model, mask):
    """eta > 0 with the in-kernel counter-based draws (noise="philox"; not torch.randn_like): check
    determinism per seed and the moments of the recovered noise (parity is statistical)."""
    x, _ = synthetic_batch(4096, seed=1)
    x = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    model.set_schedule(seq, _betas(51), eta=1.0)
    et = torch.zeros_like(x)
    xn, x0 = model.ddim_update(x, et, step=0, seed=123)
    xn2, _ = model.ddim_update(x, et, step=0, seed=123)
    xn3, _ = model.ddim_update(x, et, step=0, seed=124)
    assert torch.equal(xn, xn2) and not torch.equal(xn, xn3)
    from diffpose_amd.schedule import alpha_bar_table, ddim_coeffs
    c = ddim_coeffs(alpha_bar_table(_betas(51).numpy()), seq, eta=1.0)[0]
    z = ((xn.double() - float(c[2]) * x0.double()) / float(c[3])).flatten()
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1.0) < 0.01
    a = model.sample(x[:64].contiguous(), seq, _betas(51), eta=1.0, mask=mask, seed=7)
    b = model.sample(x[:64].contiguous(), seq, _betas(51), eta=1.0, mask=mask, seed=7)
    assert torch.equal(a, b)
    model.set_schedule(seq, _betas(51), eta=0.0)


def test_bad_inputs_raise(model, mask):
    with pytest.raises(TypeError):
        model(torch.zeros(2, 17, 5), mask, torch.zeros(2), 0)                 # host tensor
    with pytest.raises(ValueError):
        model(torch.zeros(2, 16, 5, device="cuda:0"), mask, torch.zeros(2, device="cuda:0"), 0)
    with pytest.raises(Exception):
        model.sample(torch.zeros(2, 17, 5, device="cuda:0"), [0, 60], _betas(51))  # t+1 beyond table


def test_non_h36m_graph_dense_path(mask):
    """An adjacency outside the compiled H36M Chebyshev pattern runs the dense graph path."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from oracle import gcndiff_oracle as O
    from diffpose_amd.gcndiff import H36M_EDGES

    edges = tuple(H36M_EDGES) + ((3, 16), (6, 13))
    adj = adj_mx_from_edges(17, edges)
    sd = synthetic_state_dict()
    m = HipGCNdiff(adj, None, device="cuda:0")
    m.load_state_dict(sd)
    x, _ = synthetic_batch(9, seed=77)
    t = torch.tensor([49., 3., 17., 0., 8., 49., 22., 31., 5.])
    eps = m(torch.from_numpy(x).cuda(), mask, t.cuda(), 0)
    ref = O.gcndiff_forward(O.params_to_torch(sd), O.adjacency(17, edges), torch.from_numpy(x),
                            torch.ones(1, 1, 17, dtype=torch.bool), t)
    assert record_delta(_maxdiff(eps, ref), EPS_TOL)
    seq = make_seq("uniform", 50, 10)
    out = m.sample(torch.from_numpy(x).cuda(), seq, _betas(51), mask=mask)
    xs, _ = O.generalized_steps(torch.from_numpy(x), torch.ones(1, 1, 17, dtype=torch.bool), seq,
                                lambda a_, m_, t_: O.gcndiff_forward(O.params_to_torch(sd), O.adjacency(17, edges),
                                                                     a_, m_, t_), _betas(51))
    assert record_delta(_maxdiff(out, xs[-1]), TRAJ_TOL)


def test_temb_cache_follows_schedule_and_weights(mask):
    """dpk_sample caches the per-step temb projections; a new schedule or new weights must
    invalidate them (results equal those of a fresh handle), and repeat calls are exact."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")

    x, _ = synthetic_batch(12, seed=5)
    xd = torch.from_numpy(x).cuda()
    sd1, sd2 = synthetic_state_dict(), synthetic_state_dict(seed=7)
    seq_a, seq_b = make_seq("uniform", 50, 10), make_seq("uniform", 50, 25)

    def fresh(sd, seq):
        m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
        m.load_state_dict(sd)
        out = m.sample(xd, seq, _betas(51), mask=mask).clone()
        m.close()
        return out

    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(sd1)
    a1 = m.sample(xd, seq_a, _betas(51), mask=mask).clone()
    assert torch.equal(m.sample(xd, seq_a, _betas(51), mask=mask), a1)      # cached projections
    assert torch.equal(m.sample(xd, seq_b, _betas(51), mask=mask), fresh(sd1, seq_b))
    m.load_state_dict(sd2)
    assert torch.equal(m.sample(xd, seq_b, _betas(51), mask=mask), fresh(sd2, seq_b))
    # another stream after the cache was filled on the current one
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        o = m.sample(xd, seq_b, _betas(51), mask=mask)
    torch.cuda.synchronize()
    assert torch.equal(o, fresh(sd2, seq_b))
    m.close()
