"""GPU parity for the rows either side of the sampler and the runner:

* HipGCNpose (dpk_pose) vs the reference GCNpose golden (g6) and the golden-pinned oracle,
  including the fused uvxyz assembly (root handling, cat, repeat(test_times));
* dpk_pose_metrics vs the reference's per-frame P-MPJPE golden (g7) and the oracle;
* runner.Diffpose.test_hyber end to end vs the oracle pipeline.

Tolerances: GCNpose output |xyz - ref| <= 5e-6 (one backbone pass, like eps); per-frame
P-MPJPE within 1e-7 m of the reference's float32-numpy values (its own rounding is ~3e-8 m);
MPJPE within 1e-9 relative of the fp64 oracle; end-to-end p1/p2 within 1e-4 mm.
"""
import numpy as np
import pytest
import torch

from conftest import record_delta

from diffpose_amd import metrics
from diffpose_amd.gcndiff import adj_mx_from_edges
from diffpose_amd.gcnpose import HipGCNpose
from diffpose_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

POSE_TOL = 5e-6


@pytest.fixture(scope="module")
def pose_model():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    m = HipGCNpose(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict(kind="pose"))
    return m


def _mask(bits=None):
    m = torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0")
    return m if bits is None else torch.from_numpy(bits).cuda()


def test_gcnpose_vs_golden(pose_model, golden):
    g = golden("g6_gcnpose.npz")
    x2d = torch.from_numpy(g["x2d"]).cuda()
    xyz = pose_model(x2d, _mask())
    assert record_delta(float((xyz.cpu() - torch.from_numpy(g["xyz"])).abs().max()), POSE_TOL)
    xyz_m = pose_model(x2d, _mask(g["mask2"]))
    assert record_delta(float((xyz_m.cpu() - torch.from_numpy(g["xyz_masked"])).abs().max()), POSE_TOL)
    uvxyz, raw = pose_model.uvxyz(x2d, _mask(), test_times=3, root_mode="quirk", return_xyz=True)
    ref = torch.from_numpy(g["uvxyz_h3"])
    assert torch.equal(uvxyz.cpu()[..., :2], ref[..., :2])                    # uv copied exactly
    assert record_delta(float((uvxyz.cpu() - ref).abs().max()), POSE_TOL)
    assert torch.equal(uvxyz[:12], uvxyz[12:24]) and torch.equal(uvxyz[:12], uvxyz[24:])
    assert torch.all(uvxyz[:, 0, 2:] == 0)
    assert torch.equal(raw, xyz)


@pytest.mark.parametrize("mode", ["relative", "raw"])
def test_gcnpose_root_modes(pose_model, mode):
    from oracle import gcndiff_oracle as O
    from diffpose_amd.data import synthetic_batch

    x, _ = synthetic_batch(9, seed=5)
    x2d = torch.from_numpy(np.ascontiguousarray(x[:, :, :2]))
    P = O.params_to_torch(synthetic_state_dict(kind="pose"))
    xyz_ref = O.gcnpose_forward(P, O.adjacency(), x2d, torch.ones(1, 1, 17, dtype=torch.bool))
    ref = O.build_uvxyz(x2d, xyz_ref, 2, mode)
    out = pose_model.uvxyz(x2d.cuda(), _mask(), test_times=2, root_mode=mode)
    assert record_delta(float((out.cpu() - ref).abs().max()), POSE_TOL)
    if mode == "relative":
        assert torch.all(out[:, 0, 2:] == 0)


@pytest.mark.parametrize("n", [1, 5, 13])
def test_gcnpose_ragged_batch_invariance(pose_model, n):
    from diffpose_amd.data import synthetic_batch

    x, _ = synthetic_batch(32, seed=8)
    x2d = torch.from_numpy(np.ascontiguousarray(x[:, :, :2])).cuda()
    full = pose_model(x2d, _mask())
    assert torch.equal(pose_model(x2d[:n].contiguous(), _mask()), full[:n])
    assert pose_model(x2d[:0], _mask()).shape == (0, 17, 3)


def test_handle_kinds_are_enforced(pose_model):
    from diffpose_amd._lib import DpkError
    from diffpose_amd.gcndiff import HipGCNdiff

    d = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    d.load_state_dict(synthetic_state_dict())
    x2d = torch.zeros(4, 17, 2, device="cuda:0")
    with pytest.raises(DpkError):
        HipGCNpose._launch(d, x2d, None, None, torch.empty(4, 17, 5, device="cuda:0"), 1, "quirk")
    with pytest.raises(DpkError):      # input shaped for the pose handle: the library refuses the kind
        HipGCNdiff.forward(pose_model, torch.zeros(4, 17, 2, device="cuda:0"), None, torch.zeros(4, device="cuda:0"))
    with pytest.raises(ValueError):    # uvxyz-shaped input: refused by the shape check first
        HipGCNdiff.forward(pose_model, torch.zeros(4, 17, 5, device="cuda:0"), None, torch.zeros(4, device="cuda:0"))
    with pytest.raises(ValueError):
        pose_model(torch.zeros(4, 17, 5, device="cuda:0"), None)
    with pytest.raises(ValueError):
        pose_model.uvxyz(x2d, None, root_mode="sideways")
    with pytest.raises(KeyError):
        pose_model.load_state_dict(synthetic_state_dict())          # a GCNdiff state_dict


def test_pose_metrics_vs_golden(golden):
    from oracle import metrics_oracle as M

    g = golden("g7_metrics.npz")
    pred, tgt = g["pred"], g["tgt"]
    out = np.zeros((len(pred), 17, 5), np.float32)
    out[:, :, 2:] = pred
    p1, p2, xyz = metrics.pose_errors(torch.from_numpy(out).cuda(), torch.from_numpy(tgt).cuda(), 1, "raw",
                                      return_xyz=True)
    assert np.array_equal(xyz.cpu().numpy(), pred)
    assert float(np.abs(p2.cpu().numpy() - g["per_pose_p2"]).max()) <= 1e-7
    ref_p1 = np.linalg.norm(pred.astype(np.float64) - tgt.astype(np.float64), axis=-1).mean(-1)
    assert np.allclose(p1.cpu().numpy(), ref_p1, rtol=1e-9, atol=0)
    # and vs the oracle's float64 SVD formulation (tight): the rotation/scale are the same optimum
    ref_p2 = M.p_mpjpe_per_pose(pred.astype(np.float64), tgt.astype(np.float64))
    assert float(np.abs(p2.cpu().numpy() - ref_p2).max()) <= 1e-12


def test_pose_metrics_hypotheses_and_root_quirk():
    from oracle import gcndiff_oracle as O
    from oracle import metrics_oracle as M

    rng = np.random.Generator(np.random.PCG64(99))
    H, F = 3, 70
    out = rng.normal(0, 0.3, size=(H * F, 17, 5)).astype(np.float32)
    tgt = rng.normal(0, 0.3, size=(F, 17, 3)).astype(np.float32)
    for mode in ("quirk", "relative"):
        p1, p2, xyz = metrics.pose_errors(torch.from_numpy(out).cuda(), torch.from_numpy(tgt).cuda(), H, mode,
                                          return_xyz=True)
        o = torch.mean(torch.from_numpy(out).reshape(H, -1, 17, 5), 0)[:, :, 2:]
        t = torch.from_numpy(tgt)
        if mode == "quirk":
            o, t = O.root_subtract_inplace_quirk(o), O.root_subtract_inplace_quirk(t)
        else:
            o, t = o - o[:, :1].clone(), t - t[:, :1].clone()
        assert float((xyz.cpu() - o).abs().max()) <= 1e-7
        r1 = np.linalg.norm(o.double().numpy() - t.double().numpy(), axis=-1).mean(-1)
        r2 = M.p_mpjpe_per_pose(o.double().numpy(), t.double().numpy())
        assert np.allclose(p1.cpu().numpy(), r1, rtol=1e-6, atol=1e-9)
        assert np.allclose(p2.cpu().numpy(), r2, rtol=1e-6, atol=1e-9)
    e = metrics.pose_errors(torch.zeros(0, 17, 5, device="cuda:0"), torch.zeros(0, 17, 3, device="cuda:0"))
    assert e[0].shape == (0,)


def test_runner_test_hyber_vs_oracle():
    """Diffpose.test_hyber (GCNpose -> uvxyz -> K=10 DDIM -> metrics -> per-action accounting)
    against the same pipeline built from the oracle, on two synthetic batches."""
    from oracle import gcndiff_oracle as O
    from oracle import metrics_oracle as M
    from diffpose_amd import runner
    from diffpose_amd.data import synthetic_eval_batches
    from diffpose_amd.schedule import get_beta_schedule, make_seq

    cfg = runner.default_config(test_times=2, test_timesteps=10, test_num_diffusion_timesteps=50, batch_size=40)
    args = runner.default_args()
    dp = runner.Diffpose(args, cfg, device="cuda:0")
    dp.create_diffusion_model()
    dp.create_pose_model()
    batches = list(synthetic_eval_batches(80, 40, seed=4242))
    p1, p2 = dp.test_hyber(batches=batches, is_train=1)

    Pd, Pp = O.params_to_torch(synthetic_state_dict()), O.params_to_torch(synthetic_state_dict(kind="pose"))
    adj = O.adjacency()
    mask = torch.ones(1, 1, 17, dtype=torch.bool)
    seq = make_seq("uniform", 50, 10)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
    err = metrics.define_error_list(metrics.TEST_ACTIONS)
    for x2d, tgt, acts in batches:
        x2d = torch.from_numpy(x2d)
        xyz = O.gcnpose_forward(Pp, adj, x2d, mask)
        x = O.build_uvxyz(x2d, xyz, 2, "quirk")
        out = O.generalized_steps(x, mask, seq, lambda a, m, t: O.gcndiff_forward(Pd, adj, a, m, t), b)[0][-1]
        o = O.root_subtract_inplace_quirk(torch.mean(out.reshape(2, -1, 17, 5), 0)[:, :, 2:])
        t = O.root_subtract_inplace_quirk(torch.from_numpy(tgt))
        r1 = M.mpjpe_per_pose(o, t).double().numpy()
        r2 = M.p_mpjpe_per_pose(o.numpy().copy(), t.numpy().copy()).astype(np.float64)
        metrics.test_calculation(r1, r2, acts, err)
    q1, q2 = metrics.print_error(None, err, 1)
    assert abs(p1 - q1) <= 1e-4 and abs(p2 - q2) <= 1e-4, (p1, q1, p2, q2)


def test_runner_track_metrics_writes_performance_file(tmp_path):
    """args.track_metrics: per-batch times and peak-memory deltas are collected and written to
    <log_path>/performance_metrics.txt in the reference's format (runners/diffpose_frame.py:407-461).
    The timed window is the sampler call alone, as the reference's (:345-370: start after the pose
    model, stop after generalized_steps and a device sync): a pose model and a metrics step made
    0.25 s slower show up in pose_times / metrics_times and not in inference_times."""
    import time

    from diffpose_amd import metrics, runner
    from diffpose_amd.data import synthetic_eval_batches

    cfg = runner.default_config(test_times=1, test_timesteps=5, test_num_diffusion_timesteps=50, batch_size=16)
    args = runner.default_args(track_metrics=True, log_path=str(tmp_path))
    dp = runner.Diffpose(args, cfg, device="cuda:0")
    dp.create_diffusion_model()
    dp.create_pose_model()
    batches = list(synthetic_eval_batches(48, 16, seed=5))
    p_fast = dp.test_hyber(batches=batches, is_train=1)
    assert len(dp.inference_times) == 3 and len(dp.memory_usage) == 3
    txt = (tmp_path / "performance_metrics.txt").read_text()
    assert txt.startswith("=== Performance Metrics ===\nTime (s): avg=")
    assert "Diffusion steps: 5\n" in txt and "Memory (MB): avg=" in txt and "=== Raw Data ===" in txt
    assert "Pose model times: [" in txt and "Metrics times: [" in txt

    slow_pose, slow_err = dp.model_pose.uvxyz, metrics.pose_errors

    def pose_delayed(*a, **k):
        time.sleep(0.25)
        return slow_pose(*a, **k)

    def errors_delayed(*a, **k):
        time.sleep(0.25)
        return slow_err(*a, **k)

    dp.model_pose.uvxyz = pose_delayed
    metrics.pose_errors = errors_delayed
    try:
        p_slow = dp.test_hyber(batches=batches, is_train=1)
    finally:
        metrics.pose_errors = slow_err
        del dp.model_pose.uvxyz
    assert p_slow == p_fast
    assert min(dp.pose_times) >= 0.25 and min(dp.metrics_times) >= 0.25
    assert max(dp.inference_times) < 0.2, dp.inference_times
