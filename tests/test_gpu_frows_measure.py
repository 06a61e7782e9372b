"""GPU: the §8 "next" rows measured beside their CPU restatements (f1 GCNpose, f2 per-frame metrics,
f3 GMM input sampling), each also checked against the oracle on the frames timed.

Prints one ``FROW {json}`` line per row (run with -s or -rP): device time per 1,024-frame batch from HIP
events over 20 back-to-back calls, the CPU restatement's frames/s on a bounded sample with the threads
this process has, and the achieved delta.  These are the path's neighbours (the step before the DDIM
loop, the reduction after it, the input pipeline), not the headline metric.
"""
import json
import time

import numpy as np
import pytest
import torch

from conftest import record_delta

pytestmark = pytest.mark.gpu


def _gpu_ms(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def _report(row, frames, gpu_ms, cpu_frames, cpu_s, delta, what):
    rec = {"row": row, "frames": frames, "gpu_ms_per_batch": round(gpu_ms, 4),
           "gpu_frames_per_s": round(frames / (gpu_ms * 1e-3), 1), "cpu_frames": cpu_frames,
           "cpu_frames_per_s": round(cpu_frames / cpu_s, 1), "cpu_threads": torch.get_num_threads(),
           "max_abs_delta": float(f"{delta:.3e}"), "what": what}
    print("FROW", json.dumps(rec))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def test_f1_gcnpose(dev):
    from diffpose_amd.data import synthetic_batch
    from diffpose_amd.gcndiff import adj_mx_from_edges
    from diffpose_amd.gcnpose import HipGCNpose
    from diffpose_amd.weights import synthetic_state_dict
    from oracle import gcndiff_oracle as O

    sd = synthetic_state_dict(kind="pose")
    m = HipGCNpose(adj_mx_from_edges(), None, device=dev)
    m.load_state_dict(sd)
    x, _ = synthetic_batch(1024, seed=91)
    x2d = torch.from_numpy(np.ascontiguousarray(x[:, :, :2]))
    xd = x2d.to(dev)
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    ms = _gpu_ms(lambda: m.uvxyz(xd, mask, 1, "quirk"))
    xyz = m(xd, mask).cpu()
    P, adj = O.params_to_torch(sd), O.adjacency()
    n = 128
    t0 = time.perf_counter()
    ref = O.gcnpose_forward(P, adj, x2d[:n], torch.ones(1, 1, 17, dtype=torch.bool))
    cpu_s = time.perf_counter() - t0
    d = float((xyz[:n] - ref).abs().max())
    _report("f1 GCNpose + uvxyz assembly (models/gcnpose.py:101-113, runners/diffpose_frame.py:337-342)",
            1024, ms, n, cpu_s, d, "dpk_pose vs the oracle's GCNpose.forward")
    assert record_delta(d, 5e-6)
    m.close()


def test_f2_metrics(dev):
    from diffpose_amd.data import synthetic_batch
    from diffpose_amd.metrics import pose_errors
    from oracle import metrics_oracle as MO

    x, tgt = synthetic_batch(1024, seed=92)
    out = torch.from_numpy(x).to(dev)
    t = torch.from_numpy(tgt).to(dev)
    ms = _gpu_ms(lambda: pose_errors(out, t, 1, "relative"))
    p1, p2 = pose_errors(out, t, 1, "relative")
    pred = x[:, :, 2:].astype(np.float64)
    pred = pred - pred[:, :1]
    t64 = tgt.astype(np.float64) - tgt[:, :1].astype(np.float64)
    n = 1024
    t0 = time.perf_counter()
    r2 = MO.p_mpjpe_per_pose(pred[:n].copy(), t64[:n].copy())
    r1 = np.linalg.norm(pred[:n] - t64[:n], axis=-1).mean(-1)
    cpu_s = time.perf_counter() - t0
    d = max(float(np.abs(p2.cpu().numpy()[:n] - r2).max()), float(np.abs(p1.cpu().numpy()[:n] - r1).max()))
    _report("f2 per-frame MPJPE / P-MPJPE (common/loss.py:7-64, common/utils.py:96-187)", 1024, ms, n, cpu_s, d,
            "dpk_pose_metrics (fp64) vs the oracle's numpy SVD Procrustes in float64 (metres)")
    assert record_delta(d, 1e-9)


def test_f3_gmm_sampling(dev):
    from diffpose_amd.gmm import PoseGeneratorGMM, numpy_atol
    from oracle import gmm_oracle as GO

    rng = np.random.Generator(np.random.PCG64(93))
    n_src, kn = 4096, 5
    w = rng.dirichlet(np.ones(kn), size=(n_src, 17))
    g = np.empty((n_src, 17, kn, 5))
    g[..., 0] = w
    g[..., 1:3] = rng.uniform(-1, 1, size=(n_src, 17, kn, 2))
    g[..., 3:5] = rng.uniform(1e-4, 1e-2, size=(n_src, 17, kn, 2))
    g = g.astype(np.float32)
    p3 = rng.normal(0.0, 0.4, size=(n_src, 17, 3)).astype(np.float32)
    ds = PoseGeneratorGMM([p3], [g], [["Walking 1"] * n_src], [np.zeros((n_src, 9), np.float32)], device=dev)
    idx = rng.integers(0, n_src, size=1024)
    u = rng.random((1024, 17))
    ms = _gpu_ms(lambda: ds.batch(idx, u=u))
    uv = ds.batch(idx, u=u)[0].cpu().numpy()
    rel = p3 - p3[:, :1]
    n = 256
    atol = numpy_atol(np.float32)
    t0 = time.perf_counter()
    ref = np.stack([GO.gmm_item(rel, g, int(i), u[k], atol)[0] for k, i in enumerate(idx[:n])])
    cpu_s = time.perf_counter() - t0
    d = float(np.abs(uv[:n] - ref).max())
    _report("f3 GMM 2D-keypoint sampling (common/generators.py:24-53)", 1024, ms, n, cpu_s, d,
            "dpk_gmm_sample vs the oracle's per-item np.random.choice restatement (bitwise expected)")
    assert d == 0.0
