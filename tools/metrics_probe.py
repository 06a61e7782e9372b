"""Time dpk_pose_metrics (per-frame MPJPE / P-MPJPE, fp64) on a gpurun box: python tools/metrics_probe.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))
from diffpose_amd.data import synthetic_batch  # noqa: E402
from diffpose_amd.metrics import pose_errors  # noqa: E402

for F, H in ((1024, 1), (8192, 1), (1024, 20)):
    x, tgt = synthetic_batch(F * H, seed=3)
    out = torch.from_numpy(x).cuda()
    t = torch.from_numpy(tgt[:F]).cuda()
    pose_errors(out, t, H, "relative")
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(20):
        pose_errors(out, t, H, "relative")
    ev[1].record()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pose_errors(out, t, H, "relative")
    torch.cuda.synchronize()
    print(f"F={F} H={H}: {ev[0].elapsed_time(ev[1]) / 20:.3f} ms per call (events), one call + sync {1e3 * (time.perf_counter() - t0):.3f} ms")

# after sampler launches (what bench.py's final reduction follows)
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges  # noqa: E402
from diffpose_amd.schedule import get_beta_schedule, make_seq  # noqa: E402
from diffpose_amd.weights import synthetic_state_dict  # noqa: E402

m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
m.load_state_dict(synthetic_state_dict())
b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
x, tgt = synthetic_batch(1024, seed=3)
xt = torch.from_numpy(x).cuda()
t = torch.from_numpy(tgt).cuda()
for rep in range(3):
    out = m.sample(xt, make_seq("uniform", 50, 50), b)
    torch.cuda.synchronize()
    for k in range(3):
        t0 = time.perf_counter()
        pose_errors(out, t, 1, "relative")
        torch.cuda.synchronize()
        print(f"after sampler rep {rep}, metrics call {k}: {1e3 * (time.perf_counter() - t0):.3f} ms")
