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
