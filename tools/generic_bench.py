"""Throughput of the generic-shape path (csrc/dpk_generic.inc) beside the persistent sampler, for
DESIGN.md (run on a gpurun box): B=1024, K=50, whole-call time between syncs, median of 5.
  python tools/generic_bench.py
"""
import os
import sys
import time
from types import SimpleNamespace as ns

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))
from diffpose_amd.data import synthetic_batch  # noqa: E402
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges  # noqa: E402
from diffpose_amd.schedule import get_beta_schedule, make_seq  # noqa: E402
from diffpose_amd.weights import synthetic_state_dict  # noqa: E402


def run(label, hid, heads, layers, force=False, n=1024, k=50, per_op=False):
    cfg = ns(model=ns(hid_dim=hid, emd_dim=hid, coords_dim=[5, 5], num_layer=layers, n_head=heads, dropout=0.0,
                      n_pts=17))
    if force:
        os.environ["DPK_FORCE_GENERIC"] = "1"
    if per_op:                     # the per-op launches even where a fused width instance exists
        os.environ["DPK_GEN_FUSED"] = "0"
    try:
        m = HipGCNdiff(adj_mx_from_edges(), cfg, device="cuda:0")
    finally:
        os.environ.pop("DPK_FORCE_GENERIC", None)
        os.environ.pop("DPK_GEN_FUSED", None)
    m.load_state_dict(synthetic_state_dict(hid=hid, n_layers=layers))
    x = torch.from_numpy(synthetic_batch(n, seed=1)[0]).cuda()
    seq = make_seq("uniform", 50, k)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
    m.sample(x, seq, b)
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.sample(x, seq, b)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[2]
    print(f"{label:48s} {t * 1e3:9.2f} ms  {n / t:10.0f} poses/s")
    m.close()


if __name__ == "__main__":
    if len(sys.argv) > 1:          # one shape: generic_bench.py HID HEADS LAYERS [force]  (profiling runs)
        hid, heads, layers = (int(v) for v in sys.argv[1:4])
        run(f"hid {hid} / {heads} heads / {layers} layers", hid, heads, layers, force=len(sys.argv) > 4)
        sys.exit(0)
    run("persistent sampler, hid 96 / 4 heads / 5 layers", 96, 4, 5)
    run("generic path (forced), hid 96 / 4 heads / 5 layers", 96, 4, 5, force=True)
    run("generic path per-op, hid 64 / 2 heads / 2 layers", 64, 2, 2, per_op=True)
    run("fused sampler (dpkn), hid 64 / 2 heads / 2 layers", 64, 2, 2)
    run("generic path per-op, hid 64 / 2 heads / 5 layers", 64, 2, 5, per_op=True)
    run("fused sampler (dpkn), hid 64 / 2 heads / 5 layers", 64, 2, 5)
    run("generic path per-op, hid 128 / 8 heads / 5 layers", 128, 8, 5, per_op=True)
    run("fused wide sampler (dpkw), hid 128 / 8 heads / 5 layers", 128, 8, 5)
    run("generic path per-op, hid 128 / 4 heads / 5 layers", 128, 4, 5, per_op=True)
    run("fused sampler (dpkw4), hid 128 / 4 heads / 5 layers", 128, 4, 5)
    run("generic path per-op, hid 64 / 4 heads / 5 layers", 64, 4, 5, per_op=True)
    run("fused sampler (dpkn4), hid 64 / 4 heads / 5 layers", 64, 4, 5)
