"""Sampler throughput against batch size on one GPU (B poses, K=50): full rounds of 4-pose tiles (256 per
round, one per CU), partial rounds, and the 2-pose tail round (launch_sampler).

  python tools/batch_sweep.py            # GPU box
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))


def main():
    import numpy as np
    import torch
    from diffpose_amd.data import synthetic_batch
    from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict

    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict())
    seq = make_seq("uniform", 50, 50)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
    xall = torch.from_numpy(synthetic_batch(8192)[0]).cuda()
    print(f"{'B':>6} {'launch ms':>10} {'poses/s':>10} {'vs B=1024':>10}  rounds", flush=True)
    ref = None
    for B in (64, 256, 512, 768, 1000, 1024, 1100, 1280, 1536, 2048, 2560, 3072, 4096, 8192):
        x = xall[:B].contiguous()
        out = torch.empty_like(x)
        m.sample(x, seq, b, out=out)
        torch.cuda.synchronize()
        # stream-ordered events around 5 whole calls (a call may launch a full-round and a tail-round kernel)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            m.sample(x, seq, b, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        rate = B / (ms * 1e-3)
        if B == 1024:
            ref = rate
        tiles = (B + 3) // 4
        print(f"{B:>6} {ms:>10.3f} {rate:>10.0f} {'' if ref is None else f'{rate / ref:>10.3f}'}  {tiles / 256:.2f} x 4-pose",
              flush=True)
    m.close()


if __name__ == "__main__":
    main()
