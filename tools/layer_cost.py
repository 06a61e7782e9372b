"""Per-layer and per-step-fixed cost of the sampler launch (GPU box): times the B=1024, K=50 sampler
with num_layer = 1..5 (a run-time layer count of the same kernel) and fits t = fixed + L * per_layer.

  python tools/layer_cost.py
"""
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))


def main():
    import numpy as np
    import torch
    from diffpose_amd.data import synthetic_batch
    from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict

    x = torch.from_numpy(synthetic_batch(1024)[0]).cuda()
    seq = make_seq("uniform", 50, 50)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
    res = {}
    for nl in (1, 2, 3, 4, 5):
        cfg = SimpleNamespace(model=SimpleNamespace(hid_dim=96, num_layer=nl, n_head=4, n_pts=17, coords_dim=[5, 5]))
        m = HipGCNdiff(adj_mx_from_edges(), cfg, device="cuda:0")
        m.load_state_dict(synthetic_state_dict(n_layers=nl))
        out = torch.empty_like(x)
        m.sample(x, seq, b, out=out)
        torch.cuda.synchronize()
        m.profile(True)
        for _ in range(10):
            m.sample(x, seq, b, out=out)
        torch.cuda.synchronize()
        t = m.kernel_times_ms()[-10:]
        res[nl] = float(np.median(t))
        m.close()
        print(f"num_layer {nl}: median launch {res[nl]:.4f} ms", flush=True)
    L = np.array(sorted(res))
    T = np.array([res[k] for k in L])
    per_layer, fixed = np.polyfit(L, T, 1)
    print(f"fit: launch = {fixed:.4f} ms + L x {per_layer:.4f} ms  (per DDIM step: {fixed / 50 * 1e3:.2f} us fixed, "
          f"{per_layer / 50 * 1e3:.2f} us per layer; residuals {np.round(T - (fixed + per_layer * L), 4).tolist()})")


if __name__ == "__main__":
    main()
