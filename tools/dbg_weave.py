"""Debug aid (GPU box): run-to-run determinism of a gemm mode at B=1024, K=50, and where two libraries'
outputs differ (poses within their 4-pose tile, joints, channels).
  python tools/dbg_weave.py MODE OUT.npy          # writes two runs' outputs (2, N, 17, 5)
  python tools/dbg_weave.py --compare A.npy B.npy
"""
import os
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for name, x in (("A run-to-run", a[0] - a[1]), ("B run-to-run", b[0] - b[1]), ("A vs B", a[0] - b[0])):
        d = np.abs(x)
        print(f"{name}: max {d.max():.3e}, poses differing {int((d.reshape(d.shape[0], -1).max(1) > 1e-6).sum())}")
        if d.max() > 1e-6:
            bad = d.max(axis=(1, 2)) > 1e-6
            idx = np.nonzero(bad)[0]
            print("   first poses", idx[:12].tolist(), " pose % 4 histogram", np.bincount(idx % 4, minlength=4).tolist())
            j = d[bad].max(axis=(0, 2))
            print("   per-joint max", np.round(j, 5).tolist())
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "diffpose-nw_amd"))
from diffpose_amd.data import synthetic_batch  # noqa: E402
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges  # noqa: E402
from diffpose_amd.schedule import get_beta_schedule, make_seq  # noqa: E402
from diffpose_amd.weights import synthetic_state_dict  # noqa: E402

m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
m.load_state_dict(synthetic_state_dict())
m.set_gemm_mode(sys.argv[1])
x = torch.from_numpy(synthetic_batch(1024, seed=19960903)[0]).cuda()
b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
seq = make_seq("uniform", 50, 50)
outs = [m.sample(x, seq, b).cpu().numpy() for _ in range(2)]
np.save(sys.argv[2], np.stack(outs))
