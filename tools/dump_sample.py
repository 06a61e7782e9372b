# Dump one K=50 sampler output (1024 poses, mixed per-pose masks) for bitwise A/B of two builds:
#   DPK_LIB=... python tools/dump_sample.py out.npy [gemm mode]
import sys, numpy as np, torch
sys.path.insert(0, "diffpose-nw_amd")
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.weights import synthetic_state_dict
from diffpose_amd.data import synthetic_batch
from diffpose_amd.schedule import get_beta_schedule, make_seq
m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0"); m.load_state_dict(synthetic_state_dict())
if len(sys.argv) > 2: m.set_gemm_mode(sys.argv[2])
x, _ = synthetic_batch(1024, seed=5)
b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
mk = torch.ones(1024, 1, 17, dtype=torch.bool); mk[1::3, 0, [2, 16]] = False
out = m.sample(torch.from_numpy(x).cuda(), make_seq("uniform", 50, 50), b, mask=mk.cuda())
np.save(sys.argv[1], out.cpu().numpy())
