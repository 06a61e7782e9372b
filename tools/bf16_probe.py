import sys, os, numpy as np, torch, time
sys.path.insert(0, "diffpose-nw_amd"); sys.path.insert(0, ".")
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.data import synthetic_batch
from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict
from oracle import gcndiff_oracle as O
torch.set_num_threads(16)
def betas(T): return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=T)).float()
def mpjpe(o, t):
    o = np.asarray(o, np.float64); xyz = o[:, :, 2:] - o[:, :1, 2:]
    return float(np.mean(np.linalg.norm(xyz - t, axis=-1)) * 1000)
sd = synthetic_state_dict()
m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0"); m.load_state_dict(sd)
g = np.load("tests/golden/g2_modules.npz")
mask = torch.ones(1,1,17,dtype=torch.bool,device="cuda:0")
for mode in ("fp32","f16x3","bf16"):
    m.set_gemm_mode(mode)
    e = m(torch.from_numpy(g["x"]).cuda(), mask, torch.from_numpy(g["t"]).cuda(), 0).cpu().numpy()
    print(mode, "eps maxdiff", np.abs(e-g["eps"]).max(), "eps maxabs", np.abs(g["eps"]).max())
P = O.params_to_torch(sd)
for (T, Tt, K, n) in ((51, 50, 50, 256), (101, 100, 100, 256)):
    x, tgt = synthetic_batch(n, seed=19960903)
    seq = make_seq("uniform", Tt, K)
    xs, _ = O.generalized_steps(torch.from_numpy(x), torch.ones(1,1,17,dtype=torch.bool), seq, lambda a, mk, t: O.gcndiff_forward(P, O.adjacency(), a, mk, t), betas(T))
    ref = xs[-1].numpy()
    for mode in ("fp32","f16x3","bf16"):
        m.set_gemm_mode(mode)
        out = m.sample(torch.from_numpy(x).cuda(), seq, betas(T)).cpu().numpy()
        print(f"K={K} T={T} {mode}: maxdiff {np.abs(out-ref).max():.3e} mpjpe hip {mpjpe(out,tgt):.6f} ref {mpjpe(ref,tgt):.6f} delta {abs(mpjpe(out,tgt)-mpjpe(ref,tgt)):.3e}")
