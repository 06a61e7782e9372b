"""Localise a fused-vs-per-op difference of the other-width sampler instances (debug aid, GPU box):
per (hid, heads, layers, graph, batch): max |fused - per-op| and |fused - oracle| of the K=10 final.
  python tools/dbg_dpkn.py
"""
import os
import sys
from types import SimpleNamespace as ns

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))
sys.path.insert(0, ROOT)
from diffpose_amd.data import synthetic_batch  # noqa: E402
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges  # noqa: E402
from diffpose_amd.schedule import get_beta_schedule, make_seq  # noqa: E402
from diffpose_amd.weights import synthetic_state_dict  # noqa: E402
from oracle import gcndiff_oracle as O  # noqa: E402


def cfg(hid, heads, layers):
    return ns(model=ns(hid_dim=hid, emd_dim=hid, coords_dim=[5, 5], num_layer=layers, n_head=heads, dropout=0.0,
                       n_pts=17))


def main():
    torch.set_num_threads(8)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
    rng = np.random.default_rng(3)
    dense = adj_mx_from_edges() + 0.1 * (rng.random((17, 17)) > 0.6)
    dense = ((dense + dense.T) / 2).astype(np.float32)
    ones = torch.ones(1, 1, 17, dtype=torch.bool)
    for hid, heads in ((64, 2), (128, 8)):
        for layers, gname in ((2, "dense"), (2, "h36m"), (5, "dense")):
            adj = dense if gname == "dense" else adj_mx_from_edges()
            sd = synthetic_state_dict(hid=hid, n_layers=layers)
            P = O.params_to_torch(sd)
            fwd = lambda a, mk, tt: O.gcndiff_forward(P, torch.from_numpy(adj), a, mk, tt, n_layers=layers, heads=heads)  # noqa: E731
            for n, k in ((37, 10), (8, 1), (8, 2)):
                x = torch.from_numpy(synthetic_batch(n, seed=91)[0])
                seq = make_seq("uniform", 50, k)
                res = {}
                for fused in ("1", "0"):
                    os.environ["DPK_GEN_FUSED"] = fused
                    m = HipGCNdiff(adj, cfg(hid, heads, layers), device="cuda:0")
                    m.load_state_dict(sd)
                    res[fused] = m.sample(x.cuda(), seq, b, mask=ones.cuda(), trajectory=True)[0].cpu()
                    m.close()
                os.environ.pop("DPK_GEN_FUSED", None)
                rxs, _ = O.generalized_steps(x, ones, seq, fwd, b)
                ref = torch.stack(rxs)
                d_fp = float((res["1"] - res["0"]).abs().max())
                d_fo = float((res["1"] - ref).abs().max())
                d_po = float((res["0"] - ref).abs().max())
                # first step index where fused departs from the oracle by more than 5e-6
                per_step = [(float((res["1"][i] - ref[i]).abs().max())) for i in range(ref.shape[0])]
                bad = next((i for i, v in enumerate(per_step) if v > 5e-6), None)
                worst_pose = int((res["1"][-1] - ref[-1]).abs().amax(dim=(1, 2)).argmax())
                print(f"hid {hid:3d}/{heads} L{layers} {gname:5s} N={n:2d} K={k:2d}: fused-perop {d_fp:.2e} "
                      f"fused-oracle {d_fo:.2e} perop-oracle {d_po:.2e}  first bad step {bad}  worst pose {worst_pose}",
                      flush=True)


if __name__ == "__main__":
    main()
