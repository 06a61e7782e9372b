"""Generate golden vectors from the REFERENCE itself (runs in the build container only).

Imports the reference read-only from /root/reference (PYTHONPATH), loads the
build's seeded synthetic weights into the reference ``GCNdiff``, runs the
reference ``generalized_steps`` / modules on seeded synthetic inputs on CPU,
and writes small .npz fixtures to tests/golden/.  Nothing here runs on the GPU
box; only the fixtures are committed.

The reference hard-codes ``.cuda()`` in ``generalized_steps``
(common/utils_diff.py:53-54); on this CPU-only container the shim
``torch.Tensor.cuda = identity`` keeps everything on CPU.

Usage:  python tools/gen_goldens.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden"))
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    sys.dont_write_bytecode = True

    import torch
    torch.Tensor.cuda = lambda self, *a, **k: self          # CPU shim (see module doc)
    torch.set_num_threads(8)

    from models.gcndiff import GCNdiff, get_timestep_embedding, nonlinearity
    from models.GraFormer import adj_mx_from_edges, LAM_Gconv
    from models.ChebConv import ChebConv
    from common.utils_diff import generalized_steps, get_beta_schedule
    from common.loss import mpjpe

    from diffpose_amd.weights import synthetic_state_dict, state_dict_sha256
    from diffpose_amd.data import synthetic_batch

    os.makedirs(args.out, exist_ok=True)
    cfg = types.SimpleNamespace(model=types.SimpleNamespace(
        hid_dim=96, emd_dim=96, coords_dim=[5, 5], num_layer=5, n_head=4, dropout=0.25, n_pts=17))
    edges = torch.tensor([[0, 1], [1, 2], [2, 3], [0, 4], [4, 5], [5, 6], [0, 7], [7, 8], [8, 9], [9, 10],
                          [8, 11], [11, 12], [12, 13], [8, 14], [14, 15], [15, 16]], dtype=torch.long)
    adj = adj_mx_from_edges(num_pts=17, edges=edges, sparse=False)

    sd = synthetic_state_dict()
    sha = state_dict_sha256(sd)
    model = GCNdiff(adj, cfg)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval()
    mask = torch.tensor([[[True] * 17]])
    meta = {"weights_sha256": sha, "torch": torch.__version__, "generator": "tools/gen_goldens.py",
            "reference": "nwicakson/diffpose-nw @ /root/reference"}

    # ---------------- G1: graph constants ----------------
    L = ChebConv.get_laplacian(adj, True)
    cheb = ChebConv(96, 96, K=2).cheb_polynomial(L)
    lam = LAM_Gconv(96, 96)
    lg = np.stack([lam.laplacian_batch(model.atten_layers[i].feed_forward.A_hat.detach()[None])[0].numpy()
                   for i in range(5)])
    np.savez(os.path.join(args.out, "g1_graph.npz"), adj=adj.numpy(), cheb=cheb.numpy(), lg=lg)

    # ---------------- G2: per-module outputs ----------------
    x6, _ = synthetic_batch(6, seed=101)
    x6 = torch.from_numpy(x6)
    with torch.no_grad():
        t6 = torch.tensor([49.0, 0.0, 12.0, 12.0, 49.0, 31.0])
        temb = get_timestep_embedding(t6, 96)
        d0 = model.temb.dense[0](temb)
        temb_full = model.temb.dense[1](nonlinearity(d0))
        h_in = model.gconv_input(x6, adj)
        al = model.atten_layers[0]
        ln0 = al.sublayer[0].norm(h_in)
        mha = al.self_attn(ln0, ln0, ln0, mask)
        p_attn = al.self_attn.attn
        x_a = h_in + mha
        ln1 = al.sublayer[1].norm(x_a)
        gn = al.feed_forward(ln1)
        x_b = x_a + gn
        res = model.gconv_layers[0](x_b, temb_full)
        h_out_in = torch.randn(6, 17, 96, generator=torch.Generator().manual_seed(7))
        cheb_out = model.gconv_output(h_out_in, adj)
        eps = model(x6, mask, t6, 0)
        # masked attention (a key mask with two False entries) through the whole model
        mask2 = mask.clone()
        mask2[0, 0, 3] = False
        mask2[0, 0, 11] = False
        eps_masked = model(x6, mask2, t6, 0)
    np.savez(os.path.join(args.out, "g2_modules.npz"), x=x6.numpy(), t=t6.numpy(), temb=temb.numpy(),
             temb_full=temb_full.numpy(), h_in=h_in.numpy(), ln0=ln0.numpy(), mha=mha.numpy(),
             p_attn=p_attn.numpy(), x_a=x_a.numpy(), ln1=ln1.numpy(), graphnet=gn.numpy(),
             x_b=x_b.numpy(), res_cheb=res.numpy(), h_out_in=h_out_in.numpy(), cheb_out=cheb_out.numpy(),
             eps=eps.numpy(), mask2=mask2.numpy(), eps_masked=eps_masked.numpy())

    # ---------------- G3/G4: sampler trajectories ----------------
    def betas_for(T):
        b = get_beta_schedule("linear", beta_start=0.0001, beta_end=0.001, num_diffusion_timesteps=T)
        return torch.from_numpy(b).float()

    def run(n, seq, T, seed, eta=0.0):
        x, tgt = synthetic_batch(n, seed=seed)
        x = torch.from_numpy(x)
        xs, x0s = generalized_steps(x, mask, seq, model, betas_for(T), eta=eta)
        return x.numpy(), tgt, xs, x0s

    seq10 = list(range(0, 50, 5))
    x, tgt, xs, x0s = run(64, seq10, 51, 202)
    out = xs[-1]
    xyz = out[:, :, 2:].clone()
    xyz = xyz - xyz[:, :1, :].clone()
    tt = torch.from_numpy(tgt)
    np.savez(os.path.join(args.out, "g3_traj_n64_k10.npz"), x=x, seq=np.array(seq10), T=51,
             xs=torch.stack(xs).numpy(), x0s=torch.stack(x0s).numpy(), targets=tgt,
             mpjpe_mm=np.float64(mpjpe(xyz, tt).item() * 1000.0))

    seq50 = list(range(0, 50, 1))
    x, tgt, xs, x0s = run(16, seq50, 51, 303)
    np.savez(os.path.join(args.out, "g4_final_n16_k50.npz"), x=x, seq=np.array(seq50), T=51,
             out=xs[-1].numpy(), x0_last=x0s[-1].numpy(), targets=tgt)

    seq100 = list(range(0, 100, 1))
    x, tgt, xs, x0s = run(16, seq100, 101, 404)
    np.savez(os.path.join(args.out, "g4_final_n16_k100_T101.npz"), x=x, seq=np.array(seq100), T=101,
             out=xs[-1].numpy(), x0_last=x0s[-1].numpy(), targets=tgt)

    seqq = [int(s) for s in list(np.linspace(0, np.sqrt(50 * 0.8), 10) ** 2)]   # quad skip, has duplicates
    x, tgt, xs, x0s = run(8, seqq, 51, 505)
    np.savez(os.path.join(args.out, "g4_final_n8_quad.npz"), x=x, seq=np.array(seqq), T=51,
             out=xs[-1].numpy(), targets=tgt)

    # ---------------- G5: in-place root subtraction quirk ----------------
    q = torch.from_numpy(synthetic_batch(3, seed=606)[0][:, :, 2:].copy())
    q_in = q.clone()
    q[:, :, :] -= q[:, :1, :]
    try:
        q1 = q_in[:1].clone()
        q1[:, :, :] -= q1[:, :1, :]
        b1_raises = False
    except RuntimeError:
        b1_raises = True
    np.savez(os.path.join(args.out, "g5_root_quirk.npz"), x=q_in.numpy(), out=q.numpy(), b1_raises=b1_raises)

    with open(os.path.join(args.out, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
