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
import hashlib
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
    ap.add_argument("--only", default="", help="comma list of fixture groups (g1, g2, g34, g5..g9, g11); default all")
    args = ap.parse_args()
    only = set(x for x in args.only.split(",") if x)

    def want(g):
        return not only or g in only
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
    meta_path = os.path.join(args.out, "meta.json")
    meta = json.load(open(meta_path)) if (only and os.path.exists(meta_path)) else {}
    meta.update({"weights_sha256": sha, "torch": torch.__version__, "generator": "tools/gen_goldens.py",
                 "reference": "nwicakson/diffpose-nw @ /root/reference"})

    # ---------------- G1: graph constants ----------------
    if want("g1"):
        L = ChebConv.get_laplacian(adj, True)
        cheb = ChebConv(96, 96, K=2).cheb_polynomial(L)
        lam = LAM_Gconv(96, 96)
        lg = np.stack([lam.laplacian_batch(model.atten_layers[i].feed_forward.A_hat.detach()[None])[0].numpy()
                       for i in range(5)])
        np.savez(os.path.join(args.out, "g1_graph.npz"), adj=adj.numpy(), cheb=cheb.numpy(), lg=lg)

    # ---------------- G2: per-module outputs ----------------
    if want("g2"):
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
    if want("g34"):
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
    if want("g5"):
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

    # ---------------- G6: GCNpose front-end + uvxyz assembly ----------------
    if want("g6"):
        from models.gcnpose import GCNpose

        psd = synthetic_state_dict(kind="pose")
        pcfg = types.SimpleNamespace(model=types.SimpleNamespace(
            hid_dim=96, emd_dim=96, coords_dim=[2, 3], num_layer=5, n_head=4, dropout=0.25, n_pts=17))
        pm = GCNpose(adj, pcfg)
        pm.load_state_dict({k: torch.from_numpy(v) for k, v in psd.items()})
        pm.eval()
        x12, _ = synthetic_batch(12, seed=707)
        x2d = torch.from_numpy(np.ascontiguousarray(x12[:, :, :2]))
        mask2 = mask.clone()
        mask2[0, 0, 5] = False
        with torch.no_grad():
            xyz = pm(x2d, mask)
            xyz_masked = pm(x2d, mask2)
            # test_hyber's assembly (runners/diffpose_frame.py:337-342), same torch ops
            inputs_xyz = xyz.clone()
            inputs_xyz[:, :, :] -= inputs_xyz[:, :1, :]
            uvxyz = torch.cat([x2d, inputs_xyz], dim=2).repeat(3, 1, 1)
        np.savez(os.path.join(args.out, "g6_gcnpose.npz"), x2d=x2d.numpy(), xyz=xyz.numpy(),
                 xyz_masked=xyz_masked.numpy(), mask2=mask2.numpy(), uvxyz_h3=uvxyz.numpy())
        meta["pose_weights_sha256"] = state_dict_sha256(psd, kind="pose")

    # ---------------- G7: metrics and per-action accounting ----------------
    if want("g7"):
        from common.loss import mpjpe as loss_mpjpe, p_mpjpe as loss_p_mpjpe
        from common.utils import define_error_list, print_error, test_calculation
        from common.utils import p_mpjpe as utils_p_mpjpe

        rng = np.random.Generator(np.random.PCG64(808))
        n = 48
        tgt = rng.normal(0.0, 0.25, size=(n, 17, 3))
        tgt = tgt - tgt[:, :1]
        pred = np.empty_like(tgt)
        for i in range(n):                      # scaled, rotated (some reflected), shifted, noisy
            q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
            if i % 5 == 0:
                q[:, 0] = -q[:, 0] if np.linalg.det(q) > 0 else q[:, 0]
            pred[i] = rng.uniform(0.7, 1.3) * tgt[i] @ q + rng.normal(0, 0.1, 3) + rng.normal(0, 0.03, (17, 3))
        tgt = tgt.astype(np.float32)
        pred = pred.astype(np.float32)
        names = ["Directions", "Discussion", "Eating", "Greeting", "Phoning", "Photo", "Posing", "Purchases",
                 "Sitting", "SittingDown", "Smoking", "Waiting", "WalkDog", "Walking", "WalkTogether"]
        acts = ["Walking 1"] * 16 + [names[int(k)] + ("" if k % 3 == 0 else f" {1 + int(k) % 2}")
                                     for k in rng.integers(0, 15, size=n - 16)]
        bounds = [(0, 16), (16, 32), (32, 48)]
        err = define_error_list(names)
        for lo, hi in bounds:
            test_calculation(torch.from_numpy(pred[lo:hi]), torch.from_numpy(tgt[lo:hi]), acts[lo:hi], err, None, None)
        p1, p2 = print_error(None, err, 1)
        np.savez(os.path.join(args.out, "g7_metrics.npz"), pred=pred, tgt=tgt, actions=np.array(acts),
                 bounds=np.array(bounds), per_pose_p2=utils_p_mpjpe(pred, tgt),
                 loss_p2=np.float64(loss_p_mpjpe(pred, tgt)),
                 loss_p1=np.float64(loss_mpjpe(torch.from_numpy(pred), torch.from_numpy(tgt)).item()),
                 p1=np.float64(p1), p2=np.float64(p2), action_names=np.array(names),
                 action_p1=np.array([err[a]["p1"].avg for a in names], dtype=np.float64),
                 action_p2=np.array([err[a]["p2"].avg for a in names], dtype=np.float64))

    # ---------------- G8: GMM input sampler (common/generators.py) ----------------
    if want("g8"):
        from common.generators import PoseGenerator_gmm

        rng = np.random.Generator(np.random.PCG64(4242))
        lens, kn = (7, 5, 9), 5
        p3s, gms, acts, cams = [], [], [], []
        for si, n in enumerate(lens):
            w = rng.dirichlet(np.ones(kn), size=(n, 17))
            w[0, 0] = [1, 0, 0, 0, 0]                # one-hot rows and interior zeros
            w[0, 1] = [0, 0, 0, 0, 1]
            w[1, 2] = [0.5, 0, 0.25, 0, 0.25]
            g = np.empty((n, 17, kn, 5))
            g[..., 0] = w
            g[..., 1:3] = rng.uniform(-1, 1, size=(n, 17, kn, 2))
            g[..., 3:5] = rng.uniform(1e-4, 1e-2, size=(n, 17, kn, 2))
            gms.append(g.astype(np.float32))
            p3s.append(rng.normal(0.0, 0.4, size=(n, 17, 3)).astype(np.float32) + np.float32(si))
            acts.append([f"Walking {si}"] * n)
            cams.append(rng.normal(size=(n, 9)).astype(np.float32))
        ds = PoseGenerator_gmm([a.copy() for a in p3s], [a.copy() for a in gms], acts, cams)
        indices = [0, 3, 20, 7, 21, 13, 5, 20, 1]
        np.random.seed(2024)
        items = [ds[i] for i in indices]
        np.random.seed(2024)
        u = np.random.random_sample((len(indices), 17))
        np.savez(os.path.join(args.out, "g8_gmm.npz"), poses_3d=np.concatenate(p3s), gmm=np.concatenate(gms),
                 lens=np.array(lens), indices=np.array(indices), u=u,
                 uvxyz=np.stack([it[0].numpy() for it in items]), noise_scale=np.stack([it[1].numpy() for it in items]),
                 pose_2d=np.stack([it[2].numpy() for it in items]), pose_3d=np.stack([it[3].numpy() for it in items]),
                 actions=np.array([it[4] for it in items]), camerapara=np.stack([it[5].numpy() for it in items]))

    # ---------------- G9/G10: other weight distributions ----------------
    # G9: the reference's OWN initialisers (a freshly constructed GCNdiff under torch.manual_seed(s),
    # models/ChebConv.py:62-67, models/gcndiff.py:70-98), s = 0, 1; G10: the build's generator at a
    # second seed (7).  Each: eps at mixed t, and the K=50 final in fp32 and in fp64 (the model and
    # schedule cast to double; the timestep embedding and the Chebyshev tables are float32 by
    # construction, so they are cast for that run) — the fp32-vs-fp64 gap sets the tolerance scale for these weights.
    if want("g9"):
        import models.gcndiff as gcndiff_mod
        from diffpose_amd.weights import reference_init_state_dict

        def fixture(m, name, seed_x, extra):
            xq, tgt = synthetic_batch(32, seed=seed_x)
            xq = torch.from_numpy(xq)
            t8 = torch.tensor([49.0, 0.0, 12.0, 31.0, 7.0, 49.0, 25.0, 3.0])
            b = torch.from_numpy(get_beta_schedule("linear", beta_start=0.0001, beta_end=0.001,
                                                   num_diffusion_timesteps=51)).float()
            seq50 = list(range(0, 50, 1))
            with torch.no_grad():
                eps = m(xq[:8], mask, t8, 0)
            xs, _ = generalized_steps(xq, mask, seq50, m, b, eta=0.0)
            m64 = copy.deepcopy(m).double()
            m64.adj = adj.double()
            for layer in m64.gconv_layers:
                layer.adj = m64.adj
            # float32 by construction in the reference: the timestep embedding and the Chebyshev
            # tables (models/ChebConv.py:98-99); cast to double for this run only
            orig = gcndiff_mod.get_timestep_embedding
            orig_cp = ChebConv.cheb_polynomial
            gcndiff_mod.get_timestep_embedding = lambda t, d: orig(t, d).double()
            ChebConv.cheb_polynomial = lambda self_, L: orig_cp(self_, L.float()).to(L.dtype)
            try:
                xs64, _ = generalized_steps(xq.double(), mask, seq50, m64, b.double(), eta=0.0)
            finally:
                gcndiff_mod.get_timestep_embedding = orig
                ChebConv.cheb_polynomial = orig_cp
            np.savez(os.path.join(args.out, name), x=xq.numpy(), t8=t8.numpy(), eps=eps.numpy(), seq=np.array(seq50),
                     T=51, out=xs[-1].numpy(), out64=xs64[-1].numpy(), targets=tgt, **extra)

        import copy
        shas = {}
        for s_ in (0, 1):
            torch.manual_seed(s_)
            m = GCNdiff(adj, cfg)
            m.eval()
            ref_sd = {k: v.detach().numpy() for k, v in m.state_dict().items()}
            shas[str(s_)] = state_dict_sha256(ref_sd)
            assert shas[str(s_)] == state_dict_sha256(reference_init_state_dict(s_)), "restated initialisers drifted"
            fixture(m, f"g9_refinit_seed{s_}.npz", 900 + s_, {"init_seed": s_})
        meta["refinit_sha256"] = shas
        sd7 = synthetic_state_dict(seed=7)
        m7 = GCNdiff(adj, cfg)
        m7.load_state_dict({k: torch.from_numpy(v) for k, v in sd7.items()})
        m7.eval()
        fixture(m7, "g10_synth_seed7.npz", 907, {"weights_seed": 7})
        meta["seed7_weights_sha256"] = state_dict_sha256(sd7)

    # ---------------- G11: eta > 0 with the reference's own per-step randn_like ----------------
    # generalized_steps draws torch.randn_like(x) once per step (common/utils_diff.py:65); under
    # torch.manual_seed(s) the K draws are reproducible, so the fixture stores them beside the
    # trajectory they produced.  test_hyber draws one more randn_like before the sampler
    # (runners/diffpose_frame.py:359): the "hyber" final is the sampler run after that draw.
    if want("g11"):
        def betas51():
            return torch.from_numpy(get_beta_schedule("linear", beta_start=0.0001, beta_end=0.001,
                                                      num_diffusion_timesteps=51)).float()
        x, tgt = synthetic_batch(16, seed=1111)
        x = torch.from_numpy(x)
        seq10 = list(range(0, 50, 5))
        torch.manual_seed(11)
        xs, x0s = generalized_steps(x, mask, seq10, model, betas51(), eta=0.5)
        torch.manual_seed(11)
        noise10 = torch.stack([torch.randn_like(x) for _ in seq10])
        torch.manual_seed(12)
        _e = torch.randn_like(x)                       # runners/diffpose_frame.py:359 (unused by the sampler)
        xs_h, _ = generalized_steps(x, mask, seq10, model, betas51(), eta=0.5)
        seq50 = list(range(0, 50, 1))
        torch.manual_seed(13)
        xs50, _ = generalized_steps(x, mask, seq50, model, betas51(), eta=1.0)
        torch.manual_seed(13)
        noise50 = torch.stack([torch.randn_like(x) for _ in seq50])
        np.savez(os.path.join(args.out, "g11_eta.npz"), x=x.numpy(), targets=tgt, T=51,
                 seq10=np.array(seq10), eta10=np.float32(0.5), seed10=11, noise10=noise10.numpy(),
                 xs10=torch.stack(xs).numpy(), x0s10=torch.stack(x0s).numpy(),
                 seed_hyber=12, out_hyber=xs_h[-1].numpy(),
                 seq50=np.array(seq50), eta50=np.float32(1.0), seed50=13, noise50=noise50.numpy(),
                 out50=xs50[-1].numpy())

    # ---------------- G12: other model shapes (round 6) ----------------
    # The reference builds GCNdiff from any config.model (models/gcndiff.py:55-99; d_k = hid / n_head,
    # models/GraFormer.py:116-124): the shapes the build runs on its other persistent-sampler instances
    # (hid 128 / 8 heads, 128 / 4, 64 / 2, 64 / 4 on the H36M graph) and on the per-op generic path
    # (hid 48 / 4 heads on a 16-joint chain), each with the build's generator weights at that shape: eps at
    # 8 mixed t with the all-ones and a two-key mask, and a K=10 trajectory on 8 frames.
    if want("g12"):
        chain16 = torch.tensor([[i, i + 1] for i in range(15)], dtype=torch.long)
        shapes = [(128, 8, 5, 17, edges), (128, 4, 3, 17, edges), (64, 2, 2, 17, edges), (64, 4, 5, 17, edges),
                  (48, 4, 1, 16, chain16)]
        b51 = torch.from_numpy(get_beta_schedule("linear", beta_start=0.0001, beta_end=0.001,
                                                 num_diffusion_timesteps=51)).float()
        shas = {}
        for hid, nh, nl, npts, ed in shapes:
            scfg = types.SimpleNamespace(model=types.SimpleNamespace(
                hid_dim=hid, emd_dim=hid, coords_dim=[5, 5], num_layer=nl, n_head=nh, dropout=0.25, n_pts=npts))
            sadj = adj_mx_from_edges(num_pts=npts, edges=ed, sparse=False)
            ssd = synthetic_state_dict(hid=hid, n_layers=nl, n_pts=npts)
            sm = GCNdiff(sadj, scfg)
            sm.load_state_dict({k: torch.from_numpy(v) for k, v in ssd.items()})
            sm.eval()
            smask = torch.tensor([[[True] * npts]])
            smask2 = smask.clone()
            smask2[0, 0, 2] = False
            smask2[0, 0, npts - 1] = False
            name = f"g12_shape_h{hid}_n{nh}_l{nl}_j{npts}"
            x8, _ = synthetic_batch(8, seed=1200 + hid + nh, num_pts=npts)
            x8 = torch.from_numpy(x8)
            t8 = torch.tensor([49.0, 0.0, 12.0, 31.0, 7.0, 49.0, 25.0, 3.0])
            with torch.no_grad():
                eps = sm(x8, smask, t8, 0)
                eps_masked = sm(x8, smask2, t8, 0)
            seq10 = list(range(0, 50, 5))
            xs, x0s = generalized_steps(x8, smask, seq10, sm, b51, eta=0.0)
            np.savez(os.path.join(args.out, name + ".npz"), hid=hid, n_head=nh, num_layer=nl, n_pts=npts,
                     edges=ed.numpy(), adj=sadj.numpy(), x=x8.numpy(), t8=t8.numpy(), eps=eps.numpy(),
                     mask2=smask2.numpy(), eps_masked=eps_masked.numpy(), seq=np.array(seq10), T=51,
                     xs=torch.stack(xs).numpy(), x0s=torch.stack(x0s).numpy())
            hh = hashlib.sha256()
            for k_, v_ in ssd.items():        # the generator's layout order at this shape
                hh.update(k_.encode())
                hh.update(np.ascontiguousarray(v_, dtype="<f4").tobytes())
            shas[name] = hh.hexdigest()
        meta["shape_weights_sha256"] = shas

    with open(os.path.join(args.out, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
