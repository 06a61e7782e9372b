"""Bitwise A/B of two libdpk builds (GPU box): every kernel instance's outputs on fixed inputs.

  DPK_LIB=build/ab/x.so python tools/bitwise_ab.py dump OUT.npz [--quick]
  python tools/bitwise_ab.py compare A.npz B.npz

The dump runs, on one process and device:
  - the 4-pose sampler at B=1024, K=50 in gemm modes fp32 / f16x3 / bf16 with mixed per-pose key masks
    (twice for the half-width modes: run-to-run determinism is part of the check);
  - bf16 at K=100 over T=101 (BASELINE config 3's schedule);
  - B=1100 (step-split last round) and B=1026 (2-pose tail tiles) in fp32 and bf16;
  - one eps evaluation per gemm mode at mixed t (the M_EPS instance);
  - GCNpose (the M_POSE instance);
  - the wide / narrow persistent-sampler instances of the generic path (dpkw hid 128 / 8 heads,
    dpkw4 hid 128 / 4, dpkn hid 64 / 2, dpkn4 hid 64 / 4) at B=512, K=50.
`compare` prints per key whether the two files are bitwise equal (and the max |diff| if not) and exits
non-zero on any difference.  Used to prove that a source change (a hazard pad, a deleted experiment
branch) leaves every shipped instance's results untouched.
"""
import os
import sys
from types import SimpleNamespace as ns

import numpy as np


def compare(a_path, b_path):
    a, b = np.load(a_path), np.load(b_path)
    bad = 0
    for k in sorted(set(a.files) | set(b.files)):
        if k not in a.files or k not in b.files:
            print(f"{k:28s} MISSING in {'A' if k not in a.files else 'B'}")
            bad += 1
            continue
        x, y = a[k], b[k]
        same = x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
        if same:
            print(f"{k:28s} bitwise equal  {x.shape}")
        else:
            d = np.abs(x.astype(np.float64) - y.astype(np.float64)) if x.shape == y.shape else np.array([np.inf])
            print(f"{k:28s} DIFFERS        max |d| {d.max():.3e}")
            bad += 1
    # run-to-run pairs inside each file
    for name, f in (("A", a), ("B", b)):
        for k in f.files:
            if k.endswith("_run2"):
                base = k[: -len("_run2")]
                if not np.array_equal(f[k].view(np.uint32), f[base].view(np.uint32)):
                    print(f"{name}: {base} NOT run-to-run stable")
                    bad += 1
    print("ALL EQUAL" if bad == 0 else f"{bad} DIFFERENCES")
    return bad


def dump(out_path, quick=False):
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "diffpose-nw_amd"))
    from diffpose_amd.data import synthetic_batch
    from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
    from diffpose_amd.gcnpose import HipGCNpose
    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict

    dev = torch.device("cuda", 0)
    res = {}

    def betas(T):
        return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                                  num_diffusion_timesteps=T)).float()

    m = HipGCNdiff(adj_mx_from_edges(), None, device=dev)
    m.load_state_dict(synthetic_state_dict())
    x_all = torch.from_numpy(synthetic_batch(1100, seed=5)[0]).to(dev)
    mk = torch.ones(1100, 1, 17, dtype=torch.bool)
    mk[1::3, 0, [2, 16]] = False
    mk = mk.to(dev)
    seq50 = make_seq("uniform", 50, 50)
    for mode in ("fp32", "f16x3", "bf16"):
        m.set_gemm_mode(mode)
        res[f"s1024_{mode}"] = m.sample(x_all[:1024], seq50, betas(51), mask=mk[:1024]).cpu().numpy()
        if mode != "fp32":
            res[f"s1024_{mode}_run2"] = m.sample(x_all[:1024], seq50, betas(51), mask=mk[:1024]).cpu().numpy()
        t = torch.arange(1024, device=dev, dtype=torch.float32) % 51
        res[f"eps_{mode}"] = m(x_all[:1024], mk[:1024], t).cpu().numpy()
    m.set_gemm_mode("bf16")
    res["s1024_bf16_k100"] = m.sample(x_all[:1024], make_seq("uniform", 100, 100), betas(101)).cpu().numpy()
    if not quick:
        for mode in ("fp32", "bf16"):
            m.set_gemm_mode(mode)
            res[f"s1100_{mode}"] = m.sample(x_all, seq50, betas(51), mask=mk).cpu().numpy()
            res[f"s1026_{mode}"] = m.sample(x_all[:1026], seq50, betas(51), mask=mk[:1026]).cpu().numpy()
    m.close()

    pm = HipGCNpose(adj_mx_from_edges(), None, device=dev)
    pm.load_state_dict(synthetic_state_dict(kind="pose"))
    res["pose"] = pm(x_all[:1024, :, :2].contiguous()).cpu().numpy()
    pm.close()

    if not quick:
        for hid, heads, layers in ((128, 8, 5), (128, 4, 3), (64, 2, 2), (64, 4, 5)):
            cfg = ns(model=ns(hid_dim=hid, emd_dim=hid, coords_dim=[5, 5], num_layer=layers, n_head=heads,
                              dropout=0.25, n_pts=17))
            w = HipGCNdiff(adj_mx_from_edges(), cfg, device=dev)
            w.load_state_dict(synthetic_state_dict(hid=hid, n_layers=layers))
            res[f"wide_h{hid}_n{heads}_l{layers}"] = w.sample(x_all[:512], seq50, betas(51), mask=mk[:512]).cpu().numpy()
            w.close()
    torch.cuda.synchronize()
    np.savez(out_path, **res)
    print(f"dumped {len(res)} arrays to {out_path} (DPK_LIB={os.environ.get('DPK_LIB', 'in-tree')})")


if __name__ == "__main__":
    if sys.argv[1] == "compare":
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
    dump(sys.argv[2], quick="--quick" in sys.argv)
