"""GPU: BASELINE config 4 — 8,192 synthetic H36M frames, K=50, batch-sharded over 8 GPUs — on the
HIP path of one GPU.  The 8 frame shards (data.shard_frames(8192, 8, r), 1,024 frames each, what
rank r of the 8-GPU run computes) run one after another on this GPU, are reassembled in
dist.shard_rows order, and must equal the unsharded 8,192-frame run bit for bit: every pose's result
depends only on its own workgroup tile, and each shard starts on a tile boundary.  Frames drawn
from every shard are checked against the golden-pinned oracle at the fp32 bars of
test_gpu_parity.py (elementwise 5e-6, MPJPE 1e-4 mm).
Reference: runners/diffpose_frame.py:126-127 (one DataParallel replica), :342 (hypothesis-major
rows), common/utils_diff.py:46-68 (the loop each rank runs)."""
import numpy as np
import pytest
import torch

from conftest import record_delta
from diffpose_amd import dist as D
from diffpose_amd.data import shard_frames, synthetic_batch
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

WORLD, FRAMES = 8, 8192


def _betas(T=51):
    return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                              num_diffusion_timesteps=T)).float()


def _mpjpe_mm(o, tgt):
    o = np.asarray(o, np.float64)
    xyz = o[:, :, 2:] - o[:, :1, 2:]
    return float(np.mean(np.linalg.norm(xyz - np.asarray(tgt, np.float64), axis=-1)) * 1000.0)


def test_config4_eight_shards_equal_unsharded_and_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from oracle import gcndiff_oracle as O

    x, tgt = synthetic_batch(FRAMES, seed=19960903)
    seq = make_seq("uniform", 50, 50)
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict())
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0")
    xd = torch.from_numpy(x).cuda()
    full = m.sample(xd, seq, _betas(), mask=mask)
    assembled = torch.empty_like(full)
    for r in range(WORLD):
        lo, hi = shard_frames(FRAMES, WORLD, r)
        assert hi - lo == FRAMES // WORLD
        part = m.sample(xd[lo:hi].contiguous(), seq, _betas(), mask=mask)
        assembled[D.shard_rows(FRAMES, 1, WORLD, r).cuda()] = part
    torch.cuda.synchronize()
    m.close()
    assert torch.equal(assembled, full)
    assert torch.isfinite(full).all()
    # 8 frames from each shard (its first, last and 6 spread between) against the oracle
    sel = np.concatenate([np.linspace(r * 1024, r * 1024 + 1023, 8).astype(np.int64) for r in range(WORLD)])
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    P, adj = O.params_to_torch(synthetic_state_dict()), O.adjacency()
    xs, _ = O.generalized_steps(torch.from_numpy(x[sel]), torch.ones(1, 1, 17, dtype=torch.bool), seq,
                                lambda a_, m_, t_: O.gcndiff_forward(P, adj, a_, m_, t_), _betas())
    ref = xs[-1].double().numpy()
    hip = full[torch.from_numpy(sel).cuda()].cpu().double().numpy()
    d = float(np.abs(hip - ref).max())
    dm = abs(_mpjpe_mm(hip, tgt[sel]) - _mpjpe_mm(ref, tgt[sel]))
    print(f"\nconfig 4: 8 shards of 1024 == unsharded 8192 bitwise; oracle on {sel.size} frames: "
          f"max|d| {d:.3e}, MPJPE d {dm:.3e} mm")
    assert record_delta(d, 5e-6)
    assert record_delta(dm, 1e-4)
