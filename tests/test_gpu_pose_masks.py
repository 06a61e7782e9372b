"""Per-pose attention key masks: the reference's ``scores.masked_fill(mask == 0, -1e9)`` with a
[N,1,17] mask broadcast over heads and queries (models/GraFormer.py:107-108, ``mask.unsqueeze(1)``),
through dpk_set_pose_masks.

  * vs the golden-pinned oracle (the same masked_fill on the same per-pose mask): one denoiser
    call within EPS_TOL, a K=10 DDIM trajectory's final x within TRAJ_TOL (the bars of
    test_gpu_parity.py);
  * bitwise: each pose of a per-pose-masked batch equals the same pose of a batch run with its
    mask as the handle-wide one (same launch geometry, only the mask's source differs);
  * a batch whose size differs from the mask's is rejected (Python: ValueError, C ABI:
    DPK_E_INVALID), and a later (1,1,17) mask restores the handle-wide path.
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import record_delta

from diffpose_amd import _lib
from diffpose_amd.data import synthetic_batch
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

EPS_TOL = 5e-6
TRAJ_TOL = 5e-6


def _betas(T):
    return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                              num_diffusion_timesteps=T)).float()


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict())
    return m


def _masks(n, seed=5):
    """n key masks: all ones, single keys, the root only dropped, and random patterns (every
    mask keeps at least one key, as a softmax row needs)."""
    rng = np.random.default_rng(seed)
    m = rng.random((n, 1, 17)) < 0.6
    m[0] = True
    m[1] = False
    m[1, 0, 16] = True          # key 16 alone (the VALU border key)
    m[2] = False
    m[2, 0, 3] = True           # one MFMA key alone
    m[3] = True
    m[3, 0, 0] = False
    for i in range(n):
        if not m[i].any():
            m[i, 0, i % 17] = True
    return torch.from_numpy(m)


def _maxdiff(a, b):
    return float((a.detach().cpu().double() - b.detach().cpu().double()).abs().max())


def test_eps_per_pose_masks_vs_oracle(model):
    from oracle import gcndiff_oracle as O

    n = 12
    x, _ = synthetic_batch(n, seed=21)
    x = torch.from_numpy(x)
    t = torch.arange(n, dtype=torch.float32) * 4.0
    m = _masks(n)
    eps = model(x.cuda(), m.cuda(), t.cuda(), 0)
    ref = O.gcndiff_forward(O.params_to_torch(synthetic_state_dict()), O.adjacency(), x, m, t)
    assert record_delta(_maxdiff(eps, ref), EPS_TOL)
    # the masks matter: the all-ones run differs for the masked poses
    ones = model(x.cuda(), torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0"), t.cuda(), 0)
    assert _maxdiff(ones[1:3], eps[1:3]) > 1e-3
    assert torch.equal(ones[0], eps[0])


def test_sample_per_pose_masks_vs_oracle(model):
    from oracle import gcndiff_oracle as O

    n = 16
    x, _ = synthetic_batch(n, seed=22)
    x = torch.from_numpy(x)
    seq = make_seq("uniform", 50, 10)
    m = _masks(n, seed=9)
    out = model.sample(x.cuda(), seq, _betas(51), mask=m.cuda())
    P = O.params_to_torch(synthetic_state_dict())
    adj = O.adjacency()
    xs, _ = O.generalized_steps(x, m, seq, lambda a, mm, tt: O.gcndiff_forward(P, adj, a, mm, tt), _betas(51))
    assert record_delta(_maxdiff(out, xs[-1]), TRAJ_TOL)


def test_per_pose_masks_bitwise_vs_handle_mask(model):
    """Two mask patterns alternating over 64 poses: each pose equals the same pose of the batch
    run with its pattern as the handle-wide mask."""
    n = 64
    x, _ = synthetic_batch(n, seed=23)
    x = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    a = torch.ones(1, 1, 17, dtype=torch.bool)
    b = torch.ones(1, 1, 17, dtype=torch.bool)
    b[0, 0, [0, 5, 16]] = False
    per = torch.where((torch.arange(n) % 2 == 0).view(n, 1, 1), a, b).cuda()
    out = model.sample(x, seq, _betas(51), mask=per)
    out_a = model.sample(x, seq, _betas(51), mask=a.cuda())
    out_b = model.sample(x, seq, _betas(51), mask=b.cuda())
    assert torch.equal(out[0::2], out_a[0::2])
    assert torch.equal(out[1::2], out_b[1::2])
    assert not torch.equal(out_a[1::2], out_b[1::2])


def test_per_pose_mask_batch_checks(model):
    x, _ = synthetic_batch(8, seed=24)
    x = torch.from_numpy(x).cuda()
    t = torch.full((8,), 7.0, device="cuda:0")
    with pytest.raises(ValueError):
        model(x, _masks(4).cuda(), t, 0)
    with pytest.raises(ValueError):
        model(x, torch.ones(8, 17, 17, dtype=torch.bool, device="cuda:0"), t, 0)
    # C ABI: masks for 4 poses, a launch of 8
    bits = torch.full((4,), (1 << 17) - 1, dtype=torch.int32, device="cuda:0")
    L = _lib.lib()
    assert L.dpk_set_pose_masks(model._h, bits.data_ptr(), 4) == 0
    eps = torch.empty_like(x)
    stream = torch.cuda.current_stream().cuda_stream
    rc = L.dpk_eps(model._h, x.data_ptr(), t.data_ptr(), eps.data_ptr(), 8, stream)
    assert rc == -1 and b"dpk_set_pose_masks covers 4" in L.dpk_last_error(model._h)
    assert L.dpk_set_pose_masks(model._h, None, 0) == 0
    model._pose_bits = None
    model._mask_key = model._mask_ref = None
    # back on the handle-wide mask: equal to a fresh all-ones run
    ones = torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0")
    e1 = model(x, _masks(8).cuda(), t, 0)
    e2 = model(x, ones, t, 0)
    e3 = model(x, None, t, 0)
    assert torch.equal(e2, e3) and not torch.equal(e1, e2)


def test_gcnpose_per_pose_masks_vs_oracle():
    """GCNpose.forward(x, mask) with a [N,1,17] mask (dpk_pose reads the same per-pose words)."""
    from oracle import gcndiff_oracle as O
    from diffpose_amd.gcnpose import HipGCNpose

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    pm = HipGCNpose(adj_mx_from_edges(), None, device="cuda:0")
    pm.load_state_dict(synthetic_state_dict(kind="pose"))
    n = 10
    x, _ = synthetic_batch(n, seed=25)
    x2d = torch.from_numpy(np.ascontiguousarray(x[:, :, :2]))
    m = _masks(n, seed=13)
    xyz = pm(x2d.cuda(), m.cuda())
    ref = O.gcnpose_forward(O.params_to_torch(synthetic_state_dict(kind="pose")), O.adjacency(), x2d, m)
    assert record_delta(_maxdiff(xyz, ref), 5e-6)          # POSE_TOL of test_gpu_pose_metrics.py
    ones = pm(x2d.cuda(), torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0"))
    assert torch.equal(ones[0], xyz[0]) and _maxdiff(ones[1:3], xyz[1:3]) > 1e-4
    with pytest.raises(ValueError):
        pm(x2d.cuda(), _masks(4).cuda())


@pytest.mark.parametrize("mode", ["eps", "sample"])
def test_per_pose_masks_both_tile_sizes(model, mode):
    """N = 1,100 poses: one full round of 4-pose workgroups (poses 0..1023, the 4-pose kernel's
    mask word wave / (NW/P) with pose_off 0) and a tail of 76 poses, in 2-pose workgroups (eps
    mode, and sample mode under the "two_pose" plan: the second launch, pose_off 1024) or, in
    sample mode's default "step_split" plan, in 19 4-pose tiles whose steps run as two halves on
    two workgroups (blocks numbered apart from their tiles).  Four mask patterns in an irregular
    order: every pose equals the same pose of the batch run with its pattern as the handle-wide
    mask, bitwise (same launch geometry, only the mask's source differs)."""
    n = 1100
    x, _ = synthetic_batch(n, seed=26)
    x = torch.from_numpy(x).cuda()
    pats = torch.ones(4, 1, 17, dtype=torch.bool)
    pats[1, 0, [0, 5, 16]] = False
    pats[2, 0, :16] = False                    # key 16 alone
    pats[3, 0, 1::2] = False
    which = torch.from_numpy((np.arange(n) * 7 + np.arange(n) // 5) % 4)
    per = pats[which].cuda()
    t = (torch.arange(n, dtype=torch.float32) % 50).cuda()
    seq = make_seq("uniform", 50, 10)

    def run(mask):
        if mode == "eps":
            return model(x, mask, t, 0)
        return model.sample(x, seq, _betas(51), mask=mask)

    for plan in (["step_split", "two_pose"] if mode == "sample" else ["step_split"]):
        model.set_tail_plan(plan)
        try:
            out = run(per)
            for k in range(4):
                ref = run(pats[k : k + 1].cuda())
                sel = (which == k).nonzero().flatten().cuda()
                assert torch.equal(out[sel], ref[sel]), (mode, plan, k)
        finally:
            model.set_tail_plan("step_split")
    head = (which[:1024] == 2).nonzero().flatten()
    tail = 1024 + (which[1024:] == 2).nonzero().flatten()
    assert head.numel() > 0 and tail.numel() > 0   # the key-16-alone pattern lands in both tile sizes


def test_per_pose_masks_under_graph_capture(model):
    """A captured sampler keeps reading the per-pose mask array it was captured with: replacing
    the mask afterwards (and churning the caching allocator) does not change the replay."""
    n = 40
    x, _ = synthetic_batch(n, seed=27)
    x = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    m1 = _masks(n, seed=31).cuda()
    m2 = _masks(n, seed=32).cuda()
    ref1 = model.sample(x, seq, _betas(51), mask=m1).clone()
    ref2 = model.sample(x, seq, _betas(51), mask=m2).clone()
    assert not torch.equal(ref1, ref2)
    out = torch.empty_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        model.sample(x, seq, _betas(51), mask=m1, out=out)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        model.sample(x, seq, _betas(51), mask=m1, out=out)
    assert torch.equal(model.sample(x, seq, _betas(51), mask=m2), ref2)    # a new mask array bound
    junk = [torch.zeros(n, dtype=torch.int32, device="cuda:0") for _ in range(64)]   # reuse bait
    for _ in range(2):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref1)
    del junk, g
