"""GPU tolerance study of the bf16 GEMM mode (BASELINE config 3: human36m_diffpose_uvxyz_gt eval,
K=100 DDIM steps, T=101, bf16).  dpk_set_gemm_mode(h, 2) / HipGCNdiff.set_gemm_mode("bf16")
rounds the operands of the per-layer GEMMs and (round 5) of attention's score and P.V products to bf16
(8-bit mantissa) and accumulates in fp32; the GraphNet products take bf16 X against L_g as a bf16 hi + lo
pair (two products, L_g to ~16 bits); LayerNorm, the softmax, the I/O ChebConvs and the DDIM update stay
fp32.  (L_g rounded to bf16 alone measured +1.1 % at 30x the MPJPE delta, the hi + lo pair +1.4 % at 5.6x
on 128 frames, 3.8e-4 -> 2.1e-3 mm: DESIGN.md 4.2.)  Round 6 put joint 16's attention products and the
GEMM tail rows on the same bf16 MFMAs as the other joints (DESIGN.md 4.2 "Round 6").

It is a reduced-precision mode, so it is NOT held to the fp32 bar (MPJPE delta <= 1e-4 mm).
Measured on MI355X against the golden-pinned CPU oracle (tools/bf16_probe.py): one eps
evaluation max |d eps| 7.6e-3 (|eps| <= 1.46); finals after K=50 max |d| 8.6e-4 and MPJPE
delta 1.1e-3 mm; after K=100 (T=101) on the whole 1,024-frame batch (round 6) 1.09e-3 and 2.93e-3 mm,
the fp32 mode on the same frames 2.0e-6 and 9.0e-6 mm.  The bars below sit ~3x above those (bf16
rounding is deterministic, so they only guard against regressions), and the fp32 bar is asserted to
FAIL so the study keeps saying what it says.
"""
import numpy as np
import pytest
import torch

from conftest import record_delta
from diffpose_amd.data import synthetic_batch
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

EPS_TOL_BF16 = 2.5e-2          # max |eps_hip - eps_ref|, one evaluation
FINAL_TOL_BF16 = 4e-3          # max |x_hip - x_ref| after the whole loop
MPJPE_TOL_BF16_MM = 1e-2       # |MPJPE_hip - MPJPE_ref| on the 1,024 frames (measured 2.93e-3 mm)
MPJPE_FP32_BAR_MM = 1e-4       # the fp32 bar bf16 does not meet


def _betas(T):
    return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                              num_diffusion_timesteps=T)).float()


def _mpjpe_mm(out, targets):
    o = np.asarray(out, np.float64)
    xyz = o[:, :, 2:] - o[:, :1, 2:]
    return float(np.mean(np.linalg.norm(xyz - np.asarray(targets, np.float64), axis=-1)) * 1000.0)


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict())
    m.set_gemm_mode("bf16")
    return m


def test_eps_bf16_vs_golden(model, golden):
    g = golden("g2_modules.npz")
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0")
    eps = model(torch.from_numpy(g["x"]).cuda(), mask, torch.from_numpy(g["t"]).cuda(), 0).cpu().numpy()
    d = float(np.abs(eps - g["eps"]).max())
    assert np.isfinite(eps).all()
    assert 1e-5 < d <= EPS_TOL_BF16, d      # really reduced precision, within the study's bar


def test_config3_k100_vs_oracle(model):
    """BASELINE config 3's whole batch: K=100 over T'=100 (T=101), 1,024 frames, bf16 vs the CPU oracle,
    and fp32 vs the same oracle (the bench line's variants.config3_bf16.parity repeats this)."""
    from oracle import gcndiff_oracle as O

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    x, tgt = synthetic_batch(1024, seed=19960903)
    seq = make_seq("uniform", 100, 100)
    P = O.params_to_torch(synthetic_state_dict())
    xs, _ = O.generalized_steps(torch.from_numpy(x), torch.ones(1, 1, 17, dtype=torch.bool), seq,
                                lambda a, m, t: O.gcndiff_forward(P, O.adjacency(), a, m, t), _betas(101))
    ref = xs[-1].numpy()
    out = model.sample(torch.from_numpy(x).cuda(), seq, _betas(101)).cpu().numpy()
    d_mm = abs(_mpjpe_mm(out, tgt) - _mpjpe_mm(ref, tgt))
    assert record_delta(float(np.abs(out - ref).max()), FINAL_TOL_BF16)
    assert record_delta(d_mm, MPJPE_TOL_BF16_MM)
    assert d_mm > MPJPE_FP32_BAR_MM           # the study's finding: bf16 misses the fp32 bar
    model.set_gemm_mode("fp32")
    try:
        out32 = model.sample(torch.from_numpy(x).cuda(), seq, _betas(101)).cpu().numpy()
    finally:
        model.set_gemm_mode("bf16")
    assert record_delta(float(np.abs(out32 - ref).max()), 5e-6)
    assert record_delta(abs(_mpjpe_mm(out32, tgt) - _mpjpe_mm(ref, tgt)), MPJPE_FP32_BAR_MM)


@pytest.mark.parametrize("n", [1, 5, 37])
def test_bf16_ragged_batches_are_batch_invariant(model, n):
    x, _ = synthetic_batch(40, seed=7)
    xd = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    full = model.sample(xd, seq, _betas(51))
    part = model.sample(xd[:n].contiguous(), seq, _betas(51))
    assert torch.equal(full[:n], part)
