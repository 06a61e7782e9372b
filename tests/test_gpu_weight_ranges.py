"""GPU: the sampler on weight distributions other than the build's default generator
(verdict r01 "parity pinned on one weight distribution"):
  * g9: the reference's OWN initialisers (a freshly built reference GCNdiff under
    torch.manual_seed(0/1): xavier_normal_ Chebyshev weights, zero biases, identical attention
    projections, A_hat = I, models/ChebConv.py:62-67, models/gcndiff.py:70-98);
  * g10: the build's generator at a second seed (7).
Goldens are the reference's own K=50 finals in fp32 and in fp64; the reference's own fp32-vs-fp64
gap on the same weights and inputs is g = |out32 - out64| (elementwise max) and gm = |MPJPE32 -
MPJPE64| (mm).  Bars (verdict r02: set from what the kernel achieves, not from 10x the noise):
    elementwise  |hip - ref32| <= ELEM_TOL = 5e-6 (the achieved deltas are printed and kept in
                 profiles/r03_weight_ranges.txt; the old bar, max(2e-5, 10 g), was ~18x g)
    MPJPE        |hip - ref32| <= 1e-4 mm (the north-star bar) on every case, g9 seed 1 included,
                 although there the reference's own fp32-vs-fp64 gap (gm = 2.8e-4 mm) is above that
                 bar; its line also reports the 2 gm bar the round-2 test used.
Achieved on the MI355X (r03): final max|d| 6.0e-7 .. 9.0e-7, MPJPE d 2.9e-6 .. 1.9e-5 mm.
fp32 and the f16x3 GEMM mode are both held to these bars.
"""
import numpy as np
import pytest
import torch

from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.schedule import get_beta_schedule
from diffpose_amd.weights import reference_init_state_dict, synthetic_state_dict

pytestmark = pytest.mark.gpu

ELEM_TOL = 5e-6
CASES = ["g9_refinit_seed0.npz", "g9_refinit_seed1.npz", "g10_synth_seed7.npz"]


def _weights(name):
    if name.startswith("g9_refinit_seed"):
        return reference_init_state_dict(int(name[len("g9_refinit_seed"):].split(".")[0]))
    return synthetic_state_dict(seed=7)


def _mpjpe_mm(o, tgt):
    o = np.asarray(o, np.float64)
    xyz = o[:, :, 2:] - o[:, :1, 2:]
    return float(np.mean(np.linalg.norm(xyz - np.asarray(tgt, np.float64), axis=-1)) * 1000.0)


@pytest.mark.parametrize("gemm", ["fp32", "f16x3"])
@pytest.mark.parametrize("name", CASES)
def test_sampler_on_other_weights(golden, name, gemm):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = golden(name)
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(_weights(name))
    m.set_gemm_mode(gemm)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                           num_diffusion_timesteps=int(g["T"]))).float()
    x = torch.from_numpy(g["x"]).cuda()
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0")
    eps = m(x[:8].contiguous(), mask, torch.from_numpy(g["t8"]).cuda(), 0).cpu().numpy()
    assert np.abs(eps - g["eps"]).max() <= ELEM_TOL
    out = m.sample(x, [int(s) for s in g["seq"]], b, mask=mask).cpu().numpy()
    m.close()
    ref, ref64 = g["out"].astype(np.float64), g["out64"]
    gap = float(np.abs(ref - ref64).max())
    gap_mm = abs(_mpjpe_mm(ref, g["targets"]) - _mpjpe_mm(ref64, g["targets"]))
    d = float(np.abs(out - ref).max())
    dm = abs(_mpjpe_mm(out, g["targets"]) - _mpjpe_mm(ref, g["targets"]))
    de = float(np.abs(eps - g["eps"]).max())
    seed1 = name == "g9_refinit_seed1.npz"
    print(f"\nweight-range {name} {gemm}: eps max|d| {de:.3e}; K=50 final max|d| {d:.3e} (ref fp32-fp64 gap "
          f"{gap:.3e}); MPJPE d {dm:.3e} mm (ref gap {gap_mm:.3e} mm) -> 1e-4 mm bar "
          f"{'met' if dm <= 1e-4 else 'NOT met'}" + (f", 2*gap bar {2 * gap_mm:.3e} mm "
                                                       f"{'met' if dm <= 2 * gap_mm else 'NOT met'}" if seed1 else ""))
    assert d <= ELEM_TOL
    assert dm <= 1e-4


def test_f16x3_range_guard():
    """gemm mode f16x3 packs weights as x64 fp16 hi/lo pairs: a GEMM weight with |w| >= 1015 is
    refused (DPK_E_UNSUPPORTED) instead of overflowing, and fp32 mode still runs it."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from diffpose_amd._lib import DpkError

    sd = synthetic_state_dict()
    sd["atten_layers.2.feed_forward.gconv1.fc.weight"] = sd["atten_layers.2.feed_forward.gconv1.fc.weight"].copy()
    sd["atten_layers.2.feed_forward.gconv1.fc.weight"][3, 5] = 2000.0
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(sd)
    x = torch.zeros(4, 17, 5, device="cuda:0")
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                           num_diffusion_timesteps=51)).float()
    m.set_gemm_mode("f16x3")
    with pytest.raises(DpkError) as ei:
        m.sample(x, [0, 25], b)
    assert ei.value.code == -2
    m.set_gemm_mode("fp32")
    assert torch.isfinite(m.sample(x, [0, 25], b)).all()
    m.close()
