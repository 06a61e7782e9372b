"""GPU parity of the split-fp16 GEMM mode (dpk_set_gemm_mode(h, 1), HipGCNdiff.set_gemm_mode("f16x3")).

Mode 1 computes every per-layer GEMM product as a_hi*w_hi + a_hi*w_lo + a_lo*w_hi on f16 MFMA
(a = a_hi + a_lo, 64*w = w_hi + w_lo; fp32 accumulate), so it is held to the SAME bars as the
fp32 mode (test_gpu_parity.py): |eps - eps_ref| <= 5e-6, trajectories <= 5e-6 elementwise,
|MPJPE_hip - MPJPE_ref| <= 1e-4 mm at the bench config.  The CPU emulation of the scheme
(split-fp16 GEMM mode) gave max |d eps| 7.7e-7 and MPJPE delta 8.8e-7 mm.
"""
import numpy as np
import pytest
import torch

from conftest import record_delta

from diffpose_amd import utils_diff
from diffpose_amd.data import synthetic_batch
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.gcnpose import HipGCNpose
from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

EPS_TOL = 5e-6
TRAJ_TOL = 5e-6
MPJPE_TOL_MM = 1e-4


def _betas(T):
    return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                              num_diffusion_timesteps=T)).float()


def _maxdiff(a, b):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if torch.is_tensor(b) else np.asarray(b, np.float64)
    assert a.shape == b.shape
    return float(np.abs(a - b).max())


def _mpjpe_mm(out, targets):
    o = out.detach().cpu().double() if torch.is_tensor(out) else torch.from_numpy(np.asarray(out)).double()
    xyz = o[:, :, 2:] - o[:, :1, 2:]
    t = torch.from_numpy(np.asarray(targets)).double()
    return float(torch.mean(torch.norm(xyz - t, dim=-1)) * 1000.0)


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict())
    m.set_gemm_mode("f16x3")
    return m


@pytest.fixture(scope="module")
def mask():
    return torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0")


def test_eps_vs_golden(model, mask, golden):
    g = golden("g2_modules.npz")
    x = torch.from_numpy(g["x"]).cuda()
    t = torch.from_numpy(g["t"]).cuda()
    assert record_delta(_maxdiff(model(x, mask, t, 0), g["eps"]), EPS_TOL)
    m2 = torch.from_numpy(g["mask2"]).cuda()
    assert record_delta(_maxdiff(model(x, m2, t, 0), g["eps_masked"]), EPS_TOL)


def test_trajectory_vs_golden(model, mask, golden):
    g = golden("g3_traj_n64_k10.npz")
    x = torch.from_numpy(g["x"]).cuda()
    xs, x0s = utils_diff.generalized_steps(x, mask, [int(s) for s in g["seq"]], model, _betas(51).cuda(), eta=0.0)
    assert record_delta(_maxdiff(torch.stack(xs), g["xs"]), TRAJ_TOL)
    assert record_delta(_maxdiff(torch.stack(x0s), g["x0s"]), TRAJ_TOL)


@pytest.mark.parametrize("name", ["g4_final_n16_k50.npz", "g4_final_n16_k100_T101.npz", "g4_final_n8_quad.npz"])
def test_final_vs_golden(model, mask, golden, name):
    g = golden(name)
    out = model.sample(torch.from_numpy(g["x"]).cuda(), [int(s) for s in g["seq"]], _betas(int(g["T"])), mask=mask)
    assert record_delta(_maxdiff(out, g["out"]), TRAJ_TOL)
    assert record_delta(abs(_mpjpe_mm(out, g["targets"]) - _mpjpe_mm(g["out"], g["targets"])), MPJPE_TOL_MM)


def test_bench_config_vs_oracle_and_fp32(model, mask):
    """B=1024, K=50: f16x3 vs the golden-pinned CPU oracle and vs the fp32 mode."""
    from oracle import gcndiff_oracle as O

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    x, tgt = synthetic_batch(1024, seed=19960903)
    seq = make_seq("uniform", 50, 50)
    xd = torch.from_numpy(x).cuda()
    out = model.sample(xd, seq, _betas(51), mask=mask).clone()
    P = O.params_to_torch(synthetic_state_dict())
    xs, _ = O.generalized_steps(torch.from_numpy(x), torch.ones(1, 1, 17, dtype=torch.bool), seq,
                                lambda a, m, t: O.gcndiff_forward(P, O.adjacency(), a, m, t), _betas(51))
    ref = xs[-1]
    assert record_delta(_maxdiff(out, ref), TRAJ_TOL)
    assert record_delta(abs(_mpjpe_mm(out, tgt) - _mpjpe_mm(ref, tgt)), MPJPE_TOL_MM)
    model.set_gemm_mode("fp32")
    try:
        out32 = model.sample(xd, seq, _betas(51), mask=mask)
    finally:
        model.set_gemm_mode("f16x3")
    assert record_delta(_maxdiff(out, out32), TRAJ_TOL)
    out_again = model.sample(xd, seq, _betas(51), mask=mask)          # switching back is exact
    assert torch.equal(out_again, out)


@pytest.mark.parametrize("n", [1, 3, 5, 37])
def test_ragged_batches_are_batch_invariant(model, mask, n):
    x, _ = synthetic_batch(40, seed=7)
    xd = torch.from_numpy(x).cuda()
    seq = make_seq("uniform", 50, 10)
    full = model.sample(xd, seq, _betas(51), mask=mask)
    part = model.sample(xd[:n].contiguous(), seq, _betas(51), mask=mask)
    assert torch.equal(full[:n], part)


def test_dense_graph_path(mask):
    """An adjacency outside the compiled H36M Chebyshev pattern (dense graph path) vs the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from oracle import gcndiff_oracle as O
    from diffpose_amd.gcndiff import H36M_EDGES

    edges = tuple(H36M_EDGES) + ((3, 16), (6, 13))
    sd = synthetic_state_dict()
    m = HipGCNdiff(adj_mx_from_edges(17, edges), None, device="cuda:0")
    m.load_state_dict(sd)
    m.set_gemm_mode("f16x3")
    x, _ = synthetic_batch(9, seed=77)
    t = torch.tensor([49., 3., 17., 0., 8., 49., 22., 31., 5.])
    eps = m(torch.from_numpy(x).cuda(), mask, t.cuda(), 0)
    ref = O.gcndiff_forward(O.params_to_torch(sd), O.adjacency(17, edges), torch.from_numpy(x),
                            torch.ones(1, 1, 17, dtype=torch.bool), t)
    assert record_delta(_maxdiff(eps, ref), EPS_TOL)
    m.close()


def test_gcnpose_f16x3_vs_golden(golden):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = golden("g6_gcnpose.npz")
    m = HipGCNpose(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict(kind="pose"))
    m.set_gemm_mode("f16x3")
    xyz = m(torch.from_numpy(g["x2d"]).cuda(), torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0"))
    assert record_delta(_maxdiff(xyz, g["xyz"]), EPS_TOL)
    m.close()


def test_bad_gemm_mode_raises(model):
    with pytest.raises(ValueError):
        model.set_gemm_mode("tf32")


def test_out_of_range_weights_are_refused():
    """Weights outside the fp16 split range make f16x3 calls fail loudly; fp32 still runs."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from diffpose_amd._lib import DpkError

    sd = synthetic_state_dict()
    sd["atten_layers.2.self_attn.linears.1.weight"] = sd["atten_layers.2.self_attn.linears.1.weight"].copy()
    sd["atten_layers.2.self_attn.linears.1.weight"][3, 5] = 2000.0
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(sd)
    x, _ = synthetic_batch(4, seed=1)
    xd = torch.from_numpy(x).cuda()
    t = torch.full((4,), 10.0, device="cuda:0")
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0")
    m(xd, mask, t, 0)
    m.set_gemm_mode("f16x3")
    with pytest.raises(DpkError, match="UNSUPPORTED|split-fp16"):
        m(xd, mask, t, 0)
    m.close()
