"""GPU: a GCNdiff built with num_layer < 5 (the config value is a run-time layer count of the
kernels; models/gcndiff.py:63-90 builds num_layer GraAttenLayer/_ResChebGC_diff pairs) matches
the golden-pinned oracle run with the same layer count.  Tolerances as test_gpu_parity.py."""
from types import SimpleNamespace

import pytest
import torch

from conftest import record_delta

from diffpose_amd.data import synthetic_batch
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

EPS_TOL = 5e-6
TRAJ_TOL = 5e-6


def _cfg(nl):
    return SimpleNamespace(model=SimpleNamespace(hid_dim=96, num_layer=nl, n_head=4, n_pts=17, coords_dim=[5, 5]))


@pytest.mark.parametrize("nl", [1, 3])
def test_num_layer_eps_and_sample_vs_oracle(nl):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from oracle import gcndiff_oracle as O

    sd = synthetic_state_dict(n_layers=nl)
    m = HipGCNdiff(adj_mx_from_edges(), _cfg(nl), device="cuda:0")
    m.load_state_dict(sd)
    with pytest.raises(KeyError):                 # a 5-layer state_dict does not fit a 3-layer model
        HipGCNdiff(adj_mx_from_edges(), _cfg(nl), device="cuda:0").load_state_dict(synthetic_state_dict())
    P, adj = O.params_to_torch(sd), O.adjacency()
    mask = torch.ones(1, 1, 17, dtype=torch.bool)
    x, _ = synthetic_batch(37, seed=21)
    t = (torch.arange(37) % 50).float()
    eps = m(torch.from_numpy(x).cuda(), mask.cuda(), t.cuda(), 0).cpu()
    ref = O.gcndiff_forward(P, adj, torch.from_numpy(x), mask, t, n_layers=nl)
    assert record_delta((eps - ref).abs().max().item(), EPS_TOL)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                           num_diffusion_timesteps=51)).float()
    seq = make_seq("uniform", 50, 10)
    out = m.sample(torch.from_numpy(x).cuda(), seq, b).cpu()
    xs, _ = O.generalized_steps(torch.from_numpy(x), mask, seq,
                                lambda a_, m_, t_: O.gcndiff_forward(P, adj, a_, m_, t_, n_layers=nl), b)
    assert record_delta((out - xs[-1]).abs().max().item(), TRAJ_TOL)
    m.close()
