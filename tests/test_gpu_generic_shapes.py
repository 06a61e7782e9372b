"""GPU: GCNdiff / GCNpose at model shapes other than the compiled one (hid_dim 96, n_head 4,
n_pts 17), which run on the generic-shape path (csrc/dpk_generic.inc) — per-op launches, or for hid 128 /
8 or 4 heads and hid 64 / 2 or 4 heads on 17 joints the persistent-sampler instances (dpk_genfused.inc).
The reference builds its models from any config (models/gcndiff.py:55-99, models/gcnpose.py:55-98).
Round 6: fixtures produced by the reference itself at five such shapes (tests/golden/g12_*, from
tools/gen_goldens.py) pin both paths directly (test_shapes_vs_reference_goldens), and the oracle is
bit-exact on them (tests/test_oracle_golden.py::test_other_shapes_vs_reference); the other tests here
use the oracle as the checker on further inputs (per-pose masks, eta > 0, dense graphs, GCNpose).

Tolerances as tests/test_gpu_parity.py: 5e-6 elementwise for eps and trajectories (fp32 sums in
another order).
"""
import os
from types import SimpleNamespace as ns

import numpy as np
import pytest
import torch

from conftest import record_delta

from diffpose_amd.data import synthetic_batch
from diffpose_amd.gcndiff import H36M_EDGES, HipGCNdiff, adj_mx_from_edges
from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

TOL = 5e-6
CHAIN16 = tuple((i, i + 1) for i in range(15))


def _betas(T=51):
    return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                              num_diffusion_timesteps=T)).float()


def _cfg(hid, heads, layers, npts, coords=(5, 5)):
    return ns(model=ns(hid_dim=hid, emd_dim=hid, coords_dim=list(coords), num_layer=layers, n_head=heads,
                       dropout=0.25, n_pts=npts))


def _maxdiff(a, b):
    return float((a.detach().cpu().double() - b.detach().cpu().double()).abs().max())


def _inputs(n, npts, seed):
    x, _ = synthetic_batch(n, seed=seed)
    x = torch.from_numpy(x)
    if npts != 17:
        x = x[:, :npts].contiguous()
    return x


SHAPES = [
    (64, 2, 2, 17, H36M_EDGES),     # narrower, fewer heads and layers, the H36M skeleton
    (128, 8, 3, 17, H36M_EDGES),    # wider, more heads
    (48, 4, 1, 16, CHAIN16),        # another skeleton: a 16-joint chain
]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("hid,heads,layers,npts,edges", SHAPES)
def test_generic_eps_and_sample_vs_oracle(dev, monkeypatch, hid, heads, layers, npts, edges, fused):
    """fused "1": hid 128 / 8 heads and hid 64 / 2 heads on 17 joints run a persistent-sampler instance
    (dpkw, dpkn; round 5), the 16-joint chain the per-op path; "0" (DPK_GEN_FUSED=0): all per-op."""
    from oracle import gcndiff_oracle as O

    monkeypatch.setenv("DPK_GEN_FUSED", fused)
    sd = synthetic_state_dict(hid=hid, n_layers=layers, n_pts=npts)
    adj = adj_mx_from_edges(npts, edges)
    m = HipGCNdiff(adj, _cfg(hid, heads, layers, npts), device=dev)
    m.load_state_dict(sd)
    P = O.params_to_torch(sd)
    g = torch.from_numpy(adj)
    fwd = lambda a, mk, t: O.gcndiff_forward(P, g, a, mk, t, n_layers=layers, heads=heads)  # noqa: E731
    x = _inputs(24, npts, seed=40 + hid)
    t = torch.arange(24, dtype=torch.float32) * 2.0
    ones = torch.ones(1, 1, npts, dtype=torch.bool)
    eps = m(x.to(dev), ones.to(dev), t.to(dev), 0)
    ref = fwd(x, ones, t)
    assert eps.shape == ref.shape and record_delta(_maxdiff(eps, ref), TOL)
    # a handle-wide key mask and per-pose masks (the reference's masked_fill broadcast)
    mk = ones.clone()
    mk[0, 0, [0, npts - 1]] = False
    assert record_delta(_maxdiff(m(x.to(dev), mk.to(dev), t.to(dev), 0), fwd(x, mk, t)), TOL)
    per = torch.ones(24, 1, npts, dtype=torch.bool)
    per[::3, 0, 1::2] = False
    per[1::5, 0, :npts - 1] = False
    assert record_delta(_maxdiff(m(x.to(dev), per.to(dev), t.to(dev), 0), fwd(x, per, t)), TOL)
    # the K=10 sampler with its trajectory
    seq = make_seq("uniform", 50, 10)
    xs, x0s = m.sample(x.to(dev), seq, _betas(), mask=ones.to(dev), trajectory=True)
    rxs, rx0s = O.generalized_steps(x, ones, seq, fwd, _betas())
    assert record_delta(_maxdiff(xs, torch.stack(rxs)), TOL) and record_delta(_maxdiff(x0s, torch.stack(rx0s)), TOL)
    out = m.sample(x.to(dev), seq, _betas(), mask=ones.to(dev))
    assert torch.equal(out, xs[-1])
    m.close()


def test_generic_path_matches_fused_at_the_compiled_shape(dev):
    """DPK_FORCE_GENERIC=1 puts the compiled shape on the generic path: it agrees with the fused
    sampler within the fp32 bars (different summation orders), on 64 poses at K=50."""
    x = _inputs(64, 17, seed=50).to(dev)
    seq = make_seq("uniform", 50, 50)
    fused = HipGCNdiff(adj_mx_from_edges(), None, device=dev)
    fused.load_state_dict(synthetic_state_dict())
    os.environ["DPK_FORCE_GENERIC"] = "1"
    try:
        gen = HipGCNdiff(adj_mx_from_edges(), None, device=dev)
    finally:
        del os.environ["DPK_FORCE_GENERIC"]
    gen.load_state_dict(synthetic_state_dict())
    a = fused.sample(x, seq, _betas())
    b = gen.sample(x, seq, _betas())
    assert record_delta(_maxdiff(a, b), TOL)
    # eta > 0: both paths draw the same counter-based noise, keyed by (seed, step, element)
    seq10 = make_seq("uniform", 50, 10)
    a = fused.sample(x, seq10, _betas(), eta=0.5, seed=7)
    b = gen.sample(x, seq10, _betas(), eta=0.5, seed=7)
    assert record_delta(_maxdiff(a, b), TOL)
    assert _maxdiff(a, fused.sample(x, seq10, _betas(), eta=0.5, seed=8)) > 1e-3
    with pytest.raises(RuntimeError):
        gen.set_gemm_mode("f16x3")
        gen.sample(x, seq, _betas())
    fused.close()
    gen.close()


def test_generic_gcnpose_vs_oracle(dev):
    from diffpose_amd.gcnpose import HipGCNpose
    from oracle import gcndiff_oracle as O

    hid, heads, layers = 64, 2, 2
    sd = synthetic_state_dict(kind="pose", hid=hid, n_layers=layers)
    m = HipGCNpose(adj_mx_from_edges(), _cfg(hid, heads, layers, 17, coords=(2, 3)), device=dev)
    m.load_state_dict(sd)
    x2d = _inputs(20, 17, seed=60)[:, :, :2].contiguous()
    ones = torch.ones(1, 1, 17, dtype=torch.bool)
    xyz = m(x2d.to(dev), ones.to(dev))
    ref = O.gcnpose_forward(O.params_to_torch(sd), O.adjacency(), x2d, ones, n_layers=layers, heads=heads)
    assert record_delta(_maxdiff(xyz, ref), TOL)
    uv = m.uvxyz(x2d.to(dev), ones.to(dev), test_times=3, root_mode="quirk")
    assert record_delta(_maxdiff(uv, O.build_uvxyz(x2d, ref, 3, "quirk")), TOL)
    m.close()


@pytest.mark.parametrize("fused", ["0", "1"])
def test_generic_path_under_caller_capture(dev, monkeypatch, fused):
    """A caller's torch.cuda.graph around the generic path (config 5's pattern, common/utils_diff.py:46-68
    called from runners/diffpose_frame.py:365): the launches are recorded into the caller's graph on the
    capture's own scratch (the model's spare, sized by the uncaptured warm-up), and every replay is
    bitwise the eager result, for dpk_sample (K=4), dpk_eps and a captured loop of two samples on one
    stream; the scratch returns to the spare when the graph is destroyed.  fused "0": the per-op
    launches (DPK_GEN_FUSED=0); "1": the hid-64 persistent-sampler instance (dpkn)."""
    monkeypatch.setenv("DPK_GEN_FUSED", fused)
    hid, heads, layers = 64, 2, 2
    m = HipGCNdiff(adj_mx_from_edges(), _cfg(hid, heads, layers, 17), device=dev)
    m.load_state_dict(synthetic_state_dict(hid=hid, n_layers=layers))
    ones = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    x = _inputs(24, 17, seed=70).to(dev)
    t = (torch.arange(24, dtype=torch.float32) * 2.0).to(dev)
    seq = make_seq("uniform", 50, 4)
    eager = m.sample(x, seq, _betas(), mask=ones).clone()
    eps_eager = m(x, ones, t, 0).clone()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):                 # warm-up on the capture's side stream (torch's pattern)
        m.sample(x, seq, _betas(), mask=ones)
        m(x, ones, t, 0)
    torch.cuda.current_stream(dev).wait_stream(s)
    spare0 = m.debug_resources()["generic_spare_kib"]
    assert spare0 > 0, "the uncaptured warm-up reserves the capture's scratch"
    out = torch.empty_like(x)
    out2 = torch.empty_like(x)
    eps = torch.empty_like(x)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.sample(x, seq, _betas(), mask=ones, out=out)
        m.sample(out, seq, _betas(), mask=ones, out=out2)      # a captured loop: the second shares the scratch
        eps.copy_(m(x, ones, t, 0))
    assert m.debug_resources()["captures"] >= 1
    second = m.sample(eager, seq, _betas(), mask=ones).clone()
    for _ in range(2):
        out.zero_()
        out2.zero_()
        eps.zero_()
        g.replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(out, eager) and torch.equal(out2, second) and torch.equal(eps, eps_eager)
    del g
    import gc

    gc.collect()
    torch.cuda.synchronize(dev)
    m.sample(x, seq, _betas(), mask=ones)       # an uncaptured call recycles the capture's resources
    r = m.debug_resources()
    assert r["released"] == 0 and r["generic_spare_kib"] >= spare0   # the capture's scratch came back
    m.close()


@pytest.mark.parametrize("fused", ["0", "1"])
def test_generic_capture_without_warmup_is_refused(dev, monkeypatch, fused):
    monkeypatch.setenv("DPK_GEN_FUSED", fused)
    m = HipGCNdiff(adj_mx_from_edges(), _cfg(64, 2, 1, 17), device=dev)
    m.load_state_dict(synthetic_state_dict(hid=64, n_layers=1))
    x = _inputs(8, 17, seed=70).to(dev)
    seq = make_seq("uniform", 50, 2)
    m.set_schedule(seq, _betas())
    g = torch.cuda.CUDAGraph()
    with pytest.raises(Exception):
        with torch.cuda.graph(g):
            m.sample(x, seq, _betas())          # no uncaptured call has sized the spare
    m.close()


def test_generic_eta0_seed_shares_one_loop_graph(dev, monkeypatch):
    """advisor r04: at eta = 0 the seed is not read, so calls that differ only in seed (test_hyber
    passes seed + i per batch) replay one recorded loop instead of recording one each; at eta > 0
    the seed keys the graph (the counter-based draws depend on it).  (Per-op path: DPK_GEN_FUSED=0.)"""
    monkeypatch.setenv("DPK_GEN_FUSED", "0")
    m = HipGCNdiff(adj_mx_from_edges(), _cfg(64, 2, 1, 17), device=dev)
    m.load_state_dict(synthetic_state_dict(hid=64, n_layers=1))
    ones = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    x = _inputs(16, 17, seed=72).to(dev)
    seq = make_seq("uniform", 50, 5)
    a = m.sample(x, seq, _betas(), mask=ones, seed=1).clone()
    n0 = m.debug_resources()["generic_loop_graphs"]
    for sd in range(2, 12):
        assert torch.equal(m.sample(x, seq, _betas(), mask=ones, seed=sd), a)
    assert m.debug_resources()["generic_loop_graphs"] == n0 == 1
    m.sample(x, seq, _betas(), mask=ones, eta=0.5, seed=1)
    m.sample(x, seq, _betas(), mask=ones, eta=0.5, seed=2)
    assert m.debug_resources()["generic_loop_graphs"] == 3
    m.close()


def test_generic_default_mask_and_wide_input_through_c_abi(dev):
    """advisor r03: a generic-shape handle's default key mask covers all n_pts joints (here 21,
    GraFormer's default joint count) without any dpk_set_mask call — plain C callers get the
    all-ones src_mask the header promises — and an input ChebConv wider than the hidden width
    (coords 9 -> 9 on hid 8: the Chebyshev operand of the input, 27 floats a row, fits its scratch)
    computes the oracle's eps.  Driven through the C ABI directly (the Python wrapper always sets
    the mask)."""
    import ctypes

    from diffpose_amd import _lib
    from oracle import gcndiff_oracle as O

    L = _lib.lib()
    for hid, heads, npts, coords in ((32, 4, 21, 5), (8, 2, 17, 9)):
        edges = tuple((i, i + 1) for i in range(npts - 1))
        sd = synthetic_state_dict(hid=hid, n_layers=2, n_pts=npts, coords=(coords, coords))
        adj = adj_mx_from_edges(npts, edges)
        m = HipGCNdiff(adj, _cfg(hid, heads, 2, npts, coords=(coords, coords)), device=dev)
        m.load_state_dict(sd)
        n = 12
        x = torch.randn(n, npts, coords, generator=torch.Generator().manual_seed(hid))
        t = torch.arange(n, dtype=torch.float32) * 4.0
        xd, td = x.to(dev).contiguous(), t.to(dev).contiguous()
        eps = torch.empty_like(xd)
        rc = L.dpk_eps(m._h, xd.data_ptr(), td.data_ptr(), eps.data_ptr(), n,
                       torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(m._h, "dpk_eps", rc)
        P = O.params_to_torch(sd)
        ref = O.gcndiff_forward(P, torch.from_numpy(adj), x, torch.ones(1, 1, npts, dtype=torch.bool), t,
                                n_layers=2, heads=heads)
        assert record_delta(_maxdiff(eps, ref), TOL)
        m.close()


def test_generic_loop_graph_matches_direct_launches(dev, monkeypatch):
    """The generic path records its K-step loop as one hipGraph (keyed by stream scratch, schedule,
    batch size, mask and seed) and replays it: bitwise the directly launched loop (DPK_GEN_GRAPH=0),
    across a new key after every change — a per-pose mask, another schedule, a larger batch (the
    scratch grows, the graphs over the old buffer are dropped), eta > 0 with another seed — and when
    an earlier key comes back.  (Per-op path: DPK_GEN_FUSED=0.)"""
    monkeypatch.setenv("DPK_GEN_FUSED", "0")
    hid, heads, layers = 64, 2, 2
    sd = synthetic_state_dict(hid=hid, n_layers=layers)
    m = HipGCNdiff(adj_mx_from_edges(), _cfg(hid, heads, layers, 17), device=dev)
    m.load_state_dict(sd)
    ones = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    per = torch.ones(40, 1, 17, dtype=torch.bool, device=dev)
    per[::4, 0, 3:9] = False
    x40 = _inputs(40, 17, seed=70).to(dev)
    x90 = _inputs(90, 17, seed=71).to(dev)
    cases = [(x40, make_seq("uniform", 50, 10), ones, 0.0, 0), (x40, make_seq("uniform", 50, 10), per, 0.0, 0),
             (x40, make_seq("uniform", 50, 5), ones, 0.0, 0), (x90, make_seq("uniform", 50, 10), ones, 0.0, 0),
             (x40, make_seq("uniform", 50, 10), ones, 0.0, 0), (x40, make_seq("uniform", 50, 10), ones, 0.4, 3),
             (x40, make_seq("uniform", 50, 10), ones, 0.4, 4)]
    for x, seq, mk, eta, seed in cases:
        monkeypatch.setenv("DPK_GEN_GRAPH", "1")
        a = m.sample(x, seq, _betas(), eta=eta, mask=mk, seed=seed).clone()
        a2 = m.sample(x, seq, _betas(), eta=eta, mask=mk, seed=seed).clone()      # replay of the same graph
        monkeypatch.setenv("DPK_GEN_GRAPH", "0")
        b = m.sample(x, seq, _betas(), eta=eta, mask=mk, seed=seed)
        assert torch.equal(a, b) and torch.equal(a2, b), (x.shape[0], len(seq), eta, seed)
    m.close()


@pytest.mark.parametrize("fused", ["0", "1"])
def test_generic_eta_with_caller_noise_vs_oracle(dev, monkeypatch, fused):
    """eta > 0 on the generic path with the caller's draws (dpk_sample_noise; the launches go
    straight to the stream, the recorded loop only covers eta's counter-based draws): the K=10
    trajectory equals the oracle's run on the same draws within the bar."""
    from oracle import gcndiff_oracle as O

    monkeypatch.setenv("DPK_GEN_FUSED", fused)
    hid, heads, layers = 64, 2, 2
    sd = synthetic_state_dict(hid=hid, n_layers=layers)
    adj = adj_mx_from_edges()
    m = HipGCNdiff(adj, _cfg(hid, heads, layers, 17), device=dev)
    m.load_state_dict(sd)
    x = _inputs(20, 17, seed=81)
    seq = make_seq("uniform", 50, 10)
    z = torch.randn((10,) + tuple(x.shape), generator=torch.Generator().manual_seed(8))
    ones = torch.ones(1, 1, 17, dtype=torch.bool)
    xs, _ = m.sample(x.to(dev), seq, _betas(), eta=0.6, mask=ones.to(dev), trajectory=True, noise=z.to(dev))
    P = O.params_to_torch(sd)
    fwd = lambda a, mk, t: O.gcndiff_forward(P, torch.from_numpy(adj), a, mk, t, n_layers=layers, heads=heads)  # noqa: E731
    rxs, _ = O.generalized_steps(x, ones, seq, fwd, _betas(), eta=0.6, noise=z)
    assert record_delta(_maxdiff(xs, torch.stack(rxs)), TOL)
    m.close()


@pytest.mark.parametrize("hid,heads", [(128, 8), (128, 4), (64, 2), (64, 4)])
def test_fused_wide_sampler_matches_per_op_path(dev, monkeypatch, hid, heads):
    """hid 128 / 8 or 4 heads and hid 64 / 2 or 4 heads on 17 joints run the persistent sampler compiled
    at that width (dpkw, dpkw4: 2-pose tiles, d_k 16 / 32; dpkn, dpkn4: 4-pose tiles, d_k 32 / 16; round 5)
    instead of the per-op launches: eps (handle-wide and per-pose masks), the K=10 trajectory, eta > 0 with the caller's
    draws, a dense (non-H36M) adjacency and 2 and 5 layers agree with the per-op path (DPK_GEN_FUSED=0)
    and the oracle within the fp32 bars."""
    from oracle import gcndiff_oracle as O

    x = _inputs(37, 17, seed=91)
    t = torch.arange(37, dtype=torch.float32) * 1.5
    ones = torch.ones(1, 1, 17, dtype=torch.bool)
    per = torch.ones(37, 1, 17, dtype=torch.bool)
    per[::3, 0, 2::3] = False
    seq = make_seq("uniform", 50, 10)
    z = torch.randn((10,) + tuple(x.shape), generator=torch.Generator().manual_seed(5))
    rng = np.random.default_rng(3)
    dense = adj_mx_from_edges() + 0.1 * (rng.random((17, 17)) > 0.6)
    dense = ((dense + dense.T) / 2).astype(np.float32)
    for layers, adj in ((5, adj_mx_from_edges()), (2, dense)):
        sd = synthetic_state_dict(hid=hid, n_layers=layers)
        res = {}
        for fused in ("1", "0"):
            monkeypatch.setenv("DPK_GEN_FUSED", fused)
            m = HipGCNdiff(adj, _cfg(hid, heads, layers, 17), device=dev)
            m.load_state_dict(sd)
            res[fused] = (m(x.to(dev), ones.to(dev), t.to(dev), 0), m(x.to(dev), per.to(dev), t.to(dev), 0),
                          m.sample(x.to(dev), seq, _betas(), mask=ones.to(dev), trajectory=True)[0],
                          m.sample(x.to(dev), seq, _betas(), eta=0.7, mask=ones.to(dev), noise=z.to(dev)))
            m.close()
        for a, b in zip(res["1"], res["0"]):
            assert record_delta(_maxdiff(a, b), TOL)
        P = O.params_to_torch(sd)
        fwd = lambda a, mk, tt: O.gcndiff_forward(P, torch.from_numpy(adj), a, mk, tt, n_layers=layers, heads=heads)  # noqa: E731
        assert record_delta(_maxdiff(res["1"][0], fwd(x, ones, t)), TOL)
        assert record_delta(_maxdiff(res["1"][1], fwd(x, per, t)), TOL)
        rxs, _ = O.generalized_steps(x, ones, seq, fwd, _betas())
        assert record_delta(_maxdiff(res["1"][2], torch.stack(rxs)), TOL)
        rz, _ = O.generalized_steps(x, ones, seq, fwd, _betas(), eta=0.7, noise=z)
        assert record_delta(_maxdiff(res["1"][3], rz[-1]), TOL)


@pytest.mark.parametrize("hid,heads", [(128, 8), (64, 2)])
def test_fused_wide_sampler_under_capture(dev, hid, heads):
    """The fused other-width samplers inside a caller's torch.cuda.graph (their per-call timestep
    projections in the capture's scratch): replays bitwise equal to eager."""
    m = HipGCNdiff(adj_mx_from_edges(), _cfg(hid, heads, 2, 17), device=dev)
    m.load_state_dict(synthetic_state_dict(hid=hid, n_layers=2))
    ones = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    x = _inputs(30, 17, seed=92).to(dev)
    seq = make_seq("uniform", 50, 5)
    eager = m.sample(x, seq, _betas(), mask=ones).clone()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        m.sample(x, seq, _betas(), mask=ones)
    torch.cuda.current_stream(dev).wait_stream(s)
    out = torch.empty_like(x)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.sample(x, seq, _betas(), mask=ones, out=out)
    for _ in range(2):
        out.zero_()
        g.replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(out, eager)
    del g
    m.close()


G12 = ["g12_shape_h128_n8_l5_j17.npz", "g12_shape_h128_n4_l3_j17.npz", "g12_shape_h64_n2_l2_j17.npz",
       "g12_shape_h64_n4_l5_j17.npz", "g12_shape_h48_n4_l1_j16.npz"]


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("name", G12)
def test_shapes_vs_reference_goldens(dev, monkeypatch, golden, name, fused):
    """Round 6: the other model shapes against fixtures produced by the reference itself at that
    config.model (tools/gen_goldens.py g12; models/gcndiff.py:55-99, d_k = hid / n_head per
    models/GraFormer.py:116-124): eps at 8 mixed t with the all-ones and a two-key mask, and the K=10
    trajectory (xs, x0s) on 8 frames, at 5e-6.  fused "1": the 17-joint shapes run the persistent-sampler
    instances (dpkw hid 128 / 8 heads, dpkw4 128 / 4, dpkn 64 / 2, dpkn4 64 / 4), the 16-joint chain the
    per-op path; "0": every shape per-op.  The loop-graph count tells the two paths apart (the per-op path
    records its K-step loop as a hipGraph when no trajectory is asked for, the fused instances are one launch)."""
    g = golden(name)
    hid, nh, nl, npts = int(g["hid"]), int(g["n_head"]), int(g["num_layer"]), int(g["n_pts"])
    monkeypatch.setenv("DPK_GEN_FUSED", fused)
    m = HipGCNdiff(g["adj"], _cfg(hid, nh, nl, npts), device=dev)
    m.load_state_dict(synthetic_state_dict(hid=hid, n_layers=nl, n_pts=npts))
    x, t = torch.from_numpy(g["x"]).to(dev), torch.from_numpy(g["t8"]).to(dev)
    ones = torch.ones(1, 1, npts, dtype=torch.bool, device=dev)
    assert record_delta(_maxdiff(m(x, ones, t, 0), torch.from_numpy(g["eps"])), TOL)
    assert record_delta(_maxdiff(m(x, torch.from_numpy(g["mask2"]).to(dev), t, 0), torch.from_numpy(g["eps_masked"])), TOL)
    xs, x0s = m.sample(x, [int(s) for s in g["seq"]], _betas(int(g["T"])), mask=ones, trajectory=True)
    assert record_delta(_maxdiff(xs, torch.from_numpy(g["xs"])), TOL)
    assert record_delta(_maxdiff(x0s, torch.from_numpy(g["x0s"])), TOL)
    # the final alone (no trajectory: the per-op path records its loop as a hipGraph) equals the trajectory's
    out = m.sample(x, [int(s) for s in g["seq"]], _betas(int(g["T"])), mask=ones)
    assert torch.equal(out, xs[-1])
    loops = m.debug_resources()["generic_loop_graphs"]
    if fused == "1" and npts == 17:
        assert loops == 0, "expected the fused persistent-sampler instance"
    else:
        assert loops >= 1, "expected the per-op path"
    m.close()
