"""CPU: pin the oracle (and the host schedule/weights code) to the reference's own outputs.

Fixtures in tests/golden/ were produced by tools/gen_goldens.py, which imports the
reference (/root/reference) in the build container and runs it on CPU.  The oracle
issues the same ATen ops as the reference, so on the same torch build it must match
bit for bit; a different torch build may drift by fp32 rounding, hence the 1e-6 bound.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import gcndiff_oracle as O
from diffpose_amd.schedule import alpha_bar_table, ddim_coeffs, get_beta_schedule, make_seq, step_pairs
from diffpose_amd.weights import param_shapes, state_dict_sha256, synthetic_state_dict, strip_module_prefix, \
    normalize_state_dict
from diffpose_amd.data import synthetic_batch, shard_frames, repeat_hypotheses
from diffpose_amd.gcndiff import adj_mx_from_edges

from conftest import GOLDEN

ATOL = 1e-6


@pytest.fixture(scope="module")
def params():
    return O.params_to_torch(synthetic_state_dict())


@pytest.fixture(scope="module")
def graph():
    return O.adjacency()


def _close(a, b, atol=ATOL):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    d = float(np.abs(a.astype(np.float64) - b.astype(np.float64)).max()) if a.size else 0.0
    assert d <= atol, f"max abs diff {d} > {atol}"


def test_weights_sha_matches_fixture():
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    assert state_dict_sha256(synthetic_state_dict()) == meta["weights_sha256"]


def test_state_dict_layout_and_prefix():
    sd = synthetic_state_dict()
    assert list(sd.keys()) == list(param_shapes().keys())
    assert sum(v.size for v in sd.values()) == 1_025_674
    pref = {"module." + k: v for k, v in sd.items()}
    assert list(strip_module_prefix(pref).keys()) == list(sd.keys())
    norm = normalize_state_dict(pref)
    assert all(np.array_equal(norm[k], sd[k]) for k in sd)
    bad = dict(sd)
    bad.pop("gconv_output.bias")
    with pytest.raises(KeyError):
        normalize_state_dict(bad)
    bad = dict(sd)
    bad["gconv_output.bias"] = np.zeros((1, 1, 4), np.float32)
    with pytest.raises(ValueError):
        normalize_state_dict(bad)


def test_graph_constants(golden, graph):
    g = golden("g1_graph.npz")
    assert np.array_equal(graph.numpy(), g["adj"])
    assert np.array_equal(adj_mx_from_edges(), g["adj"])           # product-side builder too
    _close(O.cheb_basis(graph).numpy(), g["cheb"])
    sd = synthetic_state_dict()
    for i in range(5):
        a = torch.from_numpy(sd[f"atten_layers.{i}.feed_forward.A_hat"])
        _close(O.graph_laplacian(a, 1)[0].numpy(), g["lg"][i])


def test_modules(golden, params, graph):
    g = golden("g2_modules.npz")
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["t"])
    _close(O.timestep_embedding(t, 96).numpy(), g["temb"])
    h_in = O.cheb_conv(x, graph, params["gconv_input.weight"], params["gconv_input.bias"])
    _close(h_in.numpy(), g["h_in"])
    ln0 = O.layer_norm(h_in, params["atten_layers.0.sublayer.0.norm.a_2"], params["atten_layers.0.sublayer.0.norm.b_2"])
    _close(ln0.numpy(), g["ln0"])
    lw = [params[f"atten_layers.0.self_attn.linears.{j}.weight"] for j in range(4)]
    lb = [params[f"atten_layers.0.self_attn.linears.{j}.bias"] for j in range(4)]
    mha, p = O.multi_head_attention(ln0, torch.ones(1, 1, 17, dtype=torch.bool), lw, lb, 4)
    _close(mha.numpy(), g["mha"])
    _close(p.numpy(), g["p_attn"])
    out = O.cheb_conv(torch.from_numpy(g["h_out_in"]), graph, params["gconv_output.weight"], params["gconv_output.bias"])
    _close(out.numpy(), g["cheb_out"])


def test_full_eps(golden, params, graph):
    g = golden("g2_modules.npz")
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["t"])
    eps = O.gcndiff_forward(params, graph, x, torch.ones(1, 1, 17, dtype=torch.bool), t)
    _close(eps.numpy(), g["eps"])
    eps_m = O.gcndiff_forward(params, graph, x, torch.from_numpy(g["mask2"]), t)
    _close(eps_m.numpy(), g["eps_masked"])


def _betas(T):
    return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                              num_diffusion_timesteps=T)).float()


def test_trajectory_k10(golden, params, graph):
    g = golden("g3_traj_n64_k10.npz")
    fn = lambda xt, m, tt: O.gcndiff_forward(params, graph, xt, m, tt)  # noqa: E731
    xs, x0s = O.generalized_steps(torch.from_numpy(g["x"]), torch.ones(1, 1, 17, dtype=torch.bool),
                                  [int(s) for s in g["seq"]], fn, _betas(int(g["T"])))
    _close(torch.stack(xs).numpy(), g["xs"])
    _close(torch.stack(x0s).numpy(), g["x0s"])
    xyz = O.post_process(xs[-1], 1)
    assert abs(O.mpjpe(xyz.double(), torch.from_numpy(g["targets"]).double()).item() * 1000 - float(g["mpjpe_mm"])) < 1e-4


@pytest.mark.parametrize("name", ["g4_final_n8_quad.npz", "g4_final_n16_k50.npz"])
def test_final_sample(golden, params, graph, name):
    g = golden(name)
    fn = lambda xt, m, tt: O.gcndiff_forward(params, graph, xt, m, tt)  # noqa: E731
    xs, _ = O.generalized_steps(torch.from_numpy(g["x"]), torch.ones(1, 1, 17, dtype=torch.bool),
                                [int(s) for s in g["seq"]], fn, _betas(int(g["T"])))
    _close(xs[-1].numpy(), g["out"])


def test_eta_trajectory_reference_noise(golden, params, graph):
    """eta > 0 (g11): under the reference's seed the oracle draws the same per-step randn_like and
    reproduces the reference's trajectory; the stored draws replayed explicitly give the same bits,
    and ``utils_diff.draw_noise("torch-cpu")`` draws exactly those tensors."""
    from diffpose_amd.utils_diff import draw_noise

    g = golden("g11_eta.npz")
    fn = lambda xt, m, tt: O.gcndiff_forward(params, graph, xt, m, tt)  # noqa: E731
    mask = torch.ones(1, 1, 17, dtype=torch.bool)
    x = torch.from_numpy(g["x"])
    seq10 = [int(s) for s in g["seq10"]]
    torch.manual_seed(int(g["seed10"]))
    xs, x0s = O.generalized_steps(x, mask, seq10, fn, _betas(51), eta=float(g["eta10"]))
    _close(torch.stack(xs).numpy(), g["xs10"], 0.0)
    _close(torch.stack(x0s).numpy(), g["x0s10"], 0.0)
    torch.manual_seed(int(g["seed10"]))
    z = draw_noise(x, len(seq10), "torch-cpu")
    assert torch.equal(z, torch.from_numpy(g["noise10"]))
    xs_n, _ = O.generalized_steps(x, mask, seq10, fn, _betas(51), eta=float(g["eta10"]), noise=z)
    _close(xs_n[-1].numpy(), g["xs10"][-1], 0.0)
    # test_hyber's extra draw before the sampler (runners/diffpose_frame.py:359)
    torch.manual_seed(int(g["seed_hyber"]))
    torch.randn_like(x)
    xs_h, _ = O.generalized_steps(x, mask, seq10, fn, _betas(51), eta=float(g["eta10"]))
    _close(xs_h[-1].numpy(), g["out_hyber"], 0.0)
    seq50 = [int(s) for s in g["seq50"]]
    xs50, _ = O.generalized_steps(x, mask, seq50, fn, _betas(51), eta=float(g["eta50"]),
                                  noise=torch.from_numpy(g["noise50"]))
    _close(xs50[-1].numpy(), g["out50"], ATOL)
    # the noise term is live: another seed's draws give another trajectory
    assert float(np.abs(g["xs10"][-1] - xs_h[-1].numpy()).max()) > 1e-3


def test_schedule_tables():
    for kind in ("linear", "quad", "const", "jsd", "sigmoid"):
        for T in (51, 101):
            b = _betas(T) if kind == "linear" else torch.from_numpy(
                get_beta_schedule(kind, beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=T)).float()
            ref = (1 - torch.cat([torch.zeros(1), b])).cumprod(0).numpy()
            assert np.array_equal(alpha_bar_table(b.numpy()), ref), (kind, T)
            t = torch.arange(-1, T, dtype=torch.long)
            assert np.array_equal(O.alpha_at(b, t).reshape(-1).numpy(), ref)
    with pytest.raises(NotImplementedError):
        get_beta_schedule("cosine", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=10)


def test_seq_and_pairs():
    assert make_seq("uniform", 50, 10) == list(range(0, 50, 5))
    assert make_seq("uniform", 24, 2) == [0, 12]                     # cpn config defaults
    q = make_seq("quad", 50, 10)
    assert q[:2] == [0, 0] and len(q) == 10                           # duplicates are legal
    assert step_pairs([0, 12]) == [(12, 0), (0, -1)]
    with pytest.raises(NotImplementedError):
        make_seq("cosine", 10, 2)


def test_ddim_coeffs_match_reference_ops():
    b = _betas(51)
    seq = list(range(0, 50, 5))
    c = ddim_coeffs(alpha_bar_table(b.numpy()), seq, eta=0.5)
    for k, (i, j) in enumerate(step_pairs(seq)):
        at = O.alpha_at(b, torch.tensor([i]))
        an = O.alpha_at(b, torch.tensor([j]))
        c1 = 0.5 * ((1 - at / an) * (1 - an) / (1 - at)).sqrt()
        c2 = ((1 - an) - c1 ** 2).sqrt()
        ref = [(1 - at).sqrt(), at.sqrt(), an.sqrt(), c1, c2]
        for col, r in enumerate(ref):
            assert c[k, col] == np.float32(r.item()), (k, col)
    with pytest.raises(IndexError):
        ddim_coeffs(alpha_bar_table(b.numpy()), [0, 60])             # K=100-with-T=51 impossibility


def test_root_quirk(golden):
    g = golden("g5_root_quirk.npz")
    out = O.root_subtract_inplace_quirk(torch.from_numpy(g["x"]))
    assert np.array_equal(out.numpy(), g["out"])
    assert bool(g["b1_raises"])


def test_synthetic_data_and_sharding():
    a, ta = synthetic_batch(32, seed=5)
    b, tb = synthetic_batch(32, seed=5)
    assert np.array_equal(a, b) and np.array_equal(ta, tb)
    assert a.shape == (32, 17, 5) and ta.shape == (32, 17, 3)
    assert np.all(a[:, 0, 2:] == 0) and np.all(np.abs(a[:, :, :2]) <= 1)
    spans = [shard_frames(1000, 8, r) for r in range(8)]
    assert spans[0][0] == 0 and spans[-1][1] == 1000
    assert all(spans[i][1] == spans[i + 1][0] for i in range(7))
    r = repeat_hypotheses(a[:4], 3)
    assert r.shape == (12, 17, 5) and np.array_equal(r[4:8], a[:4])


def test_gcnpose_oracle(golden, graph):
    """GCNpose front-end + test_hyber's uvxyz assembly (g6, from the reference GCNpose)."""
    from diffpose_amd.weights import synthetic_state_dict, state_dict_sha256

    g = golden("g6_gcnpose.npz")
    sd = synthetic_state_dict(kind="pose")
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    assert state_dict_sha256(sd, kind="pose") == meta["pose_weights_sha256"]
    P = O.params_to_torch(sd)
    x2d = torch.from_numpy(g["x2d"])
    xyz = O.gcnpose_forward(P, graph, x2d, torch.ones(1, 1, 17, dtype=torch.bool))
    assert np.array_equal(xyz.numpy(), g["xyz"])
    assert np.array_equal(O.gcnpose_forward(P, graph, x2d, torch.from_numpy(g["mask2"])).numpy(), g["xyz_masked"])
    assert np.array_equal(O.build_uvxyz(x2d, xyz, 3, "quirk").numpy(), g["uvxyz_h3"])


def test_load_checkpoint_reference_format(tmp_path):
    """A checkpoint shaped like the reference's (runners/diffpose_frame.py:131-132: torch.save of a list
    whose [0] is the DataParallel state_dict, "module." prefixed) loads with weights_only=True."""
    import torch

    from diffpose_amd.weights import load_checkpoint

    sd = synthetic_state_dict()
    states = [{"module." + k: torch.from_numpy(v.copy()) for k, v in sd.items()},
              {"state": {}, "param_groups": [{"lr": 1e-3, "params": [0, 1]}]}]
    path = tmp_path / "ckpt_diff.pth"
    torch.save(states, str(path))
    got = load_checkpoint(str(path), kind="diff")
    assert list(got.keys()) == list(sd.keys())
    assert all(np.array_equal(got[k], sd[k]) for k in sd)
    # GCNpose checkpoints use the same container (diffpose_frame.py:146-147)
    psd = synthetic_state_dict(kind="pose")
    torch.save([{"module." + k: torch.from_numpy(v.copy()) for k, v in psd.items()}], str(path))
    gp = load_checkpoint(str(path), kind="pose")
    assert all(np.array_equal(gp[k], psd[k]) for k in psd)


# ---- other weight distributions (golden groups g9/g10) ----------------------------------------
def _weights_for(name):
    from diffpose_amd.weights import reference_init_state_dict

    if name.startswith("g9_refinit_seed"):
        return reference_init_state_dict(int(name[len("g9_refinit_seed"):].split(".")[0]))
    return synthetic_state_dict(seed=7)


def test_reference_initialisers_restated_exactly():
    """weights.reference_init_state_dict(s) == the state_dict of the reference GCNdiff built under
    torch.manual_seed(s) (sha256 taken by tools/gen_goldens.py from the reference model itself)."""
    from diffpose_amd.weights import reference_init_state_dict

    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    for s, sha in meta["refinit_sha256"].items():
        assert state_dict_sha256(reference_init_state_dict(int(s))) == sha
    assert state_dict_sha256(synthetic_state_dict(seed=7)) == meta["seed7_weights_sha256"]


@pytest.mark.parametrize("name", ["g9_refinit_seed0.npz", "g9_refinit_seed1.npz", "g10_synth_seed7.npz"])
def test_oracle_on_other_weights(golden, graph, name):
    g = golden(name)
    P = O.params_to_torch(_weights_for(name))
    mask = torch.ones(1, 1, 17, dtype=torch.bool)
    _close(O.gcndiff_forward(P, graph, torch.from_numpy(g["x"][:8]), mask, torch.from_numpy(g["t8"])).numpy(), g["eps"])
    fn = lambda xt, m, tt: O.gcndiff_forward(P, graph, xt, m, tt)  # noqa: E731
    xs, _ = O.generalized_steps(torch.from_numpy(g["x"]), mask, [int(s) for s in g["seq"]], fn, _betas(int(g["T"])))
    _close(xs[-1].numpy(), g["out"])


def test_draw_noise_sources():
    """utils_diff.draw_noise: "torch" draws randn_like(x) K times on x's device in the reference's
    order (common/utils_diff.py:65); "philox"/None draw nothing (in-kernel noise); a tensor is
    checked for shape; anything else raises."""
    from diffpose_amd.utils_diff import draw_noise

    x = torch.zeros(5, 17, 5)
    torch.manual_seed(21)
    z = draw_noise(x, 3, "torch")
    torch.manual_seed(21)
    ref = torch.stack([torch.randn_like(x) for _ in range(3)])
    assert torch.equal(z, ref) and z.dtype == torch.float32
    g1, g2 = torch.Generator().manual_seed(5), torch.Generator().manual_seed(5)
    assert torch.equal(draw_noise(x, 2, "torch", generator=g1), draw_noise(x, 2, "torch-cpu", generator=g2))
    assert draw_noise(x, 3, "philox") is None and draw_noise(x, 3, None) is None
    assert torch.equal(draw_noise(x, 3, ref), ref)
    with pytest.raises(ValueError):
        draw_noise(x, 2, ref)
    with pytest.raises(ValueError):
        draw_noise(x, 2, "gaussian")


G12 = ["g12_shape_h128_n8_l5_j17.npz", "g12_shape_h128_n4_l3_j17.npz", "g12_shape_h64_n2_l2_j17.npz",
       "g12_shape_h64_n4_l5_j17.npz", "g12_shape_h48_n4_l1_j16.npz"]


@pytest.mark.parametrize("name", G12)
def test_other_shapes_vs_reference(golden, name):
    """Round 6: the oracle's shape-generic code (d_k 16 / 32 / 12, 2 / 8 heads, a 16-joint chain) pinned
    bit-exact to the reference GCNdiff built at that config.model (models/gcndiff.py:55-99,
    models/GraFormer.py:116-124; fixtures from tools/gen_goldens.py --only g12): eps with two masks and a
    K=10 trajectory, with the build's generator weights at that shape (sha256 in meta.json)."""
    import hashlib
    g = golden(name)
    hid, nh, nl, npts = int(g["hid"]), int(g["n_head"]), int(g["num_layer"]), int(g["n_pts"])
    sd = synthetic_state_dict(hid=hid, n_layers=nl, n_pts=npts)
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v, dtype="<f4").tobytes())
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    assert meta["shape_weights_sha256"][name[:-4]] == h.hexdigest()
    P = O.params_to_torch(sd)
    graph = O.adjacency(npts, [tuple(e) for e in g["edges"].tolist()])
    assert np.array_equal(graph.numpy(), g["adj"])
    ones = torch.ones(1, 1, npts, dtype=torch.bool)
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["t8"])
    fn = lambda xt, m, tt: O.gcndiff_forward(P, graph, xt, m, tt, n_layers=nl, heads=nh)  # noqa: E731
    assert np.array_equal(fn(x, ones, t).numpy(), g["eps"])
    assert np.array_equal(fn(x, torch.from_numpy(g["mask2"]), t).numpy(), g["eps_masked"])
    xs, x0s = O.generalized_steps(x, ones, [int(s) for s in g["seq"]], fn, _betas(int(g["T"])))
    assert np.array_equal(torch.stack(xs).numpy(), g["xs"])
    assert np.array_equal(torch.stack(x0s).numpy(), g["x0s"])
