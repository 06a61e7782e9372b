"""GPU: dpk_gmm_sample (PoseGeneratorGMM) against golden g8 from the reference's
PoseGenerator_gmm — bit-exact, since the kernel only selects and copies fp32 values — plus the
numpy random-stream order, device-seeded sampling statistics and numpy's argument errors."""
import numpy as np
import pytest
import torch

from diffpose_amd.gmm import PoseGeneratorGMM

pytestmark = pytest.mark.gpu


def _split(a, lens):
    out, o = [], 0
    for n in lens:
        out.append(a[o:o + n])
        o += n
    return out


@pytest.fixture(scope="module")
def g8(golden):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = golden("g8_gmm.npz")
    lens = [int(x) for x in g["lens"]]
    acts = [[f"Walking {si}"] * n for si, n in enumerate(lens)]
    cams = _split(np.zeros((sum(lens), 9), np.float32), lens)
    ds = PoseGeneratorGMM(_split(g["poses_3d"], lens), _split(g["gmm"], lens), acts, cams)
    return g, ds


def _check(g, uv, ns, p2, p3):
    assert np.array_equal(uv.cpu().numpy(), g["uvxyz"])
    assert np.array_equal(ns.cpu().numpy(), g["noise_scale"])
    assert np.array_equal(p2.cpu().numpy(), g["pose_2d"])
    assert np.array_equal(p3.cpu().numpy(), g["pose_3d"])


def test_batch_with_reference_uniforms(g8):
    g, ds = g8
    uv, ns, p2, p3, acts, _ = ds.batch(g["indices"], u=g["u"])
    _check(g, uv, ns, p2, p3)
    assert acts == [str(a) for a in g["actions"]]
    assert len(ds) == 21


def test_global_numpy_stream_order(g8):
    g, ds = g8
    np.random.seed(2024)
    _check(g, *ds.batch(g["indices"])[:4])
    np.random.seed(2024)
    items = [ds[int(i)] for i in g["indices"]]                   # per-item draws, as the Dataset
    _check(g, *(torch.stack([it[k] for it in items]) for k in range(4)))


def test_large_batch_vs_vectorised_restatement():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    rng = np.random.Generator(np.random.PCG64(5))
    F, kn = 20000, 7
    w = rng.dirichlet(np.ones(kn), size=(F, 17)).astype(np.float32)
    g = np.concatenate([w[..., None], rng.uniform(-1, 1, size=(F, 17, kn, 4))], axis=-1).astype(np.float32)
    p3 = rng.normal(size=(F, 17, 3)).astype(np.float32)
    ds = PoseGeneratorGMM([p3], [g], [["a"] * F], [np.zeros((F, 1), np.float32)])
    idx = rng.integers(0, 2 * F, size=F)
    u = rng.random((F, 17))
    uv, ns, *_ = ds.batch(idx, u=u)
    src = idx % F
    cdf = np.cumsum(w[src].astype(np.float64), axis=-1)
    cdf /= cdf[..., -1:]
    k = (cdf <= u[..., None]).sum(-1)
    comp = np.take_along_axis(g[src], k[..., None, None], axis=2)[:, :, 0]
    assert np.array_equal(uv.cpu().numpy()[..., :2], comp[..., 1:3])
    assert np.array_equal(ns.cpu().numpy()[..., :2], comp[..., 3:5])
    assert np.array_equal(uv.cpu().numpy()[..., 2:], p3[src] - p3[src][:, :1])
    assert np.all(ns.cpu().numpy()[..., 2:] == 1.0)


def test_device_seeded_sampling_frequencies():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    w = np.array([0.1, 0.2, 0.3, 0.4], np.float32)
    g = np.zeros((1, 17, 4, 5), np.float32)
    g[..., 0] = w
    g[..., 1] = np.arange(4)                     # mu_u = component id
    ds = PoseGeneratorGMM([np.zeros((1, 17, 3), np.float32)], [g], [["a"]], [np.zeros((1, 1), np.float32)])
    uv = ds.batch(np.zeros(20000, np.int64), seed=7)[0]
    ids = uv[..., 0].round().long().cpu().numpy().ravel()
    freq = np.bincount(ids, minlength=4) / ids.size
    assert np.all(np.abs(freq - w) < 0.005)      # 340k draws: std <= 0.0009
    assert torch.equal(uv, ds.batch(np.zeros(20000, np.int64), seed=7)[0])
    assert not torch.equal(uv, ds.batch(np.zeros(20000, np.int64), seed=8)[0])


def test_numpy_argument_errors():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = np.zeros((2, 17, 3, 5), np.float32)
    g[..., 0] = [0.5, 0.25, 0.25]
    bad = g.copy()
    bad[1, 4, :, 0] = [0.6, -0.1, 0.5]
    ds = PoseGeneratorGMM([np.zeros((2, 17, 3), np.float32)], [bad], [["a", "b"]], [np.zeros((2, 1), np.float32)])
    ds.batch([0])
    with pytest.raises(ValueError, match="non-negative"):
        ds.batch([1])
    bad[1, 4, :, 0] = [0.6, 0.3, 0.2]
    ds = PoseGeneratorGMM([np.zeros((2, 17, 3), np.float32)], [bad], [["a", "b"]], [np.zeros((2, 1), np.float32)])
    with pytest.raises(ValueError, match="sum to 1"):
        ds.batch([0, 1])


def test_float64_inputs_follow_the_reference_dtype_order():
    """float64 arrays (advisor r01): the choice runs on the float64 weights and the root-relative
    subtraction in float64 before the .float() cast (generators.py:19, :46-50).  The weights are
    built so that rounding them to float32 first would move a cdf boundary across the uniform,
    and the poses so that subtract-then-round differs from round-then-subtract; the oracle's
    numpy restatement (float64 throughout, as the reference) is matched bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from oracle.gmm_oracle import gmm_item
    from diffpose_amd.gmm import numpy_atol

    rng = np.random.Generator(np.random.PCG64(64))
    F, kn = 40, 3
    w = rng.dirichlet(np.ones(kn), size=(F, 17))
    g = np.concatenate([w[..., None], rng.uniform(-1, 1, size=(F, 17, kn, 4))], axis=-1)
    p3 = rng.normal(0.0, 0.5, size=(F, 17, 3)) + 1.0 / 3.0
    u = rng.random((F, 17))
    # put the uniform exactly on the float64 cdf boundary of joint 5 of frame 0: numpy picks the
    # component past it; float32-rounded weights would move the boundary
    c0 = w[0, 5, 0] / w[0, 5].sum()
    u[0, 5] = c0
    assert np.float64(np.float32(w[0, 5, 0])) != w[0, 5, 0]
    ds = PoseGeneratorGMM([p3], [g], [["a"] * F], [np.zeros((F, 1))])
    idx = np.arange(F)
    uv, ns, *_ = ds.batch(idx, u=u)
    p3rel = p3 - p3[:, :1]
    atol = numpy_atol(np.float64)
    for f in range(F):
        ruv, rns = gmm_item(p3rel, g, f, u[f], atol)
        assert np.array_equal(uv[f].cpu().numpy(), ruv), f
        assert np.array_equal(ns[f].cpu().numpy(), rns), f
    # the float32 path on the same data rounded to float32 differs somewhere in the poses
    ds32 = PoseGeneratorGMM([p3.astype(np.float32)], [g.astype(np.float32)], [["a"] * F], [np.zeros((F, 1))])
    uv32, *_ = ds32.batch(idx, u=u)
    assert not torch.equal(uv32[..., 2:], uv[..., 2:])
