"""GCNdiff parameter layout, checkpoint loading and the synthetic-weight generator.

The key list is the state_dict of the reference denoiser ``GCNdiff``
(reference ``models/gcndiff.py:55-99``), which the reference saves as
``states[0]`` of a DataParallel-wrapped model (``runners/diffpose_frame.py:127-132``,
``:247-258``), i.e. with a ``module.`` prefix.  ``load_checkpoint`` accepts the
list-of-states file, a bare state_dict, with or without the prefix.

There are no trained checkpoints offline (reference ``README.md:48``), so the
bench and the parity tests run on ``synthetic_state_dict`` — a seeded NumPy
PCG64 draw whose distributions follow the reference's own initialisers, made
non-degenerate so every branch of the network carries signal:

* ChebConv weight ``(3,1,in,out)``: N(0, sqrt(1/(6*(in+out)))) — xavier over
  (in, out) split across the three Chebyshev terms and halved.  The reference's
  ``xavier_normal_`` on the 4-D tensor (``models/ChebConv.py:62``) treats
  ``in*out`` as the receptive field and gives std ~0.007, which would leave the
  graph-conv path numerically invisible in a parity test; a full xavier makes
  the sampler chaotic (|eps|~2, poses drift ~2 m over K=50, and the
  reference's OWN fp32-vs-fp64 gap reaches 3.3e-4 mm MPJPE at N=1024).  With
  this scale |eps|~0.6, drift ~0.26 m and that gap is ~2e-5 mm (N=256, K=50),
  so the 1e-4 mm parity target is meaningful.
* ChebConv bias ``(1,1,out)``: N(0, 0.02) (reference: zeros, ``:66``).
* nn.Linear weight/bias: U(-1/sqrt(in), 1/sqrt(in)) (torch default init).
* GraphNet ``A_hat``: I + U(0, 0.05) — keeps column sums > 0 (the reference
  ``LAM_Gconv.laplacian_batch`` ``models/GraFormer.py:174-178`` takes them to
  the power -1/2).
* LayerNorm ``a_2``: 1 + N(0, 0.1), ``b_2``: N(0, 0.1) (reference: ones/zeros).
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np

HID = 96          # config.model.hid_dim (configs/human36m_diffpose_uvxyz_cpn.yml:10)
EMB = 4 * HID     # GCNdiff.emd_dim = hid_dim*4 (models/gcndiff.py:68)
N_LAYERS = 5      # config.model.num_layer
N_HEAD = 4        # config.model.n_head
N_PTS = 17        # config.model.n_pts
COORDS = (5, 5)   # config.model.coords_dim (uvxyz in, eps out)
POSE_COORDS = (2, 3)  # GCNpose: uv in, xyz out (runners/diffpose_frame.py:138)
DEFAULT_SEED = 19960903  # main_diffpose_frame.py:20
POSE_SEED = DEFAULT_SEED + 1


def param_shapes(hid: int = HID, n_layers: int = N_LAYERS, n_pts: int = N_PTS,
                 coords=None, kind: str = "diff") -> "OrderedDict[str, tuple]":
    """Ordered (key -> shape) of GCNdiff's state_dict (models/gcndiff.py:55-99), or with
    ``kind="pose"`` of GCNpose's (models/gcnpose.py:55-98: coords [2,3], no temb_proj in its
    _ResChebGC blocks, the unused temb.dense layers still registered)."""
    if kind not in ("diff", "pose"):
        raise ValueError(f"kind must be 'diff' or 'pose', got {kind!r}")
    pose = kind == "pose"
    if coords is None:
        coords = POSE_COORDS if pose else COORDS
    emb = 4 * hid
    s: "OrderedDict[str, tuple]" = OrderedDict()
    s["gconv_input.weight"] = (3, 1, coords[0], hid)
    s["gconv_input.bias"] = (1, 1, hid)
    for i in range(n_layers):
        p = f"gconv_layers.{i}."
        for g in ("gconv1", "gconv2"):
            s[p + g + ".gconv.weight"] = (3, 1, hid, hid)
            s[p + g + ".gconv.bias"] = (1, 1, hid)
        if not pose:
            s[p + "temb_proj.weight"] = (hid, emb)
            s[p + "temb_proj.bias"] = (hid,)
    for i in range(n_layers):
        p = f"atten_layers.{i}."
        for j in range(4):
            s[p + f"self_attn.linears.{j}.weight"] = (hid, hid)
            s[p + f"self_attn.linears.{j}.bias"] = (hid,)
        s[p + "feed_forward.A_hat"] = (n_pts, n_pts)
        s[p + "feed_forward.gconv1.fc.weight"] = (2 * hid, hid)
        s[p + "feed_forward.gconv1.fc.bias"] = (2 * hid,)
        s[p + "feed_forward.gconv2.fc.weight"] = (hid, 2 * hid)
        s[p + "feed_forward.gconv2.fc.bias"] = (hid,)
        for j in range(2):
            s[p + f"sublayer.{j}.norm.a_2"] = (hid,)
            s[p + f"sublayer.{j}.norm.b_2"] = (hid,)
    s["gconv_output.weight"] = (3, 1, hid, coords[1])
    s["gconv_output.bias"] = (1, 1, coords[1])
    s["temb.dense.0.weight"] = (emb, hid)
    s["temb.dense.0.bias"] = (emb,)
    s["temb.dense.1.weight"] = (emb, emb)
    s["temb.dense.1.bias"] = (emb,)
    return s


def _draw(rng: np.random.Generator, key: str, shape: tuple) -> np.ndarray:
    if key.endswith("A_hat"):
        n = shape[0]
        a = np.eye(n) + rng.uniform(0.0, 0.05, size=shape)
    elif key.endswith("norm.a_2"):
        a = 1.0 + rng.normal(0.0, 0.1, size=shape)
    elif key.endswith("norm.b_2"):
        a = rng.normal(0.0, 0.1, size=shape)
    elif len(shape) == 4:                      # ChebConv weight (K+1, 1, in, out)
        fan_in, fan_out = shape[2], shape[3]
        a = rng.normal(0.0, np.sqrt(1.0 / (6.0 * (fan_in + fan_out))), size=shape)
    elif len(shape) == 3:                      # ChebConv bias (1, 1, out)
        a = rng.normal(0.0, 0.02, size=shape)
    elif len(shape) == 2:                      # nn.Linear weight (out, in)
        bound = 1.0 / np.sqrt(shape[1])
        a = rng.uniform(-bound, bound, size=shape)
    else:                                      # nn.Linear bias (out,)
        # bound from the matching weight's fan_in, resolved by the caller
        raise KeyError(key)
    return np.ascontiguousarray(a, dtype=np.float32)


def synthetic_state_dict(seed: int | None = None, **shape_kw) -> "OrderedDict[str, np.ndarray]":
    """Deterministic synthetic GCNdiff (or, ``kind="pose"``, GCNpose) weights (float32 numpy
    arrays, no prefix).  Default seeds: DEFAULT_SEED (diff), POSE_SEED (pose)."""
    if seed is None:
        seed = POSE_SEED if shape_kw.get("kind") == "pose" else DEFAULT_SEED
    rng = np.random.Generator(np.random.PCG64(seed))
    shapes = param_shapes(**shape_kw)
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, shape in shapes.items():
        if len(shape) == 1 and not key.endswith(("a_2", "b_2")):
            wshape = shapes[key[: -len("bias")] + "weight"]
            bound = 1.0 / np.sqrt(wshape[1])
            out[key] = np.ascontiguousarray(rng.uniform(-bound, bound, size=shape), dtype=np.float32)
        else:
            out[key] = _draw(rng, key, shape)
    return out


def state_dict_sha256(sd, kind: str = "diff") -> str:
    """sha256 over key names and little-endian float32 payloads, in layout order."""
    h = hashlib.sha256()
    for key in param_shapes(kind=kind):
        a = np.ascontiguousarray(np.asarray(sd[key], dtype="<f4"))
        h.update(key.encode())
        h.update(a.tobytes())
    return h.hexdigest()


def strip_module_prefix(sd) -> "OrderedDict[str, object]":
    """Accept DataParallel ('module.'-prefixed) or bare keys (runners/diffpose_frame.py:130-132)."""
    out = OrderedDict()
    for k, v in sd.items():
        out[k[len("module."):] if k.startswith("module.") else k] = v
    return out


def normalize_state_dict(sd, kind: str = "diff", n_layers: int = N_LAYERS, hid: int = HID, n_pts: int = N_PTS,
                         coords=None) -> "OrderedDict[str, np.ndarray]":
    """Validate a GCNdiff (GCNpose) state_dict against the layout; return float32 numpy arrays.

    Raises KeyError for missing/unexpected keys and ValueError for shape
    mismatches, mirroring ``nn.Module.load_state_dict(strict=True)``.
    """
    sd = strip_module_prefix(sd)
    shapes = param_shapes(kind=kind, n_layers=n_layers, hid=hid, n_pts=n_pts, coords=coords)
    missing = [k for k in shapes if k not in sd]
    unexpected = [k for k in sd if k not in shapes]
    if missing or unexpected:
        raise KeyError(f"state_dict mismatch: missing={missing[:5]}... unexpected={unexpected[:5]}...")
    out = OrderedDict()
    for k, shape in shapes.items():
        v = sd[k]
        if hasattr(v, "detach"):
            v = v.detach().cpu().numpy()
        a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
        if tuple(a.shape) != tuple(shape):
            raise ValueError(f"{k}: shape {tuple(a.shape)} != expected {tuple(shape)}")
        out[k] = a
    return out


def load_checkpoint(path: str, kind: str = "diff", n_layers: int = N_LAYERS) -> "OrderedDict[str, np.ndarray]":
    """Load a reference checkpoint (list with states[0] = model state_dict) safely.

    Uses ``torch.load(weights_only=True)`` — never unpickles arbitrary objects.
    """
    import torch

    states = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(states, (list, tuple)):
        states = states[0]
    return normalize_state_dict(states, kind=kind, n_layers=n_layers)


def reference_init_state_dict(seed: int, n_layers: int = N_LAYERS, hid: int = HID, n_pts: int = N_PTS,
                              coords=COORDS) -> "OrderedDict[str, np.ndarray]":
    """GCNdiff's weights exactly as the reference constructor draws them after
    ``torch.manual_seed(seed)`` (float32 numpy, no prefix) — the initialisers a freshly built
    reference model carries, for parity on the reference's own value range.

    Restates the parameter-drawing order of ``GCNdiff.__init__`` (models/gcndiff.py:55-99) with
    torch's own initialisers, consuming torch's global generator in the same sequence:
      1. gconv_input ``ChebConv(5, 96, K=2)``: xavier_normal_ on the (3,1,in,out) weight, zero
         bias (models/ChebConv.py:59-67);
      2. one ``nn.Linear(96, 96)`` deep-copied into the 4 attention projections
         (``clones``, models/GraFormer.py:55, :123) and ``copy.deepcopy``'d into every layer
         (models/gcndiff.py:80-89): all 4 projections of all layers start equal;
      3. one ``GraphNet(96, 96, 17)``: A_hat = I, fc 96->192 then 192->96 (GraFormer.py:191-196),
         likewise copied into every layer;
      4. per layer: Cheb 96->96 (gconv1), Cheb 96->96 (gconv2), temb_proj Linear(384, 96)
         (models/gcndiff.py:39-46); LayerNorm gains 1, shifts 0 (GraFormer.py:63-64);
      5. gconv_output ``ChebConv(96, 5, K=2)``; 6. temb.dense Linear(96, 384), Linear(384, 384).
    Pinned by the sha256 the golden generator takes of the reference model built under the same
    seed (tests/golden/meta.json "refinit_sha256")."""
    import torch
    from torch import nn

    emb = 4 * hid
    state = torch.random.get_rng_state()
    try:
        torch.manual_seed(seed)

        def cheb(cin, cout):
            w = torch.empty(3, 1, cin, cout)
            nn.init.xavier_normal_(w)
            return w, torch.zeros(1, 1, cout)

        def linear(cin, cout):
            m = nn.Linear(cin, cout)
            return m.weight.detach().clone(), m.bias.detach().clone()

        win, bin_ = cheb(coords[0], hid)
        attn = linear(hid, hid)
        fc1 = linear(hid, 2 * hid)
        fc2 = linear(2 * hid, hid)
        layers = []
        for _ in range(n_layers):
            layers.append((cheb(hid, hid), cheb(hid, hid), linear(emb, hid)))
        wout, bout = cheb(hid, coords[1])
        d0 = linear(hid, emb)
        d1 = linear(emb, emb)
    finally:
        torch.random.set_rng_state(state)
    sd = {"gconv_input.weight": win, "gconv_input.bias": bin_}
    for i, (g1, g2, tp) in enumerate(layers):
        p = f"gconv_layers.{i}."
        sd[p + "gconv1.gconv.weight"], sd[p + "gconv1.gconv.bias"] = g1
        sd[p + "gconv2.gconv.weight"], sd[p + "gconv2.gconv.bias"] = g2
        sd[p + "temb_proj.weight"], sd[p + "temb_proj.bias"] = tp
    for i in range(n_layers):
        p = f"atten_layers.{i}."
        for j in range(4):
            sd[p + f"self_attn.linears.{j}.weight"], sd[p + f"self_attn.linears.{j}.bias"] = attn
        sd[p + "feed_forward.A_hat"] = torch.eye(n_pts)
        sd[p + "feed_forward.gconv1.fc.weight"], sd[p + "feed_forward.gconv1.fc.bias"] = fc1
        sd[p + "feed_forward.gconv2.fc.weight"], sd[p + "feed_forward.gconv2.fc.bias"] = fc2
        for j in range(2):
            sd[p + f"sublayer.{j}.norm.a_2"] = torch.ones(hid)
            sd[p + f"sublayer.{j}.norm.b_2"] = torch.zeros(hid)
    sd["gconv_output.weight"], sd["gconv_output.bias"] = wout, bout
    sd["temb.dense.0.weight"], sd["temb.dense.0.bias"] = d0
    sd["temb.dense.1.weight"], sd["temb.dense.1.bias"] = d1
    shapes = param_shapes(hid=hid, n_layers=n_layers, n_pts=n_pts, coords=coords)
    return OrderedDict((k, np.ascontiguousarray(sd[k].numpy(), dtype=np.float32)) for k in shapes)
