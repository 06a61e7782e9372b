"""ORACLE — test infrastructure only.  CPU restatement of the reference hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``diffpose-nw_amd/``) never imports it and fails loudly when
its HIP library is missing.

What it restates (reference at /root/reference, file:line):

* ``adjacency``        — ``adj_mx_from_edges`` + ``normalize``  models/GraFormer.py:13-20, :32-44
* ``cheb_basis``       — ``ChebConv.get_laplacian`` / ``cheb_polynomial``  models/ChebConv.py:90-130
* ``cheb_conv``        — ``ChebConv.forward``  models/ChebConv.py:74-88
* ``timestep_embedding`` — ``get_timestep_embedding``  models/gcndiff.py:15-33
* ``layer_norm``       — GraFormer ``LayerNorm.forward`` (unbiased std, eps on std)  models/GraFormer.py:58-70
* ``multi_head_attention`` — ``MultiHeadedAttention.forward`` + ``attention``  models/GraFormer.py:99-140
* ``graph_net``        — ``GraphNet`` / ``LAM_Gconv``  models/GraFormer.py:162-201
* ``gcndiff_forward``  — ``GCNdiff.forward``  models/gcndiff.py:101-113 (with
  ``GraAttenLayer`` GraFormer.py:84-96, ``SublayerConnection`` :73-81,
  ``_ResChebGC_diff`` gcndiff.py:39-53, ``_GraphConv`` ChebConv.py:133-151; eval mode,
  dropout = identity)
* ``gcnpose_forward``  — ``GCNpose.forward``  models/gcnpose.py:101-113 (``_ResChebGC``
  ChebConv.py:154-165); ``build_uvxyz`` — runners/diffpose_frame.py:337-342
* ``generalized_steps`` — common/utils_diff.py:46-68
* ``post_process`` / ``mpjpe`` — runners/diffpose_frame.py:382-386, common/loss.py:7-13

It issues the same ATen ops with the same shapes as the reference, so on the
same torch build it reproduces the reference's fp32 results bit for bit
(pinned by ``tests/test_oracle_golden.py`` against fixtures generated from the
reference itself by ``tools/gen_goldens.py``).  It is also the CPU baseline
timed by ``bench.py`` (the reference cannot travel to the GPU box).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# 16 skeleton edges hard-coded by the runner (runners/diffpose_frame.py:120-124)
H36M_EDGES = ((0, 1), (1, 2), (2, 3), (0, 4), (4, 5), (5, 6), (0, 7), (7, 8), (8, 9), (9, 10),
              (8, 11), (11, 12), (12, 13), (8, 14), (14, 15), (15, 16))


def adjacency(num_pts: int = 17, edges=H36M_EDGES) -> torch.Tensor:
    """Dense row-normalised D^-1 (A_sym + I), fp32 (GraFormer.py:32-44, sparse=False)."""
    a = np.zeros((num_pts, num_pts), dtype=np.float32)
    for i, j in edges:
        a[i, j] = 1.0
        a[j, i] = 1.0
    a = a + np.eye(num_pts, dtype=np.float32)
    rowsum = a.sum(1, dtype=np.float32)
    r_inv = np.power(rowsum, -1).astype(np.float32)
    r_inv[np.isinf(r_inv)] = 0.0
    return torch.tensor(r_inv[:, None] * a, dtype=torch.float)


def cheb_basis(graph: torch.Tensor, order: int = 3) -> torch.Tensor:
    """[order, N, N] Chebyshev terms of the normalised Laplacian (ChebConv.py:90-130).

    The reference allocates the terms as fp32 (``torch.float``); an fp64 graph
    keeps fp64 here so the same code serves the fp64 noise-floor study.
    """
    n = graph.size(0)
    dt = torch.float if graph.dtype == torch.float32 else graph.dtype
    d = torch.diag(torch.sum(graph, dim=-1) ** (-1 / 2))
    lap = torch.eye(n, dtype=graph.dtype) - torch.mm(torch.mm(d, graph), d)
    t = torch.zeros([order, n, n], dtype=dt)
    t[0] = torch.eye(n, dtype=dt)
    if order > 1:
        t[1] = lap
    for k in range(2, order):
        t[k] = 2 * torch.mm(lap, t[k - 1]) - t[k - 2]
    return t


def cheb_conv(x: torch.Tensor, graph: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """y = sum_k (T_k x) W_k + b, Laplacian rebuilt per call like the reference (ChebConv.py:74-88)."""
    basis = cheb_basis(graph, weight.shape[0]).unsqueeze(1)     # [K,1,N,N]
    y = torch.matmul(torch.matmul(basis, x), weight)           # [K,B,N,out]
    return torch.sum(y, dim=0) + bias


def swish(x: torch.Tensor) -> torch.Tensor:
    return x * torch.sigmoid(x)                                  # gcndiff.py:35-37


def timestep_embedding(t: torch.Tensor, dim: int, dtype=torch.float32) -> torch.Tensor:
    """Sinusoidal embedding, sin half then cos half (gcndiff.py:15-33); fp32 like the reference."""
    half = dim // 2
    scale = math.log(10000) / (half - 1)
    freqs = torch.exp(torch.arange(half, dtype=dtype) * -scale)
    arg = t.to(dtype)[:, None] * freqs[None, :]
    emb = torch.cat([torch.sin(arg), torch.cos(arg)], dim=1)
    if dim % 2 == 1:
        emb = F.pad(emb, (0, 1, 0, 0))
    return emb


def layer_norm(x: torch.Tensor, gain: torch.Tensor, shift: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    mu = x.mean(-1, keepdim=True)
    sd = x.std(-1, keepdim=True)                                 # unbiased (N-1)
    return gain * (x - mu) / (sd + eps) + shift                 # GraFormer.py:67-70


def multi_head_attention(x: torch.Tensor, mask, lin_w, lin_b, heads: int):
    """4-head self attention over joints; returns (out, p_attn) (GraFormer.py:99-140)."""
    nb = x.size(0)
    dk = x.size(-1) // heads
    if mask is not None:
        mask = mask.unsqueeze(1)
    q, k, v = [F.linear(x, lin_w[j], lin_b[j]).view(nb, -1, heads, dk).transpose(1, 2) for j in range(3)]
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(dk)
    if mask is not None:
        scores = scores.masked_fill(mask == 0, -1e9)
    p = F.softmax(scores, dim=-1)
    o = torch.matmul(p, v).transpose(1, 2).contiguous().view(nb, -1, heads * dk)
    return F.linear(o, lin_w[3], lin_b[3]), p


def graph_laplacian(a_hat: torch.Tensor, nb: int) -> torch.Tensor:
    """Batched D^-1/2 A D^-1/2 with D = column sums + 1e-5 (GraFormer.py:174-178)."""
    a = a_hat.unsqueeze(0).repeat(nb, 1, 1)
    n = a.shape[1]
    d = (torch.sum(a, 1) + 1e-5) ** (-0.5)
    return d.view(nb, n, 1) * a * d.view(nb, 1, n)


def graph_net(x: torch.Tensor, a_hat, w1, b1, w2, b2) -> torch.Tensor:
    """X1 = relu(fc1(L X)); X2 = fc2(L X1)  (GraFormer.py:180-201)."""
    nb = x.size(0)
    h = F.relu(F.linear(torch.bmm(graph_laplacian(a_hat, nb), x), w1, b1))
    return F.linear(torch.bmm(graph_laplacian(a_hat, nb), h), w2, b2)


def gcndiff_forward(p: dict, graph: torch.Tensor, x: torch.Tensor, mask, t: torch.Tensor,
                    n_layers: int = 5, heads: int = 4) -> torch.Tensor:
    """GCNdiff.forward(x, mask, t, cemd) in eval mode (gcndiff.py:101-113)."""
    hid = p["gconv_input.weight"].shape[-1]
    temb = timestep_embedding(t, hid, dtype=p["gconv_input.weight"].dtype)
    temb = F.linear(temb, p["temb.dense.0.weight"], p["temb.dense.0.bias"])
    temb = swish(temb)
    temb = F.linear(temb, p["temb.dense.1.weight"], p["temb.dense.1.bias"])

    out = cheb_conv(x, graph, p["gconv_input.weight"], p["gconv_input.bias"])
    for i in range(n_layers):
        a = f"atten_layers.{i}."
        lw = [p[a + f"self_attn.linears.{j}.weight"] for j in range(4)]
        lb = [p[a + f"self_attn.linears.{j}.bias"] for j in range(4)]
        y = layer_norm(out, p[a + "sublayer.0.norm.a_2"], p[a + "sublayer.0.norm.b_2"])
        out = out + multi_head_attention(y, mask, lw, lb, heads)[0]
        y = layer_norm(out, p[a + "sublayer.1.norm.a_2"], p[a + "sublayer.1.norm.b_2"])
        out = out + graph_net(y, p[a + "feed_forward.A_hat"],
                              p[a + "feed_forward.gconv1.fc.weight"], p[a + "feed_forward.gconv1.fc.bias"],
                              p[a + "feed_forward.gconv2.fc.weight"], p[a + "feed_forward.gconv2.fc.bias"])
        g = f"gconv_layers.{i}."
        h = F.relu(cheb_conv(out, graph, p[g + "gconv1.gconv.weight"], p[g + "gconv1.gconv.bias"]))
        h = h + F.linear(swish(temb), p[g + "temb_proj.weight"], p[g + "temb_proj.bias"])[:, None, :]
        h = F.relu(cheb_conv(h, graph, p[g + "gconv2.gconv.weight"], p[g + "gconv2.gconv.bias"]))
        out = out + h
    return cheb_conv(out, graph, p["gconv_output.weight"], p["gconv_output.bias"])


def gcnpose_forward(p: dict, graph: torch.Tensor, x: torch.Tensor, mask, n_layers: int = 5,
                    heads: int = 4) -> torch.Tensor:
    """GCNpose.forward(x, mask) in eval mode (gcnpose.py:101-113): the GCNdiff backbone without
    the timestep embedding; its blocks are ``_ResChebGC`` (ChebConv.py:154-165):
    x + relu(Cheb2(relu(Cheb1(x))))."""
    out = cheb_conv(x, graph, p["gconv_input.weight"], p["gconv_input.bias"])
    for i in range(n_layers):
        a = f"atten_layers.{i}."
        lw = [p[a + f"self_attn.linears.{j}.weight"] for j in range(4)]
        lb = [p[a + f"self_attn.linears.{j}.bias"] for j in range(4)]
        y = layer_norm(out, p[a + "sublayer.0.norm.a_2"], p[a + "sublayer.0.norm.b_2"])
        out = out + multi_head_attention(y, mask, lw, lb, heads)[0]
        y = layer_norm(out, p[a + "sublayer.1.norm.a_2"], p[a + "sublayer.1.norm.b_2"])
        out = out + graph_net(y, p[a + "feed_forward.A_hat"],
                              p[a + "feed_forward.gconv1.fc.weight"], p[a + "feed_forward.gconv1.fc.bias"],
                              p[a + "feed_forward.gconv2.fc.weight"], p[a + "feed_forward.gconv2.fc.bias"])
        g = f"gconv_layers.{i}."
        h = F.relu(cheb_conv(out, graph, p[g + "gconv1.gconv.weight"], p[g + "gconv1.gconv.bias"]))
        h = F.relu(cheb_conv(h, graph, p[g + "gconv2.gconv.weight"], p[g + "gconv2.gconv.bias"]))
        out = out + h
    return cheb_conv(out, graph, p["gconv_output.weight"], p["gconv_output.bias"])


def build_uvxyz(input_2d: torch.Tensor, xyz: torch.Tensor, test_times: int, root_mode: str = "quirk"):
    """input_uvxyz of test_hyber (runners/diffpose_frame.py:337-342): root handling of the pose
    output, cat with the 2D input, repeat(test_times, 1, 1).  root_mode "quirk" = what the
    reference's in-place subtraction yields on CPU torch (root row zeroed only, golden g5);
    "relative" = xyz - xyz[:, :1]; "raw" = unchanged."""
    if root_mode == "quirk":
        xyz = root_subtract_inplace_quirk(xyz)
    elif root_mode == "relative":
        xyz = xyz - xyz[:, :1, :].clone()
    elif root_mode != "raw":
        raise ValueError(root_mode)
    return torch.cat([input_2d, xyz], dim=2).repeat(test_times, 1, 1)


def alpha_at(b: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """compute_alpha (common/utils_diff.py:40-43)."""
    b = torch.cat([torch.zeros(1, dtype=b.dtype), b], dim=0)
    return (1 - b).cumprod(dim=0).index_select(0, t + 1).view(-1, 1, 1)


def generalized_steps(x: torch.Tensor, mask, seq, eps_fn, b: torch.Tensor, eta: float = 0.0,
                      generator: torch.Generator | None = None, noise: torch.Tensor | None = None):
    """DDIM reverse loop; returns (xs[K+1], x0_preds[K]) (common/utils_diff.py:46-68).  The z of
    step k is ``torch.randn_like(x)`` as in the reference (global RNG, or ``generator``), or
    ``noise[k]`` when a [K, *x.shape] tensor is given."""
    with torch.no_grad():
        n = x.size(0)
        seq = list(seq)
        seq_next = [-1] + seq[:-1]
        xs, x0s = [x], []
        for k, (i, j) in enumerate(zip(reversed(seq), reversed(seq_next))):
            t = torch.ones(n) * i
            tn = torch.ones(n) * j
            at, an = alpha_at(b, t.long()), alpha_at(b, tn.long())
            xt = xs[-1]
            et = eps_fn(xt, mask, t.float())
            x0 = (xt - et * (1 - at).sqrt()) / at.sqrt()
            x0s.append(x0)
            c1 = eta * ((1 - at / an) * (1 - an) / (1 - at)).sqrt()
            c2 = ((1 - an) - c1 ** 2).sqrt()
            if noise is not None:
                z = noise[k].to(x.dtype)
            else:
                z = torch.randn(x.shape, generator=generator) if generator is not None else torch.randn_like(x)
            xs.append(an.sqrt() * x0 + c1 * z + c2 * et)
    return xs, x0s


def params_to_torch(sd) -> dict:
    return {k: torch.as_tensor(np.asarray(v, dtype=np.float32)) for k, v in sd.items()}


def post_process(out_uvxyz: torch.Tensor, test_times: int, num_pts: int = 17) -> torch.Tensor:
    """Hypothesis mean, xyz slice, root-relative (runners/diffpose_frame.py:382-384).

    Uses an explicit clone for the root subtraction; the reference's in-place
    ``x[:, :, :] -= x[:, :1, :]`` aliases (only the root joint is zeroed for
    B>=2) — that quirk is pinned separately by ``root_subtract_inplace_quirk``.
    """
    m = torch.mean(out_uvxyz.reshape(test_times, -1, num_pts, out_uvxyz.shape[-1]), 0)
    xyz = m[:, :, 2:]
    return xyz - xyz[:, :1, :].clone()


def root_subtract_inplace_quirk(x: torch.Tensor) -> torch.Tensor:
    """What the reference's aliased in-place root subtraction yields (diffpose_frame.py:338, :384-385)."""
    y = x.clone()
    y[:, 0, :] = 0
    return y


def mpjpe(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    assert pred.shape == target.shape
    return torch.mean(torch.norm(pred - target, dim=len(target.shape) - 1))   # common/loss.py:7-13
