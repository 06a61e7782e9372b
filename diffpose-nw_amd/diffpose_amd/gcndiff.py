"""HipGCNdiff — the GCNdiff denoiser as a handle on the HIP library.

Mirrors the reference model's construction and call surface
(``GCNdiff(adj, config)``, ``load_state_dict(states[0])``, ``model(x, mask, t, cemd)``;
reference ``models/gcndiff.py:55-113``, ``runners/diffpose_frame.py:118-132``) so a
caller can swap it in for the DataParallel-wrapped torch module at inference.
All compute runs in libdpk.so on the GPU; torch is used only for device memory
and the current stream.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .schedule import alpha_bar_table
from .weights import HID, N_HEAD, N_LAYERS, N_PTS, COORDS, normalize_state_dict

# 16 skeleton edges of the runner (runners/diffpose_frame.py:120-124)
H36M_EDGES = ((0, 1), (1, 2), (2, 3), (0, 4), (4, 5), (5, 6), (0, 7), (7, 8), (8, 9), (9, 10),
              (8, 11), (11, 12), (12, 13), (8, 14), (14, 15), (15, 16))


def adj_mx_from_edges(num_pts: int = N_PTS, edges=H36M_EDGES) -> np.ndarray:
    """Row-normalised D^-1 (A_sym + I) as float32 (reference models/GraFormer.py:32-44, sparse=False)."""
    a = np.zeros((num_pts, num_pts), dtype=np.float32)
    for i, j in np.asarray(edges, dtype=np.int64).reshape(-1, 2):
        a[i, j] = 1.0
        a[j, i] = 1.0
    a += np.eye(num_pts, dtype=np.float32)
    inv = np.power(a.sum(1, dtype=np.float32), -1).astype(np.float32)
    inv[np.isinf(inv)] = 0.0
    return (inv[:, None] * a).astype(np.float32)


def _f32p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _dev_index(device) -> int:
    if device is None:
        return torch.cuda.current_device()
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"HipGCNdiff runs on a HIP device, got {d}")
    return torch.cuda.current_device() if d.index is None else d.index


def _model_dims(config, default_coords=COORDS):
    if config is None:
        return HID, N_LAYERS, N_HEAD, N_PTS, tuple(default_coords)
    m = getattr(config, "model", config)
    return (int(m.hid_dim), int(m.num_layer), int(m.n_head), int(m.n_pts), tuple(int(c) for c in m.coords_dim))


class _HipModel:
    """A libdpk handle for one model (graph, weights, key mask) on one HIP device."""

    KIND = "diff"
    DEFAULT_COORDS = COORDS

    def __init__(self, adj, config=None, device=None):
        hid, nl, nh, npts, coords = _model_dims(config, self.DEFAULT_COORDS)
        self.device = torch.device("cuda", _dev_index(device))
        L = _lib.lib()
        cfg = _lib.DpkConfig(hid, nl, nh, npts, coords[0], coords[1], self.device.index)
        h = ctypes.c_void_p()
        rc = L.dpk_create(ctypes.byref(cfg), ctypes.byref(h))
        _lib.check(None, "dpk_create", rc)
        self._h = h
        self.n_pts = npts
        self.num_layer = nl
        self.hid_dim = hid
        self.n_head = nh
        self.coords_dim = tuple(coords)
        adj = adj.detach().cpu().numpy() if torch.is_tensor(adj) else np.asarray(adj)
        self.adj = np.ascontiguousarray(adj, dtype=np.float32)
        if self.adj.shape != (npts, npts):
            raise ValueError(f"adj must be ({npts},{npts}), got {self.adj.shape}")
        _lib.check(h, "dpk_set_graph", L.dpk_set_graph(h, _f32p(self.adj)))
        self._mask_key = None
        self._mask_ref = None
        self._pose_bits = None       # per-pose key masks (device int32 words), kept alive while bound
        self._mask_hold = []         # per-pose mask arrays a captured graph reads (kept until close)
        self._sched_key = None
        self.training = False

    # -- nn.Module-like surface -------------------------------------------------------
    def load_state_dict(self, state_dict, strict: bool = True):
        """Accept the reference's states[0] (with/without 'module.'), torch tensors or numpy."""
        sd = normalize_state_dict(state_dict, kind=self.KIND, n_layers=self.num_layer, hid=self.hid_dim,
                                  n_pts=self.n_pts, coords=self.coords_dim)
        names = list(sd.keys())
        arrs = [np.ascontiguousarray(sd[k], dtype=np.float32) for k in names]
        c_names = (ctypes.c_char_p * len(names))(*[k.encode() for k in names])
        c_ptrs = (ctypes.POINTER(ctypes.c_float) * len(arrs))(*[_f32p(a) for a in arrs])
        c_num = (ctypes.c_int64 * len(arrs))(*[a.size for a in arrs])
        L = _lib.lib()
        _lib.check(self._h, "dpk_load_weights", L.dpk_load_weights(self._h, c_names, c_ptrs, c_num, len(arrs)))
        self._state = sd
        return self

    def eval(self):
        self.training = False
        return self

    def train(self, mode: bool = True):
        if mode:
            raise NotImplementedError(f"{type(self).__name__} is inference-only (training is out of scope, "
                                      "SURVEY §8f f4)")
        return self.eval()

    def to(self, *a, **k):
        return self

    def cuda(self, *a, **k):
        return self

    def parameters(self):
        return iter(())

    # -- mask -----------------------------------------------------------------------
    def set_mask(self, mask) -> None:
        """Key mask as the reference's ``masked_fill(mask == 0, -1e9)`` (models/GraFormer.py:107-108):
        one mask for every pose ((1,1,17) as runners/diffpose_frame.py:39-40 builds it, or any 17
        entries), or one per pose ((N,1,17), broadcast over heads and queries like the reference's
        ``mask.unsqueeze(1)``; the next call's batch must then have N poses)."""
        L = _lib.lib()
        if torch.is_tensor(mask) or isinstance(mask, np.ndarray):
            shape = tuple(mask.shape)
            if len(shape) == 3 and shape[0] != 1:
                if shape[1:] != (1, self.n_pts):
                    raise ValueError(f"a per-pose mask must be (N, 1, {self.n_pts}), got {shape}")
                mt = torch.as_tensor(mask).to(self.device)
                words = (mt.reshape(shape[0], self.n_pts) != 0).to(torch.int32)
                shifts = torch.arange(self.n_pts, device=self.device, dtype=torch.int32)
                bits = (words << shifts).sum(dim=1, dtype=torch.int32).contiguous()
                _lib.check(self._h, "dpk_set_pose_masks", L.dpk_set_pose_masks(self._h, bits.data_ptr(), shape[0]))
                self._pose_bits = bits
                return
        if mask is None:
            m = np.ones(self.n_pts, dtype=np.uint8)
        else:
            mt = mask.detach().cpu() if torch.is_tensor(mask) else torch.as_tensor(np.asarray(mask))
            m = mt.reshape(-1).numpy().astype(np.uint8)
            if m.size != self.n_pts:
                raise ValueError(f"mask must have {self.n_pts} key entries, got {m.size}")
        m = np.ascontiguousarray(m)
        _lib.check(self._h, "dpk_set_mask", L.dpk_set_mask(self._h, m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        if self._pose_bits is not None:
            _lib.check(self._h, "dpk_set_pose_masks", L.dpk_set_pose_masks(self._h, None, 0))
            self._pose_bits = None

    def _check_mask_batch(self, n: int) -> None:
        """A per-pose mask broadcasts only against a batch of its own size (torch broadcasting)."""
        if self._pose_bits is not None and self._pose_bits.numel() != n:
            raise ValueError(f"per-pose mask has {self._pose_bits.numel()} poses, the batch {n}")

    def _note_mask_use(self) -> None:
        """Before a launch that reads the per-pose mask array by address (dpk_set_pose_masks):
        a captured launch keeps that address for the graph's life, so the array is held until
        close(); an eager launch on another stream than the one that allocated it must not see
        the caching allocator hand the memory out again while it runs (record_stream)."""
        bits = self._pose_bits
        if bits is None:
            return
        if torch.cuda.is_current_stream_capturing():
            if not any(b is bits for b in self._mask_hold):
                self._mask_hold.append(bits)
        else:
            bits.record_stream(torch.cuda.current_stream(self.device))

    def _sync_mask(self, mask) -> None:
        """Upload the key mask when it changed.  Cached by object identity + in-place version;
        the cached object is kept alive so its id cannot be recycled by a new tensor."""
        key = None if mask is None else (id(mask), getattr(mask, "_version", 0))
        if key is None or key != self._mask_key or mask is not self._mask_ref:
            self.set_mask(mask)
            self._mask_key = key
            self._mask_ref = mask

    def _check_x(self, x, channels: int | None = None):
        channels = self.coords_dim[0] if channels is None else channels
        if not (torch.is_tensor(x) and x.is_cuda and x.dtype == torch.float32):
            raise TypeError("x must be a float32 CUDA(HIP) tensor")
        if x.dim() != 3 or x.shape[1] != self.n_pts or x.shape[2] != channels:
            raise ValueError(f"x must be (N, {self.n_pts}, {channels}), got {tuple(x.shape)}")
        if x.device != self.device:
            raise ValueError(f"x on {x.device}, model on {self.device}")
        return x.contiguous()

    GEMM_MODES = {"fp32": 0, "f16x3": 1, "bf16": 2}

    def set_gemm_mode(self, mode: str = "fp32") -> None:
        """Arithmetic of the per-layer GEMMs (see dpk_set_gemm_mode): "fp32" (default, fp32 MFMA)
        "f16x3" (3-term fp16-split MFMA, fp32 accumulate) or "bf16" (bf16 operands, fp32
        accumulate: reduced precision, for the tolerance study).  Not a reference option: the
        reference runs fp32 throughout, and "fp32" is what its parity is pinned on."""
        if mode not in self.GEMM_MODES:
            raise ValueError(f"gemm mode must be one of {sorted(self.GEMM_MODES)}, got {mode!r}")
        _lib.check(self._h, "dpk_set_gemm_mode", _lib.lib().dpk_set_gemm_mode(self._h, self.GEMM_MODES[mode]))
        self.gemm_mode = mode

    TAIL_PLANS = {"four": 0, "two_pose": 1, "step_split": 2}

    def set_tail_plan(self, plan: str = "step_split") -> None:
        """How a partial last round of 4-pose tiles runs (see dpk_set_tail_plan): "step_split"
        (default: its tiles' K steps split over two CUs, bitwise equal to "four"), "two_pose"
        (a round of 2-pose tiles) or "four" (a round of 4-pose tiles).  Scheduling only: the
        reference has no tiles."""
        if plan not in self.TAIL_PLANS:
            raise ValueError(f"tail plan must be one of {sorted(self.TAIL_PLANS)}, got {plan!r}")
        _lib.check(self._h, "dpk_set_tail_plan", _lib.lib().dpk_set_tail_plan(self._h, self.TAIL_PLANS[plan]))

    def debug_split(self, mode: int = 0, read: bool = False):
        """Test hook (dpk_debug_split): set the step-split handoff mode; with ``read``, wait for the
        device and return the number of second halves that recomputed their first half's steps."""
        n = ctypes.c_int(0)
        _lib.check(self._h, "dpk_debug_split",
                   _lib.lib().dpk_debug_split(self._h, int(mode), ctypes.byref(n) if read else None))
        return n.value if read else None

    def debug_resources(self) -> dict:
        """Test hook (dpk_debug_resources): capture-owned resources and free flag slots."""
        buf = (ctypes.c_int * 8)()
        _lib.check(self._h, "dpk_debug_resources", _lib.lib().dpk_debug_resources(self._h, buf, 8))
        keys = ("captures", "tracked", "released", "free_slots", "retired_schedules", "eps_spare_poses",
                "generic_loop_graphs", "generic_spare_kib")
        return dict(zip(keys, list(buf)))

    def profile(self, enable: bool = True) -> None:
        """Bracket each model-kernel launch with HIP events (see dpk_profile)."""
        _lib.check(self._h, "dpk_profile", _lib.lib().dpk_profile(self._h, 1 if enable else 0))

    def kernel_times_ms(self):
        """Wait for and return the recorded kernel durations (ms), oldest first."""
        L = _lib.lib()
        cap = 4096
        buf = (ctypes.c_float * cap)()
        n = ctypes.c_int()
        _lib.check(self._h, "dpk_profile_read", L.dpk_profile_read(self._h, buf, cap, ctypes.byref(n)))
        return [buf[i] for i in range(min(n.value, cap))]

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            _lib.lib().dpk_destroy(h)
        self._mask_hold = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HipGCNdiff(_HipModel):
    """GCNdiff(adj, config) on MI355X.  ``model(x, mask, t, cemd) -> eps`` like the reference."""

    # -- schedule -------------------------------------------------------------------
    def set_schedule(self, seq, betas, eta: float = 0.0) -> None:
        """Bind seq / betas / eta (cached: re-uploaded only when they change)."""
        b = betas.detach().cpu().numpy() if torch.is_tensor(betas) else np.asarray(betas)
        b = np.ascontiguousarray(b, dtype=np.float32)
        seq = [int(s) for s in seq]
        key = (tuple(seq), b.tobytes(), float(eta))
        if key == self._sched_key:
            return
        abar = np.ascontiguousarray(alpha_bar_table(b))
        cseq = (ctypes.c_int * len(seq))(*seq)
        L = _lib.lib()
        _lib.check(self._h, "dpk_set_schedule",
                   L.dpk_set_schedule(self._h, _f32p(abar), abar.size, cseq, len(seq), ctypes.c_float(eta)))
        self._sched_key = key
        self.K = len(seq)

    # -- compute --------------------------------------------------------------------
    def forward(self, x, mask, t, cemd=0):
        """eps = GCNdiff(x, mask, t) (models/gcndiff.py:101-113); ``cemd`` is unused there too."""
        x = self._check_x(x)
        n = x.shape[0]
        t = torch.as_tensor(t, device=self.device).to(torch.float32).reshape(-1).contiguous()
        if t.numel() == 1 and n != 1:
            t = t.expand(n).contiguous()
        if t.numel() != n:
            raise ValueError(f"t must have {n} entries, got {t.numel()}")
        self._sync_mask(mask)
        self._check_mask_batch(n)
        self._note_mask_use()
        eps = torch.empty_like(x)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        L = _lib.lib()
        _lib.check(self._h, "dpk_eps", L.dpk_eps(self._h, x.data_ptr(), t.data_ptr(), eps.data_ptr(), n, stream))
        return eps

    __call__ = forward

    def sample(self, x, seq, betas, eta: float = 0.0, mask=None, seed: int = 0, trajectory: bool = False,
               out=None, noise=None):
        """Run the whole DDIM loop on device.  Returns the final x, or (xs, x0s) stacks
        ([K+1,N,17,5], [K,N,17,5]) when ``trajectory`` is set.  ``noise``: None (counter-based
        draws from ``seed`` when eta > 0) or a [K,N,17,5] float32 device tensor whose slice k is the
        z of the k-th executed step (the reference's per-step ``torch.randn_like(x)``,
        common/utils_diff.py:65; see ``utils_diff.draw_noise``)."""
        x = self._check_x(x)
        self.set_schedule(seq, betas, eta)
        if noise is not None:
            shape = (self.K,) + tuple(x.shape)
            if not (torch.is_tensor(noise) and noise.is_cuda and noise.dtype == torch.float32
                    and tuple(noise.shape) == shape and noise.device == x.device):
                raise ValueError(f"noise must be a float32 tensor of shape {shape} on {x.device}")
            noise = noise.contiguous()
        self._sync_mask(mask)
        n = x.shape[0]
        self._check_mask_batch(n)
        self._note_mask_use()
        out = torch.empty_like(x) if out is None else out
        xs = x0s = None
        if trajectory:
            xs = torch.empty((self.K + 1,) + tuple(x.shape), dtype=x.dtype, device=x.device)
            x0s = torch.empty((self.K,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        L = _lib.lib()
        xs_p = xs.data_ptr() if xs is not None else None
        x0s_p = x0s.data_ptr() if x0s is not None else None
        seed_c = ctypes.c_uint64(seed & (2**64 - 1))
        if noise is None:
            rc = L.dpk_sample(self._h, x.data_ptr(), out.data_ptr(), xs_p, x0s_p, n, seed_c, stream)
        else:
            rc = L.dpk_sample_noise(self._h, x.data_ptr(), out.data_ptr(), xs_p, x0s_p, n, seed_c,
                                    noise.data_ptr(), stream)
        _lib.check(self._h, "dpk_sample", rc)
        if trajectory:
            return xs, x0s
        return out

    def ddim_update(self, xt, et, step: int, seed: int = 0, want_x0: bool = True, noise=None):
        """x_{t-1} (and x0) from an external eps for schedule step ``step``; ``noise``: this step's
        draw z (shaped like xt, on its device) or None (counter-based from ``seed``)."""
        xt, et = xt.contiguous(), et.contiguous()
        if noise is not None:
            if not (torch.is_tensor(noise) and noise.dtype == torch.float32 and noise.shape == xt.shape
                    and noise.device == xt.device):
                raise ValueError(f"noise must be a float32 tensor shaped like xt {tuple(xt.shape)} on {xt.device}")
            noise = noise.contiguous()
        xn = torch.empty_like(xt)
        x0 = torch.empty_like(xt) if want_x0 else None
        stream = torch.cuda.current_stream(xt.device).cuda_stream
        L = _lib.lib()
        rc = L.dpk_ddim_update_noise(self._h, xt.data_ptr(), et.data_ptr(), xn.data_ptr(),
                                     x0.data_ptr() if x0 is not None else None, xt.numel(), step,
                                     ctypes.c_uint64(seed & (2**64 - 1)),
                                     noise.data_ptr() if noise is not None else None, stream)
        _lib.check(self._h, "dpk_ddim_update", rc)
        return xn, x0



def GCNdiff(adj, config, device=None) -> HipGCNdiff:   # noqa: N802  (reference constructor name)
    return HipGCNdiff(adj, config, device=device)
