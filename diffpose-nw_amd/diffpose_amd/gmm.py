"""GMM 2D-keypoint input pipeline on the GPU.

Mirrors ``PoseGenerator_gmm`` (common/generators.py:9-56): the same constructor arguments
(lists of per-sequence arrays, concatenated), ``len()``, and ``ds[index]`` returning the same
6-tuple ``(uvxyz, noise_scale, pose_2d, pose_3d, action, camerapara)``.  The per-joint
component choice — ``np.random.choice(kernel_n, 1, p=w)`` per joint in the reference — runs in
``dpk_gmm_sample`` for a whole batch at once: ``batch(indices)`` returns the collated batch as
device tensors in one launch instead of 17 numpy calls per frame in DataLoader workers.

Random stream: by default the uniforms come from numpy's global RandomState in the order the
reference's ``__getitem__`` consumes them (frame by frame, joint by joint; ``choice`` draws one
``random_sample()`` per call), so a seeded run selects exactly the components the reference
selects.  ``seed=`` uses counter-based uniforms generated on the device instead (same
distribution, no host RNG work; not numpy's stream).
"""
from __future__ import annotations

import ctypes
from functools import reduce

import numpy as np
import torch

from . import _lib

J = 17


def numpy_atol(dtype) -> float:
    """numpy RandomState.choice's tolerance on sum(p) == 1 for weights of ``dtype`` (mtrand.pyx)."""
    atol = float(np.sqrt(np.finfo(np.float64).eps))
    if np.issubdtype(np.dtype(dtype), np.floating):
        atol = max(atol, float(np.sqrt(np.finfo(dtype).eps)))
    return atol


class PoseGeneratorGMM:
    """Device-resident ``PoseGenerator_gmm`` (common/generators.py:9-56)."""

    def __init__(self, poses_3d, poses_2d_gmm, actions, camerapara, device=None):
        assert poses_3d is not None
        p3 = np.concatenate(poses_3d)
        g = np.concatenate(poses_2d_gmm)
        self._actions = reduce(lambda x, y: x + y, actions)
        self._camerapara = np.concatenate(camerapara)
        self._kernel_n = g.shape[2]
        if g.ndim != 4 or g.shape[1] != J or g.shape[3] != 5:
            raise ValueError(f"poses_2d_gmm must be (F,{J},kernel_n,5), got {g.shape}")
        if p3.shape != (g.shape[0], J, 3):
            raise ValueError(f"poses_3d must be ({g.shape[0]},{J},3), got {p3.shape}")
        assert p3.shape[0] == g.shape[0] and p3.shape[0] == len(self._actions)
        self.atol = numpy_atol(g.dtype)
        self.device = torch.device("cuda", 0) if device is None else torch.device(device)
        # on the device in the arrays' own precision: float32, or float64 when either array is float64
        # (numpy's choice runs on double(p) anyway; with float64 poses the root-relative subtraction,
        # generators.py:19, runs in double and only the outputs are rounded, as the reference's .float())
        self._f64 = g.dtype == np.float64 or p3.dtype == np.float64
        dt = np.float64 if self._f64 else np.float32
        self._gmm = torch.from_numpy(np.ascontiguousarray(g, dtype=dt)).to(self.device)
        self._p3 = torch.from_numpy(np.ascontiguousarray(p3, dtype=dt)).to(self.device)
        self._status = torch.zeros(1, dtype=torch.int32, device=self.device)

    def __len__(self):
        return len(self._actions)

    def _src(self, index):
        n = len(self._camerapara)
        return int(index) % n                       # generators.py:26-29

    def batch(self, indices, u=None, seed=None, stream=None):
        """Collated batch for frame ``indices``: (uvxyz [F,17,5], noise_scale [F,17,5], pose_2d
        [F,17,2], pose_3d [F,17,3]) device tensors, plus the actions list and camerapara [F,...]
        (host).  ``u`` [F,17] float64 uniforms, or None to draw them from np.random in the
        reference's order, or ``seed`` for device-generated uniforms."""
        idx = np.asarray(indices, dtype=np.int64).reshape(-1)
        F = idx.size
        uv = torch.empty(F, J, 5, dtype=torch.float32, device=self.device)
        ns = torch.empty(F, J, 5, dtype=torch.float32, device=self.device)
        if F:
            idx_d = torch.from_numpy(idx).to(self.device)
            if seed is None:
                if u is None:
                    u = np.random.random_sample((F, J))      # one draw per choice() call, in order
                u = np.ascontiguousarray(u, dtype=np.float64)
                if u.shape != (F, J):
                    raise ValueError(f"u must be ({F},{J}), got {u.shape}")
                u_d = torch.from_numpy(u).to(self.device)
                u_ptr, s = u_d.data_ptr(), 0
            else:
                u_ptr, s = None, int(seed) & 0xFFFFFFFFFFFFFFFF
            st = torch.cuda.current_stream(self.device) if stream is None else stream
            fn = _lib.lib().dpk_gmm_sample_f64 if self._f64 else _lib.lib().dpk_gmm_sample
            rc = fn(self._gmm.data_ptr(), self._p3.data_ptr(), self._gmm.shape[0],
                                           self._kernel_n, idx_d.data_ptr(), F, u_ptr, s, self.atol,
                                           uv.data_ptr(), ns.data_ptr(), self._status.data_ptr(),
                                           ctypes.c_void_p(st.cuda_stream))
            _lib.check(None, "dpk_gmm_sample", rc)
            flags = int(self._status.item())
            if flags & 1:
                raise ValueError("probabilities are not non-negative")
            if flags & 2:
                raise ValueError("probabilities do not sum to 1")
        srcs = [self._src(i) for i in idx]
        actions = [self._actions[i] for i in srcs]
        cam = torch.from_numpy(self._camerapara[srcs].astype(np.float32)) if F else None
        return uv, ns, uv[..., :2], uv[..., 2:], actions, cam

    def __getitem__(self, index):
        """One frame, as the reference's ``__getitem__`` returns it (CPU tensors)."""
        uv, ns, p2, p3, act, cam = self.batch([index])
        return uv[0].cpu(), ns[0].cpu(), p2[0].cpu(), p3[0].cpu(), act[0], cam[0]
