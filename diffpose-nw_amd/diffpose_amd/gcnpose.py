"""HipGCNpose — the GCNpose 2D->3D front-end as a handle on the HIP library.

Mirrors the reference ``GCNpose(adj, config)`` (``models/gcnpose.py:55-113``, built by
``Diffpose.create_pose_model``, ``runners/diffpose_frame.py:134-154``, which sets
``config.model.coords_dim = [2, 3]``).  Its forward is the GCNdiff backbone without the
timestep embedding, so it runs in the same persistent kernel in a pose mode
(``dpk_pose``).  ``uvxyz`` also performs test_hyber's sampler-input assembly in that launch:
the root subtraction, the concatenation with the 2D input and ``repeat(test_times, 1, 1)``
(``runners/diffpose_frame.py:337-342``).
"""
from __future__ import annotations

import torch

from . import _lib
from .gcndiff import _HipModel, _model_dims
from .weights import POSE_COORDS

ROOT_MODES = {"quirk": 0, "relative": 1, "raw": 2}


def root_mode_id(mode) -> int:
    """'quirk' (default) reproduces the reference's in-place `x[:, :, :] -= x[:, :1, :]` as CPU
    torch executes it: only the root row is zeroed (pinned by golden g5/g6).  'relative' is the
    intended root-relative pose, 'raw' leaves the output alone."""
    if isinstance(mode, int) and mode in ROOT_MODES.values():
        return mode
    try:
        return ROOT_MODES[mode]
    except KeyError:
        raise ValueError(f"root_mode must be one of {sorted(ROOT_MODES)}, got {mode!r}") from None


class HipGCNpose(_HipModel):
    """GCNpose(adj, config) on MI355X.  ``model(input_2d, mask) -> xyz`` like the reference."""

    KIND = "pose"
    DEFAULT_COORDS = POSE_COORDS

    def __init__(self, adj, config=None, device=None):
        coords = _model_dims(config, POSE_COORDS)[4]
        if tuple(coords) != tuple(POSE_COORDS):
            raise NotImplementedError(f"GCNpose is compiled for coords_dim {list(POSE_COORDS)} "
                                      f"(create_pose_model), got {list(coords)}")
        super().__init__(adj, config, device)

    def _launch(self, x2d, mask, xyz, uvxyz, test_times: int, root_mode) -> None:
        self._sync_mask(mask)
        self._check_mask_batch(x2d.shape[0])
        self._note_mask_use()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        L = _lib.lib()
        rc = L.dpk_pose(self._h, x2d.data_ptr(), xyz.data_ptr() if xyz is not None else None,
                        uvxyz.data_ptr() if uvxyz is not None else None, x2d.shape[0], int(test_times),
                        root_mode_id(root_mode), stream)
        _lib.check(self._h, "dpk_pose", rc)

    def forward(self, x, mask=None):
        """xyz = GCNpose(input_2d, mask) (models/gcnpose.py:101-113): (N,17,2) -> (N,17,3)."""
        x = self._check_x(x, channels=2)
        xyz = torch.empty((x.shape[0], self.n_pts, 3), dtype=x.dtype, device=x.device)
        if x.shape[0]:
            self._launch(x, mask, xyz, None, 1, "raw")
        return xyz

    __call__ = forward

    def uvxyz(self, x, mask=None, test_times: int = 1, root_mode="quirk", return_xyz: bool = False):
        """test_hyber's sampler input: cat(input_2d, root-processed GCNpose(input_2d)), repeated
        ``test_times`` times along the batch (hypothesis-major), in one launch."""
        x = self._check_x(x, channels=2)
        if int(test_times) < 1:
            raise ValueError("test_times must be >= 1")
        n = x.shape[0]
        out = torch.empty((int(test_times) * n, self.n_pts, 5), dtype=x.dtype, device=x.device)
        xyz = torch.empty((n, self.n_pts, 3), dtype=x.dtype, device=x.device) if return_xyz else None
        if n:
            self._launch(x, mask, xyz, out, test_times, root_mode)
        return (out, xyz) if return_xyz else out


def GCNpose(adj, config, device=None) -> HipGCNpose:   # noqa: N802  (reference constructor name)
    return HipGCNpose(adj, config, device=device)
