"""Synthetic Human3.6M-shaped sampler inputs (the H36M .npz files are absent offline).

Shapes follow ``test_hyber`` (reference ``runners/diffpose_frame.py:330-343``):
``input_uvxyz`` = cat(2D uv, pose-model xyz) of shape (B, 17, 5), repeated
``test_times`` times along the batch (hypothesis-major), and ``targets_3d``
(B, 17, 3) root-relative.

Distributions: uv ~ N(0, 0.3^2) clipped to [-1, 1] (normalised
screen coordinates, ``common/camera.py:10-14``); xyz ~ N(0, 0.25^2) metres with
the root joint at 0; targets = xyz + N(0, 0.05^2), root-relative.
Drawn with NumPy PCG64 so every host reproduces the same batch.
"""
from __future__ import annotations

import numpy as np

DEFAULT_SEED = 19960903


def synthetic_batch(n_frames: int, seed: int = DEFAULT_SEED, num_pts: int = 17):
    """Return (uvxyz (B,17,5) f32, targets_3d (B,17,3) f32) for B = n_frames."""
    rng = np.random.Generator(np.random.PCG64(seed))
    uv = np.clip(rng.normal(0.0, 0.3, size=(n_frames, num_pts, 2)), -1.0, 1.0)
    xyz = rng.normal(0.0, 0.25, size=(n_frames, num_pts, 3))
    xyz[:, 0, :] = 0.0
    tgt = xyz + rng.normal(0.0, 0.05, size=xyz.shape)
    tgt = tgt - tgt[:, :1, :]
    x = np.concatenate([uv, xyz], axis=2).astype(np.float32)
    return np.ascontiguousarray(x), np.ascontiguousarray(tgt.astype(np.float32))


def shard_frames(n_frames: int, world: int, rank: int):
    """Contiguous frame range [lo, hi) of ``rank`` (all hypotheses of a frame stay together)."""
    base, rem = divmod(n_frames, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def repeat_hypotheses(x: np.ndarray, test_times: int) -> np.ndarray:
    """``input_uvxyz.repeat(test_times,1,1)`` — hypothesis-major rows (diffpose_frame.py:342)."""
    return np.ascontiguousarray(np.tile(x, (test_times, 1, 1)))


def synthetic_eval_batches(n_frames: int, batch_size: int, seed: int = DEFAULT_SEED):
    """Yield (input_2d [B,17,2], targets_3d [B,17,3], actions [B]) like test_hyber's loader
    (runners/diffpose_frame.py:278-283, shuffle=False, so frames arrive grouped by action and
    most batches hold a single action string; batches at a boundary mix two)."""
    from .metrics import TEST_ACTIONS

    x, tgt = synthetic_batch(n_frames, seed=seed)
    acts = np.array([f"{TEST_ACTIONS[(f * len(TEST_ACTIONS)) // max(n_frames, 1)]} 1" for f in range(n_frames)])
    for lo in range(0, n_frames, batch_size):
        hi = min(lo + batch_size, n_frames)
        yield np.ascontiguousarray(x[lo:hi, :, :2]), tgt[lo:hi], [str(a) for a in acts[lo:hi]]
