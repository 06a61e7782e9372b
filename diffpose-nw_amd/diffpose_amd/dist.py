"""Frame-sharded multi-GPU execution of the sampling path.

The reference runs one GPU (``torch.nn.DataParallel`` over a single device,
``runners/diffpose_frame.py:126-127``).  Every pose of the DDIM loop is independent
(no BatchNorm, no cross-pose op), so N GPUs each take a contiguous range of frames —
with all ``test_times`` hypotheses of those frames, keeping the hypothesis mean local
(``runners/diffpose_frame.py:342``, ``:382``) — and run the sampler on it with no
data-path collective.  The one exchange is

* ``gather_frames``: one ``all_gather_into_tensor`` of per-frame rows (hypothesis-major layout
  restored).  The evaluation gathers each frame's (MPJPE, P-MPJPE), 16 B per frame
  (``runner.Diffpose.test_hyber``, ``bench.py``), so every rank books the whole batch with the
  reference's accounting (``common/utils.py:136-150``); per-rank metric sums cannot reproduce its
  P-MPJPE booking, which is why no sum all-reduce is used.

One process per GPU (``torch.distributed`` with backend "nccl" = RCCL on ROCm, "gloo" on
CPU for tests).  Ragged shards are padded to the largest shard for the collective.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .data import shard_frames


def world_info():
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_rows(n_frames: int, hyp: int, world: int, rank: int):
    """Global row indices (hypothesis-major) of ``rank``'s shard: for each hypothesis h, the
    frames [lo, hi) — i.e. the rows ``input_uvxyz.repeat(test_times,1,1)[idx]``."""
    lo, hi = shard_frames(n_frames, world, rank)
    return torch.cat([torch.arange(h * n_frames + lo, h * n_frames + hi) for h in range(hyp)]) if hi > lo \
        else torch.empty(0, dtype=torch.long)


def gather_frames(local: torch.Tensor, n_frames: int, hyp: int, out: torch.Tensor | None = None,
                  group=None) -> torch.Tensor:
    """All-gather every rank's shard of hypothesis-major rows (``hyp`` x local frames) and
    return the global ``[hyp * n_frames, ...]`` tensor in the reference's row order."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_frames(n_frames, world, rank)
    nf = hi - lo
    if local.shape[0] != hyp * nf:
        raise ValueError(f"rank {rank}: expected {hyp * nf} rows, got {local.shape[0]}")
    maxf = -(-n_frames // world)
    tail = tuple(local.shape[1:])
    if nf == maxf:
        send = local.contiguous()
    else:                                       # pad the ragged shard (hypothesis-major blocks)
        send = local.new_zeros((hyp, maxf) + tail)
        send[:, :nf] = local.view((hyp, nf) + tail)
        send = send.view((hyp * maxf,) + tail)
    buf = local.new_empty((world * hyp * maxf,) + tail)
    dist.all_gather_into_tensor(buf, send, group=group)
    buf = buf.view((world, hyp, maxf) + tail)
    if n_frames % world == 0 and hyp == 1 and out is None:
        return buf.view((n_frames,) + tail)
    res = out if out is not None else local.new_empty((hyp * n_frames,) + tail)
    resv = res.view((hyp, n_frames) + tail)
    for r in range(world):
        rlo, rhi = shard_frames(n_frames, world, r)
        resv[:, rlo:rhi] = buf[r, :, : rhi - rlo]
    return res


def max_over_ranks(seconds: float, device=None, group=None) -> float:
    """The slowest rank's elapsed time (bench timing contract)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
