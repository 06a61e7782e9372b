"""Evaluation of the sampler output: per-frame MPJPE / P-MPJPE on the GPU (``dpk_pose_metrics``)
and the reference's per-action accounting on the host.

Reference: test_hyber (``runners/diffpose_frame.py:377-420``) does the following per batch:
- takes the hypothesis mean and subtracts the root;
- ``epoch_loss_3d_pos.update(mpjpe(...))`` with ``common/loss.py:7-13``;
- ``epoch_loss_3d_pos_procrustes.update(p_mpjpe(...))`` with ``common/loss.py:25-64``, on host numpy;
- ``test_calculation`` → ``mpjpe_by_action_p1/_p2`` (``common/utils.py:96-152``), then
  ``print_error`` (``common/utils.py:241-271``) returns (p1, p2) in mm.

Here the per-frame errors come from one HIP kernel, which returns 2 doubles per frame to the
host. The accounting below consumes them with the reference's exact bookkeeping, quirks included:
- a batch whose action strings are all identical is booked in one update;
- a mixed batch books P-MPJPE as the *batch* mean once per frame;
- actions never seen still enter the final average with 0.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .gcnpose import root_mode_id

# runners/diffpose_frame.py:374-375
TEST_ACTIONS = ["Directions", "Discussion", "Eating", "Greeting", "Phoning", "Photo", "Posing", "Purchases",
                "Sitting", "SittingDown", "Smoking", "Waiting", "WalkDog", "Walking", "WalkTogether"]


def pose_errors(out_uvxyz: torch.Tensor, targets: torch.Tensor, test_times: int = 1, root_mode="quirk",
                return_xyz: bool = False):
    """Per-frame (MPJPE, P-MPJPE) in metres, float64 device tensors of length F, for a sampler
    output ``[test_times*F,17,5]`` (hypothesis-major) and ``targets_3d [F,17,3]``."""
    for name, t in (("out_uvxyz", out_uvxyz), ("targets", targets)):
        if not (torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float32):
            raise TypeError(f"{name} must be a float32 CUDA(HIP) tensor")
    H = int(test_times)
    if H < 1 or out_uvxyz.dim() != 3 or out_uvxyz.shape[1:] != (17, 5) or out_uvxyz.shape[0] % H:
        raise ValueError(f"out_uvxyz must be (test_times*F, 17, 5), got {tuple(out_uvxyz.shape)}")
    F = out_uvxyz.shape[0] // H
    if targets.shape != (F, 17, 3):
        raise ValueError(f"targets must be ({F}, 17, 3), got {tuple(targets.shape)}")
    if targets.device != out_uvxyz.device:
        raise ValueError("out_uvxyz and targets must be on the same device")
    out_uvxyz, targets = out_uvxyz.contiguous(), targets.contiguous()
    dev = out_uvxyz.device
    p1 = torch.empty(F, dtype=torch.float64, device=dev)
    p2 = torch.empty(F, dtype=torch.float64, device=dev)
    xyz = torch.empty((F, 17, 3), dtype=torch.float32, device=dev) if return_xyz else None
    stream = torch.cuda.current_stream(dev).cuda_stream
    rc = _lib.lib().dpk_pose_metrics(out_uvxyz.data_ptr(), targets.data_ptr(), F, H, root_mode_id(root_mode),
                                     p1.data_ptr(), p2.data_ptr(), xyz.data_ptr() if xyz is not None else None,
                                     stream)
    _lib.check(None, "dpk_pose_metrics", rc)
    return (p1, p2, xyz) if return_xyz else (p1, p2)


class AverageMeter:
    """common/utils.py:9-24 (sum += val * n)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class AccumLoss:
    """common/utils.py:212-223 (sum += val; note: not val * n)."""

    def __init__(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val
        self.count += n
        self.avg = self.sum / self.count


def define_actions(action):
    """common/utils.py:190-203."""
    if action in ("All", "all", "*"):
        return list(TEST_ACTIONS)
    if action not in TEST_ACTIONS:
        raise ValueError(f"Unrecognized action: {action}")
    return [action]


def define_error_list(actions):
    """common/utils.py:206-209."""
    return {a: {"p1": AccumLoss(), "p2": AccumLoss()} for a in actions}


def action_name(a: str) -> str:
    """Action label up to the first space ('Walking 1' -> 'Walking'), common/utils.py:110-114."""
    i = a.find(" ")
    return a[:i] if i != -1 else a


def test_calculation(p1, p2, actions, error_sum, n_joints: int = 17):
    """The bookkeeping of common/utils.py:96-152 for one batch, from per-frame MPJPE ``p1`` and
    P-MPJPE ``p2`` (metres; host arrays or device tensors)."""
    p1 = p1.detach().cpu().numpy() if torch.is_tensor(p1) else np.asarray(p1, dtype=np.float64)
    p2 = p2.detach().cpu().numpy() if torch.is_tensor(p2) else np.asarray(p2, dtype=np.float64)
    actions = list(actions)
    b = len(actions)
    if p1.shape != (b,) or p2.shape != (b,):
        raise ValueError("one action label per frame")
    if b == 0:
        return error_sum
    single = len(set(actions)) == 1
    if single:
        name = action_name(actions[0])
        error_sum[name]["p1"].update(float(np.mean(p1)) * b * n_joints, b * n_joints)
        error_sum[name]["p2"].update(float(np.mean(p2)) * b, b)
    else:
        m2 = float(np.mean(p2))
        for i in range(b):
            name = action_name(actions[i])
            error_sum[name]["p1"].update(float(p1[i]) * n_joints, n_joints)
            error_sum[name]["p2"].update(m2, 1)       # the reference books the batch mean per frame
    return error_sum


def print_error(data_type, action_error_sum, is_train):
    """common/utils.py:241-271: per-action table (printed when is_train == 0) and the mean over
    all listed actions, in mm."""
    all_p1, all_p2 = AccumLoss(), AccumLoss()
    if is_train == 0:
        print("{0:=^12} {1:=^10} {2:=^8}".format("Action", "p#1 mm", "p#2 mm"))
    for action, v in action_error_sum.items():
        e1, e2 = v["p1"].avg * 1000.0, v["p2"].avg * 1000.0
        all_p1.update(e1, 1)
        all_p2.update(e2, 1)
        if is_train == 0:
            print("{0:<12} {1:>6.2f} {2:>10.2f}".format(action, e1, e2))
    if is_train == 0:
        print("{0:<12} {1:>6.2f} {2:>10.2f}".format("Average", all_p1.avg, all_p2.avg))
    return all_p1.avg, all_p2.avg
