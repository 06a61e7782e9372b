"""Diffpose — the reference runner's evaluation path on the HIP library.

Mirrors ``Diffpose`` in ``runners/diffpose_frame.py``:

| Method | Reference lines | What it does here |
|---|---|---|
| ``__init__`` | 26-58 | src_mask and betas from the config |
| ``create_diffusion_model`` | 118-132 | ``HipGCNdiff`` handle, optional checkpoint |
| ``create_pose_model`` | 134-154 | ``HipGCNpose`` handle, optional checkpoint |
| ``test_hyber`` | 270-420 | pose front-end plus uvxyz assembly (one launch); the K-step DDIM sampler (one launch); per-frame MPJPE / P-MPJPE (one launch); the reference's per-action accounting on the host. Returns (p1, p2) in mm |

Several ranks (``torch.distributed`` initialised with world size > 1, one process per GPU): every
rank reads the same batches, takes the contiguous frame range ``shard_frames(B, world, rank)`` of
each with all ``test_times`` hypothesis rows of those frames, and runs pose, sampler and per-frame
metrics on it alone.  The one collective per batch is the final MPJPE reduction: an all-gather of
the per-frame (MPJPE, P-MPJPE) pairs (16 B per frame, fp64) back into frame order, after which
every rank runs the reference's unchanged accounting over the whole batch and returns the same
(p1, p2) as one process would.  A gather of per-frame values, not per-rank sums: the reference
books a mixed-action batch's P-MPJPE as the whole batch's mean once per frame
(``common/utils.py:136-150``), which per-shard sums cannot reproduce.  With eta > 0 the default
noise source ("torch") draws the reference's randn_like sequence for the whole batch
(``runners/diffpose_frame.py:359``, then one draw per step at ``common/utils_diff.py:65``) and each
rank keeps its rows, so the samples do not depend on the world size either.

The H36M ``.npz`` datasets are absent offline. ``test_hyber`` therefore takes an iterable of
``(input_2d [B,17,2], targets_3d [B,17,3], actions [B])`` batches, the shape the reference's
``PoseGenerator_gmm`` loader delivers after its GMM draw. If none is given, it uses seeded
synthetic batches (``data.synthetic_eval_batches``).

Checkpoints load with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import logging
import os
import time
import types

import numpy as np
import torch

import torch.distributed as dist

from . import metrics
from .data import shard_frames, synthetic_eval_batches
from .dist import gather_frames, shard_rows
from .gcndiff import HipGCNdiff, adj_mx_from_edges
from .gcnpose import HipGCNpose
from .schedule import get_beta_schedule, make_seq
from .weights import load_checkpoint, synthetic_state_dict


def default_config(test_times: int = 1, test_timesteps: int = 50, test_num_diffusion_timesteps: int = 50,
                   num_diffusion_timesteps: int = 51, batch_size: int = 1024):
    """The model / diffusion / testing values of configs/human36m_diffpose_uvxyz_cpn.yml, with the
    testing section set to the BASELINE K=50 configuration by default."""
    ns = types.SimpleNamespace
    return ns(
        model=ns(hid_dim=96, emd_dim=96, coords_dim=[5, 5], num_layer=5, n_head=4, dropout=0.25, n_pts=17),
        diffusion=ns(beta_schedule="linear", beta_start=0.0001, beta_end=0.001,
                     num_diffusion_timesteps=num_diffusion_timesteps),
        training=ns(batch_size=batch_size, num_workers=0),
        testing=ns(test_times=test_times, test_timesteps=test_timesteps,
                   test_num_diffusion_timesteps=test_num_diffusion_timesteps),
        data=ns(dataset="human36m", num_joints=17))


def default_args(**kw):
    a = types.SimpleNamespace(skip_type="uniform", eta=0.0, downsample=1, track_metrics=False, seed=19960903,
                              root_mode="quirk", noise="torch")
    for k, v in kw.items():
        setattr(a, k, v)
    return a


class Diffpose:
    def __init__(self, args, config, device=None):
        self.args = args
        self.config = config
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.src_mask = torch.ones(1, 1, 17, dtype=torch.bool, device=self.device)
        d = config.diffusion
        betas = get_beta_schedule(beta_schedule=d.beta_schedule, beta_start=d.beta_start, beta_end=d.beta_end,
                                  num_diffusion_timesteps=d.num_diffusion_timesteps)
        self.betas = torch.from_numpy(betas).float().to(self.device)
        self.num_timesteps = self.betas.shape[0]
        self.track_metrics = getattr(args, "track_metrics", False)
        self.inference_times, self.memory_usage = [], []
        self.diffusion_step_count = []
        self.model_diff = self.model_pose = None

    def _adj(self):
        return adj_mx_from_edges()        # the runner's 16 H36M edges (diffpose_frame.py:120-125)

    def create_diffusion_model(self, model_path=None, state_dict=None):
        self.model_diff = HipGCNdiff(self._adj(), self.config, device=self.device)
        if model_path:
            self.model_diff.load_state_dict(load_checkpoint(model_path, kind="diff"))
        else:
            self.model_diff.load_state_dict(state_dict if state_dict is not None else synthetic_state_dict())

    def create_pose_model(self, model_path=None, state_dict=None):
        cfg = types.SimpleNamespace(**vars(self.config))
        cfg.model = types.SimpleNamespace(**vars(self.config.model))
        cfg.model.coords_dim = [2, 3]        # diffpose_frame.py:138 (on a copy: no aliasing of config)
        self.model_pose = HipGCNpose(self._adj(), cfg, device=self.device)
        if model_path:
            logging.info("initialize model by:" + model_path)
            self.model_pose.load_state_dict(load_checkpoint(model_path, kind="pose"))
        else:
            logging.info("initialize model randomly")
            self.model_pose.load_state_dict(state_dict if state_dict is not None
                                            else synthetic_state_dict(kind="pose"))

    def _seq(self):
        te = self.config.testing
        return make_seq(self.args.skip_type, te.test_num_diffusion_timesteps, te.test_timesteps)

    @staticmethod
    def _world():
        """(world size, rank, distributed): an initialised torch.distributed job (world size 1
        included: the gather then runs over one rank), else (1, 0, False)."""
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(), dist.get_rank(), True
        return 1, 0, False

    def _batch_noise(self, n_frames: int, H: int, K: int, world: int, rank: int):
        """This rank's rows of the reference's noise draws for one batch, or None (eta = 0, or the
        in-kernel "philox" source).  The reference draws e = randn_like(input_uvxyz) before the
        sampler (runners/diffpose_frame.py:359, unused) and then one randn_like per step
        (common/utils_diff.py:65); all are drawn for the whole batch so every world size sees the
        same numbers, and each rank keeps the rows of its frames (``shard_rows``)."""
        from .utils_diff import draw_noise

        src = getattr(self.args, "noise", "torch")
        if float(self.args.eta) == 0.0 or src in (None, "philox"):
            return None
        full = torch.empty((H * n_frames, 17, 5), dtype=torch.float32, device=self.device)
        draw_noise(full, 1, src)                        # :359's e, consumed and dropped like the reference's
        z = draw_noise(full, K, src)
        if world == 1:
            return z
        return z[:, shard_rows(n_frames, H, world, rank).to(z.device)].contiguous()

    def _frame_errors(self, input_2d, targets_3d, H, seq, i, noise, root_mode):
        """Pose model, sampler and per-frame metrics for one (shard of a) batch: float64 device
        tensors (MPJPE, P-MPJPE) in metres, one per frame.  Also records the reference's per-batch
        timing window under ``track_metrics``."""
        F = input_2d.shape[0]
        if F == 0:
            e = torch.empty(0, dtype=torch.float64, device=self.device)
            return e, e.clone()
        input_2d = torch.as_tensor(input_2d).to(self.device)
        targets_3d = torch.as_tensor(targets_3d).to(self.device)
        track = self.track_metrics
        if track:
            torch.cuda.synchronize(self.device)
            tp = time.time()
        # GCNpose + root handling + cat + repeat(test_times): one launch
        x = self.model_pose.uvxyz(input_2d, self.src_mask, H, root_mode)
        if track:
            # the reference's window (runners/diffpose_frame.py:345-370): memory baseline and
            # start time after the pose model, stop after the sampler and a device sync
            torch.cuda.synchronize(self.device)
            self.pose_times.append(time.time() - tp)
            torch.cuda.reset_peak_memory_stats(self.device)
            mem0 = torch.cuda.memory_allocated(self.device)
            t0 = time.time()
        # generalized_steps(...)[0][-1]: the final sample only (no trajectory stacks)
        out = self.model_diff.sample(x, seq, self.betas, eta=self.args.eta, mask=self.src_mask,
                                     seed=self.args.seed + i, noise=noise)
        if track:
            torch.cuda.synchronize(self.device)
            self.inference_times.append(time.time() - t0)
            self.memory_usage.append((torch.cuda.max_memory_allocated(self.device) - mem0) / 2 ** 20)
            tm = time.time()
        p1, p2 = metrics.pose_errors(out, targets_3d, H, root_mode)
        if track:
            torch.cuda.synchronize(self.device)
            self.metrics_times.append(time.time() - tm)
        return p1, p2

    def test_hyber(self, batches=None, is_train=False, n_frames: int = 4096, frame_errors=None):
        """Evaluate; returns (p1, p2) = per-action-averaged MPJPE / P-MPJPE in mm.  Under a
        multi-rank torch.distributed job every rank returns the whole evaluation's (p1, p2)
        (module docstring).  ``frame_errors`` replaces the per-shard compute (tests of the
        distributed accounting on CPU): ``fn(input_2d, targets_3d, H, seq, batch_index, noise,
        root_mode) -> (p1, p2)`` for the rank's frames."""
        te = self.config.testing
        H = int(te.test_times)
        seq = self._seq()
        self.diffusion_step_count = len(seq)        # runners/diffpose_frame.py:321
        if batches is None:
            batches = synthetic_eval_batches(n_frames, self.config.training.batch_size, seed=self.args.seed)
        root_mode = getattr(self.args, "root_mode", "quirk")
        world, rank, distributed = self._world()
        if frame_errors is None:
            frame_errors = self._frame_errors
            self.model_diff.eval()
            self.model_pose.eval()
            self.model_diff.set_schedule(seq, self.betas, self.args.eta)
        epoch_p1, epoch_p2 = metrics.AverageMeter(), metrics.AverageMeter()
        err = metrics.define_error_list(metrics.TEST_ACTIONS)
        self.inference_times, self.memory_usage = [], []
        self.pose_times, self.metrics_times = [], []
        i = -1
        with torch.no_grad():
            for i, (input_2d, targets_3d, actions) in enumerate(batches):
                actions = list(actions)
                input_2d = np.asarray(input_2d, dtype=np.float32)
                targets_3d = np.asarray(targets_3d, dtype=np.float32)
                B = input_2d.shape[0]
                if targets_3d.shape[0] != B or len(actions) != B:
                    raise ValueError(f"batch {i}: {B} inputs, {targets_3d.shape[0]} targets, {len(actions)} actions")
                lo, hi = shard_frames(B, world, rank)
                noise = self._batch_noise(B, H, len(seq), world, rank)
                p1, p2 = frame_errors(np.ascontiguousarray(input_2d[lo:hi]), np.ascontiguousarray(targets_3d[lo:hi]),
                                      H, seq, i, noise, root_mode)
                if distributed:
                    # the final MPJPE reduction: per-frame (p1, p2) of every rank, in frame order
                    both = gather_frames(torch.stack([p1, p2], dim=1).to(torch.float64), B, 1)
                    p1, p2 = both[:, 0], both[:, 1]
                p1h, p2h = p1.cpu().numpy(), p2.cpu().numpy()     # 16 B per frame to the host
                epoch_p1.update(float(np.mean(p1h)) * 1000.0, B)
                epoch_p2.update(float(np.mean(p2h)) * 1000.0, B)
                metrics.test_calculation(p1h, p2h, actions, err)
        if self.track_metrics and self.inference_times:
            # Final computational metrics (runners/diffpose_frame.py:407-409)
            log_dir = getattr(self.args, "log_path", None)
            path = os.path.join(log_dir, "performance_metrics.txt" if world == 1 else
                                f"performance_metrics_rank{rank}.txt") if log_dir else None
            self.log_performance_metrics(path)
        logging.info("sum (%d) | MPJPE: %.4f | P-MPJPE: %.4f", i + 1, epoch_p1.avg, epoch_p2.avg)
        self.epoch_loss = (epoch_p1.avg, epoch_p2.avg)
        self.action_error_sum = err
        return metrics.print_error(None, err, is_train if rank == 0 else True)   # one table per job

    def log_performance_metrics(self, output_path=None):
        """Summary of the per-batch inference times and peak-memory deltas collected under
        ``args.track_metrics``, logged and (with a path) written in the reference's file format
        (runners/diffpose_frame.py:422-461).  ``inference_times`` cover the sampler call alone,
        between device syncs, as the reference's cover its generalized_steps call (:352-370);
        the pose-model and metrics times of each batch are kept beside them (``pose_times``,
        ``metrics_times``) and appended to the raw data."""
        if not self.track_metrics or not self.inference_times:
            return
        times, mem = self.inference_times, self.memory_usage
        avg_time, max_time, min_time = sum(times) / len(times), max(times), min(times)
        steps_data = f"Diffusion steps: {self.diffusion_step_count}"
        if mem:
            mem_data = f"Memory (MB): avg={sum(mem) / len(mem):.2f}, min={min(mem):.2f}, max={max(mem):.2f}"
        else:
            mem_data = "Memory: not tracked"
        logging.info("=== Performance Summary ===")
        logging.info(f"Time (s): avg={avg_time:.4f}, min={min_time:.4f}, max={max_time:.4f}")
        logging.info(steps_data)
        logging.info(mem_data)
        if output_path:
            with open(output_path, "w") as f:
                f.write("=== Performance Metrics ===\n")
                f.write(f"Time (s): avg={avg_time:.4f}, min={min_time:.4f}, max={max_time:.4f}\n")
                f.write(f"{steps_data}\n")
                f.write(f"{mem_data}\n")
                f.write("\n=== Raw Data ===\n")
                f.write(f"Times: {times}\n")
                f.write(f"Memory: {mem}\n")
                # not in the reference's file: the rest of each batch, outside its timing window
                f.write(f"Pose model times: {getattr(self, 'pose_times', [])}\n")
                f.write(f"Metrics times: {getattr(self, 'metrics_times', [])}\n")
