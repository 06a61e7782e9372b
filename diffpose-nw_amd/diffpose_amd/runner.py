"""Diffpose — the reference runner's evaluation path on the HIP library.

Mirrors ``Diffpose`` in ``runners/diffpose_frame.py``:

| Method | Reference lines | What it does here |
|---|---|---|
| ``__init__`` | 26-58 | src_mask and betas from the config |
| ``create_diffusion_model`` | 118-132 | ``HipGCNdiff`` handle, optional checkpoint |
| ``create_pose_model`` | 134-154 | ``HipGCNpose`` handle, optional checkpoint |
| ``test_hyber`` | 270-420 | pose front-end plus uvxyz assembly (one launch); the K-step DDIM sampler (one launch); per-frame MPJPE / P-MPJPE (one launch); the reference's per-action accounting on the host. Returns (p1, p2) in mm |

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

from . import metrics
from .data import synthetic_eval_batches
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
                              root_mode="quirk")
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

    def test_hyber(self, batches=None, is_train=False, n_frames: int = 4096):
        """Evaluate; returns (p1, p2) = per-action-averaged MPJPE / P-MPJPE in mm."""
        te = self.config.testing
        H = int(te.test_times)
        seq = self._seq()
        self.diffusion_step_count = len(seq)        # runners/diffpose_frame.py:321
        if batches is None:
            batches = synthetic_eval_batches(n_frames, self.config.training.batch_size, seed=self.args.seed)
        root_mode = getattr(self.args, "root_mode", "quirk")
        self.model_diff.eval()
        self.model_pose.eval()
        self.model_diff.set_schedule(seq, self.betas, self.args.eta)
        epoch_p1, epoch_p2 = metrics.AverageMeter(), metrics.AverageMeter()
        err = metrics.define_error_list(metrics.TEST_ACTIONS)
        self.inference_times, self.memory_usage = [], []
        self.pose_times, self.metrics_times = [], []
        track = self.track_metrics
        i = -1
        with torch.no_grad():
            for i, (input_2d, targets_3d, actions) in enumerate(batches):
                input_2d = torch.as_tensor(np.asarray(input_2d, dtype=np.float32)).to(self.device)
                targets_3d = torch.as_tensor(np.asarray(targets_3d, dtype=np.float32)).to(self.device)
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
                                             seed=self.args.seed + i)
                if track:
                    torch.cuda.synchronize(self.device)
                    self.inference_times.append(time.time() - t0)
                    self.memory_usage.append((torch.cuda.max_memory_allocated(self.device) - mem0) / 2 ** 20)
                    tm = time.time()
                p1, p2 = metrics.pose_errors(out, targets_3d, H, root_mode)
                p1h, p2h = p1.cpu().numpy(), p2.cpu().numpy()     # 16 B per frame to the host
                if track:
                    self.metrics_times.append(time.time() - tm)
                n = len(p1h)
                epoch_p1.update(float(np.mean(p1h)) * 1000.0, n)
                epoch_p2.update(float(np.mean(p2h)) * 1000.0, n)
                metrics.test_calculation(p1h, p2h, actions, err)
        if self.track_metrics and self.inference_times:
            # Final computational metrics (runners/diffpose_frame.py:407-409)
            log_dir = getattr(self.args, "log_path", None)
            self.log_performance_metrics(os.path.join(log_dir, "performance_metrics.txt") if log_dir else None)
        logging.info("sum (%d) | MPJPE: %.4f | P-MPJPE: %.4f", i + 1, epoch_p1.avg, epoch_p2.avg)
        self.epoch_loss = (epoch_p1.avg, epoch_p2.avg)
        return metrics.print_error(None, err, is_train)

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
