"""GPU, RCCL: the multi-GPU path of bench.py / diffpose_amd.dist on a one-GPU box.

The scaling sweep (N = 1, 2, 4, 8) is the driver's to run; what a one-GPU box can check is
that the same code runs over the "nccl" backend (RCCL) at world size 1 as launched by
torch.distributed.run: process-group init on the device, the barrier + max-over-ranks timing,
and the per-step all_gather_into_tensor of the final poses (hypothesis-major reassembly,
padded ragged shards).  The world-2 logic itself is covered on CPU over gloo
(test_dist_gloo.py).  Both checks run in child processes (fresh interpreter per rank).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "diffpose-nw_amd"), ROOT, env.get("PYTHONPATH", "")])
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def test_bench_under_launcher_runs_rccl_path():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
           "--frames", "130", "--no-cpu", "--no-variants"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 1 and res["steps"] == 2 and res["value"] > 0
    assert "RCCL all_gather" in res["config"]["parallelism"]
    assert res["roofline"]["launches"] == 2


_GATHER = r"""
import os, torch, torch.distributed as dist
from diffpose_amd import dist as D
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
for n_frames, hyp in ((7, 1), (130, 3)):
    local = torch.randn(hyp * n_frames, 17, 5, device=dev)
    g = D.gather_frames(local, n_frames, hyp)
    assert g.shape == local.shape and torch.equal(g, local), (n_frames, hyp)
assert D.max_over_ranks(0.25, device=dev) == 0.25
dist.barrier()
dist.destroy_process_group()
print("GATHER_OK")
"""


def test_gather_frames_over_rccl_world1():
    env = _env()
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", _GATHER], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "GATHER_OK" in r.stdout


_HYBER = r"""
import torch, torch.distributed as dist
from diffpose_amd import runner as R
from diffpose_amd.data import synthetic_eval_batches
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)

def run(eta):
    cfg = R.default_config(test_times=2, test_timesteps=10, test_num_diffusion_timesteps=50, batch_size=96)
    d = R.Diffpose(R.default_args(eta=eta), cfg, device=dev)
    d.create_diffusion_model()
    d.create_pose_model()
    torch.manual_seed(3)
    p = d.test_hyber(batches=list(synthetic_eval_batches(300, 96, seed=9)), is_train=1)
    acc = {a: (v["p1"].sum, v["p1"].count, v["p2"].sum, v["p2"].count) for a, v in d.action_error_sum.items()}
    return p, acc, d.epoch_loss

plain = {eta: run(eta) for eta in (0.0, 0.5)}          # one process, no collective
dist.init_process_group("nccl", device_id=dev)
for eta in (0.0, 0.5):
    got = run(eta)                                       # the distributed path: per-frame all-gather over RCCL
    assert got == plain[eta], (eta, got[0], plain[eta][0])
assert plain[0.5][0] != plain[0.0][0]
dist.destroy_process_group()
print("HYBER_OK", plain[0.0][0], plain[0.5][0])
"""


def test_runner_test_hyber_over_rccl_world1_equals_plain_run():
    """runner.Diffpose.test_hyber through its distributed code (frame shard, pose + sampler +
    per-frame metrics, the RCCL all-gather of per-frame (p1, p2), the unchanged accounting) at
    world size 1 gives exactly the plain single-process result, at eta 0 and at eta 0.5 with the
    reference's per-step randn_like draws (runners/diffpose_frame.py:330-420)."""
    env = _env()
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", _HYBER], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "HYBER_OK" in r.stdout
    print(r.stdout.strip().splitlines()[-1])
