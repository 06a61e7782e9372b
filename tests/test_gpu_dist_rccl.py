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
s = D.allreduce_sums([1.5, 2.0, 3.0], device=dev)
assert s.tolist() == [1.5, 2.0, 3.0]
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
