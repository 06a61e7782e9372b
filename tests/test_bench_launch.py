"""CPU: `python bench.py --gpus N` starts N ranks itself (verdict r01 item 1), reports
n_gpus = N and reassembles the frame-sharded batch through the all-gather, using the
--cpu-dry rehearsal (gloo, an elementwise stub in place of the HIP sampler — no oracle, no GPU).
The reference runs one DataParallel replica (runners/diffpose_frame.py:126-127); this is the
launcher for the frame-sharded replacement."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.parametrize("extra,scaling,frames_total", [
    (["--frames", "8"], "weak", 16),                        # config 2/4 shape: frames per GPU
    (["--config", "5", "--total-frames", "7"], "strong", 7),  # config 5 shape: ragged split, H=20
])
def test_bench_spawns_ranks_and_reassembles(extra, scaling, frames_total):
    rc, line, err = _run(["--gpus", "2", "--cpu-dry", "--steps", "2", "--warmup", "1"] + extra)
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2
    assert line["scaling"] == scaling
    assert line["config"]["frames_total"] == frames_total
    assert line["reassembly_ok"] is True
    assert len(line["per_rank_ms"]) == 2
    assert line["allgather_ms"] > 0


def test_bench_refuses_world_size_mismatch():
    # a launcher that started 1 rank for --gpus 2 must not produce a line claiming 2 GPUs
    rc, line, err = _run(["--gpus", "2", "--cpu-dry", "--steps", "1", "--warmup", "0", "--frames", "4"],
                         env_extra={"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    assert rc != 0
    assert line is None
    assert "WORLD_SIZE" in err


def test_bench_config4_eight_ranks_cpu_dry():
    """BASELINE config 4 (8,192 frames, 1,024 per GPU, 8 GPUs): the launcher starts 8 ranks, each
    takes its shard_frames(8192, 8, r) range, and rank 0 reassembles the whole batch through the
    all-gather (gloo here; RCCL on the node).  The same code path the driver's 8-GPU run takes,
    minus the HIP sampler (runners/diffpose_frame.py:126-127, 342)."""
    rc, line, err = _run(["--gpus", "8", "--config", "4", "--cpu-dry", "--steps", "2", "--warmup", "1"],
                         timeout=420)
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 8
    assert line["scaling"] == "weak"
    assert line["config"]["baseline_config"] == 4
    assert line["config"]["frames_total"] == 8192 and line["config"]["frames_per_gpu"] == 1024
    assert len(line["per_rank_ms"]) == 8
    assert line["reassembly_ok"] is True
    assert line["allgather_ms"] > 0
    # the final MPJPE reduction: per-frame errors of all 8 shards gathered (16 B per frame) equal the
    # MPJPE of the stub output over the whole batch computed in one process
    import numpy as np

    from diffpose_amd.data import synthetic_batch

    x, tgt = synthetic_batch(8192)
    o = 2.0 * x.astype(np.float64)[:, :, 2:]
    ref = float(np.mean(np.linalg.norm(o - o[:, :1] - tgt.astype(np.float64), axis=-1))) * 1000.0
    m = line["mpjpe"]
    assert m["frames"] == 8192 and "all_gather" in m["how"]
    assert abs(m["p1_mm"] - ref) <= 1e-6 * max(1.0, ref)


def test_bench_config5_eight_ranks_cpu_dry():
    """BASELINE config 5 at 8 GPUs (1,024 frames x H=20, strong scaling): 8 ranks, 128 frames x 20
    hypotheses = 2,560 rows each (the share the step-split last round runs on the GPU), reassembled
    through the all-gather on rank 0 (gloo here; RCCL on the node)."""
    rc, line, err = _run(["--gpus", "8", "--config", "5", "--cpu-dry", "--steps", "2", "--warmup", "1"],
                         timeout=420)
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 8
    assert line["scaling"] == "strong"
    assert line["config"]["baseline_config"] == 5
    assert line["config"]["frames_total"] == 1024 and line["config"]["frames_per_gpu"] == 128
    assert line["config"]["rows_per_gpu"] == 2560
    assert len(line["per_rank_ms"]) == 8
    assert line["reassembly_ok"] is True
