"""CPU, world size 2 over gloo: the distributed final-MPJPE reduction of ``runner.Diffpose.test_hyber``
(runners/diffpose_frame.py:330-420 run frame-sharded).

Each rank evaluates its frame shard of every batch and one all-gather brings the per-frame
(MPJPE, P-MPJPE) back into frame order, so the reference's accounting (common/utils.py:96-152 —
single-action batches booked in one update, mixed batches booking the *batch* P-MPJPE mean per
frame) runs on the whole batch on every rank.  A deterministic per-frame stand-in replaces the HIP
pose/sampler/metrics kernels (no GPU here); it folds in the rank's rows of the eta > 0 noise, so
the test also checks that each rank receives exactly its rows of the reference's whole-batch
draws.  The bar: bit-equal (p1, p2), per-action sums and epoch meters vs one process.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2
ACT = ["Directions", "Eating", "Sitting", "Walking", "WalkDog"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batches():
    rng = np.random.Generator(np.random.PCG64(77))
    out = []
    for b, (n, mixed) in enumerate([(10, False), (7, True), (1, False), (5, True), (6, False)]):
        x2d = rng.normal(0, 0.3, size=(n, 17, 2)).astype(np.float32)
        tgt = rng.normal(0, 0.25, size=(n, 17, 3)).astype(np.float32)
        if mixed:
            acts = [ACT[int(k)] + f" {1 + int(k) % 2}" for k in rng.integers(0, len(ACT), size=n)]
        else:
            acts = [f"{ACT[b % len(ACT)]} 1"] * n
        out.append((x2d, tgt, acts))
    return out


def _stub(input_2d, targets_3d, H, seq, i, noise, root_mode):
    """Per-frame values that depend only on the frame (and its noise rows), float64."""
    x = torch.from_numpy(input_2d).double()
    t = torch.from_numpy(targets_3d).double()
    F = x.shape[0]
    uv0 = torch.cat([x, torch.zeros(F, 17, 1, dtype=torch.float64)], dim=2)
    p1 = torch.norm(t - uv0, dim=-1).mean(-1) * 1e-3
    p2 = 0.5 * p1 + x.std(dim=(1, 2)) * 1e-3 if F else p1.clone()
    if noise is not None and F:
        z = noise.double().view(noise.shape[0], H, F, 17, 5)
        p2 = p2 + z.sum(dim=(0, 1, 3, 4)) * 1e-6
    return p1, p2


def _run(eta):
    from diffpose_amd import runner as R

    cfg = R.default_config(test_times=3, test_timesteps=4, test_num_diffusion_timesteps=50)
    args = R.default_args(eta=eta, noise="torch-cpu")
    d = R.Diffpose(args, cfg, device="cpu")
    torch.manual_seed(5)
    p1, p2 = d.test_hyber(batches=_batches(), is_train=True, frame_errors=_stub)
    per_action = {a: (v["p1"].sum, v["p1"].count, v["p2"].sum, v["p2"].count) for a, v in d.action_error_sum.items()}
    return p1, p2, per_action, d.epoch_loss


def _worker(rank, port, eta, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "diffpose-nw_amd"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    torch.set_num_threads(1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        q.put((rank, _run(eta)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e)))
        raise


def _spawn(eta):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, eta, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(WORLD):
            r, v = q.get(timeout=300)
            assert not isinstance(v, str), f"rank {r} failed: {v}"
            res[r] = v
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    return res


def test_test_hyber_sharded_accounting_bit_equal():
    for eta in (0.0, 0.5):
        single = _run(eta)
        res = _spawn(eta)
        for r in range(WORLD):
            p1, p2, per_action, epoch = res[r]
            assert (p1, p2) == single[:2], f"eta {eta} rank {r}: {(p1, p2)} vs {single[:2]}"
            assert per_action == single[2], f"eta {eta} rank {r}: per-action sums differ"
            assert epoch == single[3]
        assert single[0] > 0 and single[1] > 0
    # the noise reaches the stand-in: eta > 0 changes P-MPJPE
    assert _run(0.5)[1] != _run(0.0)[1]
