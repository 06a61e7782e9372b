#!/usr/bin/env python3
"""bench.py — DiffPose DDIM sampler throughput on MI355X (BASELINE.json metric).

One "step" = one pass of the hot path over one batch: the K=50-step DDIM reverse
loop (reference common/utils_diff.py:46-68) over B=1024 frames per GPU (config
human36m_diffpose_uvxyz_cpn eval, H=1), inputs already resident in HBM, plus — under a
launcher (N>1, or torch.distributed.run at N=1) — the final MPJPE reduction: per-frame errors of
each rank's frames (dpk_pose_metrics) and one RCCL all-gather of them, 16 B per frame (frame-sharded,
weak scaling; the north star's only collective).  `value` is whole-job poses/s = frames processed by all ranks / time.

Launch:
  python bench.py [--gpus N --steps K --warmup W]      N>1: spawns N ranks itself (one process per
                                                         GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set
                                                         before any HIP call; the parent never touches
                                                         the GPU) and exits non-zero if any rank fails
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
  python bench.py --config 3|4|5                        the other BASELINE configs (presets below)
  python bench.py --gpus 2 --cpu-dry                    launcher/sharding/all-gather rehearsal on CPU
                                                         (gloo, an elementwise stub instead of the
                                                         sampler; no GPU, nothing timed is meaningful)

Also reported on the same JSON line:
  roofline      the sampler kernel's algorithmic FLOP rate (25,996,254 FLOP per
                pose-step × poses × K ÷ its average launch duration, measured with HIP events
                around that kernel on the stream it is launched on) vs the fp32 MFMA peak;
  cpu_baseline  the golden-pinned oracle (torch CPU, the reference's op sequence) timed on
                this host's cores on the same batch (rank 0, N=1 only; all of it up to 1024 rows,
                --cpu-frames to change), best of --cpu-repeats after a warm-up call, at the host
                threads the job is allotted (OMP_NUM_THREADS; --cpu-threads adds legs);
  parity        MPJPE (mm) of the HIP result vs the oracle on those frames, and max |diff|;
  mpjpe         the job's MPJPE / P-MPJPE over all frames by the final reduction: per-frame errors on
                every rank (dpk_pose_metrics) and one all-gather of 16 B per frame (after the timed steps);
  variants      the same measurement (warmup, timed steps, roofline, parity) in the other GEMM
                modes: the headline is fp32 MFMA (the reference's arithmetic); "f16x3" runs the
                layer GEMMs as three fp16-split MFMA products with fp32 accumulation; "bf16"
                rounds their operands to bf16 (BASELINE config 3's tolerance study).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "diffpose-nw_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

W_ALG = 25_996_254          # FLOP per pose-step, as written (torch FlopCounterMode-verified)
PEAK_FP32_MFMA = 157.3      # TFLOP/s, MI355X FP32 matrix peak (MI355X_MICROARCH.md, chip table)
PEAK_F16_MFMA = 2516.6      # TFLOP/s, MI355X dense FP16 matrix peak (16x the f32 rate, same table)
DTYPES = {"fp32": "fp32",
          "f16x3": "fp32 (layer GEMMs as 3x fp16-split MFMA, fp32 accumulate)",
          "bf16": "bf16 MFMA operands for the layer GEMMs, attention's scores and P.V and the graph product "
                  "(L_g as a bf16 hi+lo pair); fp32 accumulate; LayerNorm, softmax and DDIM fp32: tolerance study"}
METRIC = "poses/sec (B=1024, 17j, K=50 DDIM) at 1/2/4/8 MI355X; MPJPE Δ vs ref"

# BASELINE.json configs 2-5 (config 1 is the reference's own CPU case, timed as cpu_baseline).
# frames: per GPU (weak scaling) unless total_frames is set (fixed job, strong scaling).
CONFIGS = {
    2: dict(yml="human36m_diffpose_uvxyz_cpn", frames=1024, total_frames=None, hyp=1, K=50, T_test=50, T=51,
            gemm="fp32", graph=False),
    3: dict(yml="human36m_diffpose_uvxyz_gt", frames=1024, total_frames=None, hyp=1, K=100, T_test=100, T=101,
            gemm="bf16", graph=False),
    4: dict(yml="human36m_diffpose_uvxyz_cpn", frames=1024, total_frames=None, hyp=1, K=50, T_test=50, T=51,
            gemm="fp32", graph=False),
    5: dict(yml="human36m_diffpose_uvxyz_cpn", frames=None, total_frames=1024, hyp=20, K=50, T_test=50, T=51,
            gemm="fp32", graph=True),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, choices=sorted(CONFIGS), default=2,
                    help="BASELINE.json config preset (2: cpn B=1024 K=50 fp32, the headline; 3: gt K=100 bf16; "
                         "4: cpn 1024 frames per GPU; 5: cpn 1024 frames x H=20 split over the GPUs, hipGraph)")
    ap.add_argument("--frames", type=int, default=None, help="frames per GPU (overrides the preset)")
    ap.add_argument("--total-frames", type=int, default=None,
                    help="frames of the whole job, split over the GPUs (strong scaling; overrides --frames)")
    ap.add_argument("--hyp", type=int, default=None, help="hypotheses per frame (test_times)")
    ap.add_argument("--K", type=int, default=None, help="DDIM steps (test_timesteps)")
    ap.add_argument("--T-test", type=int, default=None, help="test_num_diffusion_timesteps")
    ap.add_argument("--T", type=int, default=None, help="diffusion.num_diffusion_timesteps")
    ap.add_argument("--eta", type=float, default=0.0)
    ap.add_argument("--graph", action="store_true", default=None, help="replay the step from a captured hipGraph")
    ap.add_argument("--cpu-frames", type=int, default=None,
                    help="frames of the CPU baseline and parity sample (default: rank 0's whole batch, at most "
                         "1024 rows, i.e. 1024 // H frames)")
    ap.add_argument("--cpu-repeats", type=int, default=3)
    ap.add_argument("--c3-frames", type=int, default=1024,
                    help="frames of the config-3 (bf16, K=100) variant's parity study against the oracle")
    ap.add_argument("--cpu-threads", type=str, default=None,
                    help="comma-separated thread counts for the CPU baseline legs (default: the box's CPU share, "
                         "OMP_NUM_THREADS, or every physical core of this process's affinity when unset)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--gemm", choices=("fp32", "f16x3", "bf16"), default=None,
                    help="per-layer GEMM arithmetic of the headline (dpk_set_gemm_mode); fp32 is the reference's")
    ap.add_argument("--no-variants", dest="variants", action="store_false",
                    help="skip timing the other GEMM mode (reported under 'variants')")
    ap.add_argument("--cpu-dry", action="store_true",
                    help="rehearse the multi-rank launch, sharding and all-gather on CPU (gloo) with an "
                         "elementwise stub in place of the HIP sampler")
    args = ap.parse_args(argv)
    preset = CONFIGS[args.config]
    for k in ("hyp", "K", "T_test", "T", "gemm", "graph"):
        if getattr(args, k) is None:
            setattr(args, k, preset[k])
    if args.frames is None and args.total_frames is None:
        args.frames, args.total_frames = preset["frames"], preset["total_frames"]
    args.yml = preset["yml"]
    return args


def frames_layout(args, world):
    """(total frames of the job, scaling kind)."""
    if args.total_frames is not None:
        return args.total_frames, "strong"
    return args.frames * world, "weak"


# ---------------------------------------------------------------------------------------------
# launcher: N ranks from a plain `python bench.py --gpus N` (no torch import, no HIP call here)
# ---------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n: int, argv) -> int:
    """Start n rank processes of this script with the torch.distributed.run environment and wait
    for all of them.  Returns 0 only if every rank exited 0; when one fails the others are
    terminated (by their own PIDs) and its code is returned."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DPK_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"bench: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr)
                    for q in pending:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def host_cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def physical_cores(cpus):
    """Number of distinct (package, core) pairs among the logical CPUs ``cpus`` (SMT siblings once)."""
    seen = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            seen.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            return len(cpus)
    return len(seen) or len(cpus)


def mpjpe_mm(out_uvxyz, targets, hyp):
    import numpy as np

    o = np.asarray(out_uvxyz, dtype=np.float64).reshape(hyp, -1, 17, 5).mean(0)
    xyz = o[:, :, 2:] - o[:, :1, 2:]
    return float(np.mean(np.linalg.norm(xyz - np.asarray(targets, np.float64), axis=-1)) * 1000.0)


def cpu_baseline(args, x_all, seq, betas, K, hyp):
    """The oracle (reference op sequence, torch CPU fp32) on the first cpu_frames frames, best of
    cpu_repeats, at the host thread count this job is allotted (SURVEY §8d asks for all physical
    cores; the GPU box allots 16 CPUs per GPU through OMP_NUM_THREADS and asks that worker pools stay
    within that share, so the share is the default leg; --cpu-threads adds others).
    Returns (result dict, final poses of the share run, frames timed)."""
    import numpy as np
    import torch

    from diffpose_amd.data import repeat_hypotheses
    from diffpose_amd.weights import synthetic_state_dict
    from oracle import gcndiff_oracle as O

    cpus = sorted(os.sched_getaffinity(0))
    phys = physical_cores(cpus)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or phys
    share = max(1, min(share, len(cpus)))
    n_cpu = min(args.cpu_frames if args.cpu_frames else max(1, 1024 // hyp), x_all.shape[0])
    xc = torch.from_numpy(repeat_hypotheses(x_all[:n_cpu], hyp))
    P = O.params_to_torch(synthetic_state_dict())
    adj = O.adjacency()
    mask = torch.ones(1, 1, 17, dtype=torch.bool)

    def run(x):
        xs, _ = O.generalized_steps(x, mask, seq, lambda a, m, t: O.gcndiff_forward(P, adj, a, m, t), betas, eta=0.0)
        return xs[-1]

    legs, ref = {}, None
    legs_wanted = {share}
    if args.cpu_threads:
        legs_wanted |= {max(1, min(int(t), len(cpus))) for t in args.cpu_threads.split(",") if t.strip()}
    for threads in sorted(legs_wanted):
        torch.set_num_threads(threads)
        run(xc[: min(8, xc.shape[0])])                     # thread pool + allocator warm-up, untimed
        times = []
        for _ in range(max(1, args.cpu_repeats)):
            t0 = time.perf_counter()
            out = run(xc)
            times.append(time.perf_counter() - t0)
        legs[threads] = (n_cpu / min(times), times)
        if threads == share:
            ref = out
    best_threads = max(legs, key=lambda t: legs[t][0])
    v, times = legs[best_threads]
    res = {
        "value": round(v, 3), "unit": "poses/s", "cores": best_threads, "kind": "port",
        "sample": (f"oracle generalized_steps+GCNdiff (torch CPU fp32, reference op order, golden-pinned) on the "
                   f"first {n_cpu} frames x H={hyp} of the same batch, K={K}, best of {max(1, args.cpu_repeats)} "
                   f"after an untimed warm-up call; host '{host_cpu_model()}', {len(cpus)} logical CPUs in this "
                   f"process's affinity ({phys} physical cores); " +
                   "; ".join(f"{t} threads: {legs[t][0]:.1f} poses/s (runs {', '.join(f'{s:.2f}' for s in legs[t][1])} s)"
                             for t in sorted(legs))),
        "by_threads": {str(t): round(legs[t][0], 3) for t in sorted(legs)},
    }
    torch.set_num_threads(share)
    return res, (ref.numpy() if ref is not None else None), n_cpu


def config3_parity(args, x_all, tgt_all, out_bf16, out_fp32):
    """BASELINE config 3's tolerance study: the oracle (reference op order, torch CPU fp32) at K=100 over T=101 on
    the first --c3-frames frames; MPJPE delta and max |diff| of the bf16 run and, on the same frames, of the fp32
    mode (same schedule), against it.  bf16 is a study, not held to the fp32 bar of 1e-4 mm."""
    import numpy as np
    import torch

    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict
    from oracle import gcndiff_oracle as O

    n = min(args.c3_frames, x_all.shape[0])
    seq3 = make_seq("uniform", CONFIGS[3]["T_test"], CONFIGS[3]["K"])
    b3 = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                            num_diffusion_timesteps=CONFIGS[3]["T"])).float()
    P = O.params_to_torch(synthetic_state_dict())
    adj = O.adjacency()
    mask = torch.ones(1, 1, 17, dtype=torch.bool)
    t0 = time.perf_counter()
    xs, _ = O.generalized_steps(torch.from_numpy(x_all[:n]), mask, seq3,
                                lambda a, m, t: O.gcndiff_forward(P, adj, a, m, t), b3, eta=0.0)
    cpu_s = time.perf_counter() - t0
    ref = xs[-1].numpy()
    tg = tgt_all[:n]
    m_r = mpjpe_mm(ref, tg, 1)
    res = {"frames": n, "K": len(seq3), "T": CONFIGS[3]["T"], "mpjpe_ref_mm": round(m_r, 6), "oracle_s": round(cpu_s, 2),
           "note": "tolerance study (BASELINE config 3): bf16 operands of the layer GEMMs, attention's score and "
                   "P.V products and the graph product; fp32 beside it on the same frames and schedule; the fp32 bar is 1e-4 mm"}
    for name, o in (("bf16", out_bf16), ("fp32", out_fp32)):
        m_h = mpjpe_mm(o[:n], tg, 1)
        res[name] = {"mpjpe_hip_mm": round(m_h, 6), "mpjpe_delta_mm": float(f"{abs(m_h - m_r):.3e}"),
                     "max_abs_diff": float(f"{float(np.abs(o[:n] - ref).max()):.3e}")}
    return res


# ---------------------------------------------------------------------------------------------
# one rank
# ---------------------------------------------------------------------------------------------
def rank_main(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    from diffpose_amd import dist as D
    from diffpose_amd.data import repeat_hypotheses, shard_frames, synthetic_batch
    from diffpose_amd.schedule import get_beta_schedule, make_seq

    rank, world, local = D.world_info()
    launched = "RANK" in os.environ and "MASTER_ADDR" in os.environ
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to report a different world size",
              file=sys.stderr)
        return 2
    dry = args.cpu_dry
    if dry:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    # under a launcher (ours or torch.distributed.run) the collective path runs at every N, N=1 included,
    # so per-GPU work is the same at every point of the scaling sweep
    use_dist = world > 1 or launched
    if use_dist:
        if dry:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def sync():
        if not dry:
            torch.cuda.synchronize(dev)

    # ---- schedule, inputs (synthetic, seeded), model ----
    seq = make_seq("uniform", args.T_test, args.K)
    betas = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                               num_diffusion_timesteps=args.T)).float()
    K = len(seq)
    B_total, scaling = frames_layout(args, world)
    x_all, tgt_all = synthetic_batch(B_total)
    lo, hi = shard_frames(B_total, world, rank)
    x_host = repeat_hypotheses(x_all[lo:hi], args.hyp)
    x = torch.from_numpy(x_host).to(dev)
    out = torch.empty_like(x)
    rows = x.shape[0]
    model = None
    setup_ms = setup_cold_ms = None
    if not dry:
        from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
        from diffpose_amd.weights import synthetic_state_dict

        model = HipGCNdiff(adj_mx_from_edges(), None, device=dev)
        model.load_state_dict(synthetic_state_dict())
        sync()
        # host-synchronous: the call returns with the schedule built.  The first build in a process also
        # pays the code-object load and first launch of temb_kernel (setup_cold_ms); the schedule the
        # timed steps use is built second, warm (setup_ms: what a caller pays per new schedule)
        t_set = time.perf_counter()
        model.set_schedule(seq, betas, args.eta + 0.5)
        setup_cold_ms = (time.perf_counter() - t_set) * 1e3
        t_set = time.perf_counter()
        model.set_schedule(seq, betas, args.eta)
        setup_ms = (time.perf_counter() - t_set) * 1e3

    gathered = {}
    tg_local = torch.from_numpy(tgt_all[lo:hi]).to(dev)
    if not dry:
        from diffpose_amd.metrics import pose_errors

    def frame_errors(o):
        """Per-frame (MPJPE, P-MPJPE) in metres of this rank's frames, [frames, 2] float64: dpk_pose_metrics
        (hypothesis mean, root-relative, Procrustes, fp64); the cpu-dry stub: MPJPE only."""
        if dry:
            v = o.double().view(args.hyp, hi - lo, 17, 5).mean(0)[:, :, 2:]
            return torch.stack([torch.norm(v - v[:, :1] - tg_local.double(), dim=-1).mean(-1),
                                torch.full((hi - lo,), float("nan"), dtype=torch.float64)], dim=1)
        return torch.stack(pose_errors(o, tg_local, args.hyp, root_mode="relative"), dim=1)

    cur = {"seq": seq, "betas": betas}         # the schedule step() runs (the config-3 variant swaps it)

    def step():
        if dry:
            torch.mul(x, 2.0, out=out)                 # stand-in for the sampler: rank-independent, exact
        else:
            model.sample(x, cur["seq"], cur["betas"], eta=args.eta, out=out)
        # the final MPJPE reduction (north_star) at every N, N=1 included, so every point of the scaling
        # sweep times the same work: per-frame errors of this rank's frames (dpk_pose_metrics), and under
        # a launcher the one data-path collective, their all-gather (16 B per frame)
        fe_step = frame_errors(out)
        gathered["fe"] = D.gather_frames(fe_step, B_total, 1) if use_dist else fe_step

    def measure(gemm):
        """Time exactly args.steps steps (barrier + sync both sides, max over ranks) in one GEMM mode."""
        if model is not None:
            model.set_gemm_mode(gemm)
        for _ in range(args.warmup):
            step()
        sync()
        graph = None
        if args.graph and not dry:
            graph = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                step()                                 # warm the side stream
            torch.cuda.current_stream(dev).wait_stream(s)
            sync()
            with torch.cuda.graph(graph):
                step()
            run = graph.replay
        else:
            run = step
            if model is not None:
                model.profile(True)
        if use_dist:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        sync()
        if use_dist:
            dist.barrier()
        mine = time.perf_counter() - t0
        elapsed = D.max_over_ranks(mine, device=dev)
        kernel_ms = model.kernel_times_ms() if (graph is None and model is not None) else []
        if model is not None:
            model.profile(False)
        return elapsed, mine, kernel_ms

    def roofline(gemm, kernel_ms, K=K):
        if not kernel_ms:
            return None
        km = np.asarray(kernel_ms, dtype=np.float64)
        avg_kernel_ms = float(km.mean())
        achieved = W_ALG * rows * K / (avg_kernel_ms * 1e-3) / 1e12
        # f16x3: every fp32 product is three f16 MFMA passes, so the fp32-equivalent peak is 1/3 of f16's;
        # bf16: one pass at the dense bf16 peak (same rate as f16)
        peak = {"fp32": PEAK_FP32_MFMA, "f16x3": round(PEAK_F16_MFMA / 3, 1), "bf16": PEAK_F16_MFMA}[gemm]
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": None,
                "kernel": "dpk::sample_kernel<0, *, %d>" % {"fp32": 0, "f16x3": 1, "bf16": 2}[gemm],
                "avg_launch_ms": round(avg_kernel_ms, 4), "median_launch_ms": round(float(np.median(km)), 4),
                "min_launch_ms": round(float(km.min()), 4),
                "launches": len(kernel_ms), "flop_per_launch": W_ALG * rows * K,
                "per_unit": f"{W_ALG} FLOP per pose-step (SURVEY 8d) x {rows} poses x {K} steps"}
        tfile = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tfile):
            try:
                tr = json.load(open(tfile))
                key = f"rows{rows}_K{K}" + ("" if gemm == "fp32" else "_" + gemm)
                if key in tr:
                    roof["traffic"] = tr[key]["hbm_bytes_per_launch"]
                    roof["traffic_source"] = tr[key]["source"]
                    if "mfma_busy" in tr[key]:      # the executed-work figure beside frac
                        roof["mfma_busy"] = tr[key]["mfma_busy"]
                        roof["mfma_busy_source"] = tr[key]["mfma_busy_source"]
            except (OSError, ValueError, KeyError):
                pass
        return roof

    # ---- timed region (headline mode), then the other GEMM mode as a variant on the same line ----
    elapsed, mine, kernel_ms = measure(args.gemm)
    per_rank_ms = [mine / args.steps * 1e3]
    allgather_ms = None
    reassembly = None
    if use_dist:
        t = torch.tensor([mine / args.steps * 1e3], dtype=torch.float64, device=dev)
        lst = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(lst, t)
        per_rank_ms = [round(float(v.item()), 4) for v in lst]
        # the step's all-gather alone (per-frame errors, 16 B per frame), same barrier/sync bracket, max over ranks
        fe_local = frame_errors(out)
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        n_ag = 20
        for _ in range(n_ag):
            D.gather_frames(fe_local, B_total, 1)
        sync()
        dist.barrier()
        allgather_ms = D.max_over_ranks(time.perf_counter() - t0, device=dev) / n_ag * 1e3
        # the final poses reassembled once (not part of the step): every shard where shard_rows puts it
        full = D.gather_frames(out, B_total, args.hyp)
        if dry:   # the stub is exact, so the reassembled batch must equal the stub over the whole batch
            expect = torch.from_numpy(repeat_hypotheses(x_all, args.hyp)) * 2.0
            reassembly = bool(torch.equal(full.cpu(), expect))
        else:     # every rank's own shard must sit where shard_rows says it belongs
            idx = D.shard_rows(B_total, args.hyp, world, rank).to(dev)
            ok = torch.tensor([1 if torch.equal(full[idx], out) else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            reassembly = bool(ok.item())
    # ---- the final MPJPE reduction (runners/diffpose_frame.py:382-387): per-frame (MPJPE, P-MPJPE) of this
    #      rank's frames (dpk_pose_metrics: hypothesis mean, root-relative, Procrustes, fp64), then one
    #      all-gather of those 16 B per frame; every rank ends with the job's MPJPE.  Once, after the timed steps.
    frame_errors(out)      # untimed first (first launches in this process: the metrics kernel, torch's cat)
    if use_dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    fe = frame_errors(out)
    if use_dist:
        fe = D.gather_frames(fe, B_total, 1)
    sync()
    reduce_s = time.perf_counter() - t0
    # the timed steps' own reduction of the same output gave the same numbers
    g = gathered["fe"]
    eq = bool(((fe == g) | (torch.isnan(fe) & torch.isnan(g))).all())      # the dry stub's P-MPJPE is NaN
    same = torch.tensor([1 if eq else 0], dtype=torch.int32, device=dev)
    if use_dist:
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
    if use_dist:
        reduce_s = D.max_over_ranks(reduce_s, device=dev)
    fe_h = fe.cpu().numpy()
    if not bool(same.item()):
        print("bench: the steps' gathered per-frame errors differ from the final reduction's", file=sys.stderr)
        return 3
    mpjpe_line = {"p1_mm": round(float(fe_h[:, 0].mean()) * 1000.0, 6),
                  "p2_mm": None if dry else round(float(fe_h[:, 1].mean()) * 1000.0, 6),
                  "frames": int(fe_h.shape[0]), "reduce_ms": round(reduce_s * 1e3, 4),
                  "how": ("per-frame (MPJPE, P-MPJPE) on each rank's frames (dpk_pose_metrics, fp64), " +
                          ("one all_gather of 16 B per frame, inside every timed step" if use_dist
                           else "one rank, no collective; inside every timed step (the same work as at N>1)")),
                  "targets": "synthetic (seeded), root-relative"}
    out_main = out.detach().cpu().numpy() if (world == 1 and rank == 0 and not dry) else None
    variants = {}
    if args.variants and not dry:
        for g in ("fp32", "f16x3"):
            if g == args.gemm:
                continue
            e2, _, k2 = measure(g)
            variants[g] = {"value": round(B_total * args.steps / e2, 2), "ms_per_step": round(e2 / args.steps * 1e3, 4),
                           "roofline": roofline(g, k2),
                           "dtype": DTYPES[g]}
            if world == 1 and rank == 0:
                variants[g]["_out"] = out.detach().cpu().numpy()
        # BASELINE config 3 (human36m_diffpose_uvxyz_gt: K=100 over T'=100, T=101, bf16 tolerance study) on the
        # same frames, on the driver's line since round 6: its own roofline (dense bf16 peak) and, on rank 0 at
        # N=1, a parity study against the oracle (below)
        if args.config == 2 and args.hyp == 1:
            seq3 = make_seq("uniform", CONFIGS[3]["T_test"], CONFIGS[3]["K"])
            b3 = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                                    num_diffusion_timesteps=CONFIGS[3]["T"])).float()
            cur.update(seq=seq3, betas=b3)
            e3, _, k3 = measure("bf16")
            variants["config3_bf16"] = {
                "value": round(B_total * args.steps / e3, 2), "ms_per_step": round(e3 / args.steps * 1e3, 4),
                "roofline": roofline("bf16", k3, K=len(seq3)), "dtype": DTYPES["bf16"],
                "workload": (f"BASELINE config 3: {CONFIGS[3]['yml']} eval, {B_total} frames, K={len(seq3)} DDIM "
                             f"(uniform skip over T'={CONFIGS[3]['T_test']}, T={CONFIGS[3]['T']}), bf16 layer GEMMs")}
            if world == 1 and rank == 0:
                variants["config3_bf16"]["_out"] = out.detach().cpu().numpy()
                model.set_gemm_mode("fp32")            # the fp32 mode on the same schedule, for the parity study
                model.sample(x, seq3, b3, eta=args.eta, out=out)
                variants["config3_bf16"]["_out_fp32"] = out.detach().cpu().numpy()
            cur.update(seq=seq, betas=betas)
        model.set_gemm_mode(args.gemm)

    frames_done = B_total * args.steps
    value = frames_done / elapsed
    ms_per_step = elapsed / args.steps * 1000.0
    roof = roofline(args.gemm, kernel_ms)

    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "poses/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None,
        "dtype": DTYPES[args.gemm],
        "data": "synthetic: seeded PCG64 Human3.6M-shaped uvxyz poses and GCNdiff weights (no H36M/checkpoints offline)",
        "config": {"workload": f"BASELINE config {args.config}: {args.yml} eval, {B_total} frames x H={args.hyp} "
                               f"({rows} rows on rank 0), K={K} DDIM (uniform skip over T'={args.T_test}, "
                               f"T={args.T}), eta={args.eta}",
                   "baseline_config": args.config, "frames_total": B_total, "frames_per_gpu": hi - lo,
                   "hypotheses": args.hyp, "rows_per_gpu": rows, "K": K,
                   "parallelism": f"dp{world} frame-sharded; every step = sampler + per-frame MPJPE/P-MPJPE "
                                  f"(dpk_pose_metrics)" + (" + RCCL all_gather of the per-frame errors (the final "
                                                           "MPJPE reduction)" if use_dist else ""),
                   "hipgraph": bool(args.graph), "gemm": args.gemm},
        "per_rank_ms": per_rank_ms,
        "setup_ms": None if setup_ms is None else round(setup_ms, 4),
        "setup_cold_ms": None if setup_cold_ms is None else round(setup_cold_ms, 4),
        "setup_note": None if setup_ms is None else (
            f"per (weights, schedule), outside the timed region: dpk_set_schedule's host step scalars, upload and "
            f"temb_kernel ({K} workgroups: the timestep MLP and the 5 temb_proj rows of every step, batch-invariant, "
            f"SURVEY a7), host-synchronous wall time; every dpk_sample with that schedule reuses them, so a caller "
            f"running a single batch pays it once on top of ms_per_step; setup_cold_ms is the process's first build "
            f"(adds the code-object load and first launch)"),
        "roofline": roof,
        "cpu_baseline": None,
    }
    if dry:
        result.update({"dtype": "fp32", "data": "cpu-dry rehearsal: elementwise stub instead of the sampler",
                       "value": None, "roofline": None})
        result["config"]["parallelism"] = f"dp{world} frame-sharded + gloo all_gather (cpu-dry)"
    result["mpjpe"] = mpjpe_line
    if allgather_ms is not None:
        result["allgather_ms"] = round(allgather_ms, 4)
        result["reassembly_ok"] = reassembly
    if variants:
        result["variants"] = variants
    if args.hyp > 1 and value is not None:
        result["rows_per_s"] = round(value * args.hyp, 2)

    # ---- CPU baseline + parity (rank 0, N=1) ----
    if world == 1 and rank == 0 and not args.no_cpu and not dry:
        cb, ref_np, n_cpu = cpu_baseline(args, x_all, seq, betas, K, args.hyp)
        result["cpu_baseline"] = cb
        if args.eta == 0.0 and ref_np is not None:
            idx = np.concatenate([np.arange(h * (hi - lo), h * (hi - lo) + n_cpu) for h in range(args.hyp)])
            tg = tgt_all[:n_cpu]
            m_r = mpjpe_mm(ref_np, tg, args.hyp)

            def parity(full_out, gemm):
                hip_out = full_out[idx]
                m_h = mpjpe_mm(hip_out, tg, args.hyp)
                r = {"frames": n_cpu, "mpjpe_hip_mm": round(m_h, 6), "mpjpe_ref_mm": round(m_r, 6),
                     "mpjpe_delta_mm": float(f"{abs(m_h - m_r):.3e}"),
                     "max_abs_diff": float(f"{float(np.abs(hip_out - ref_np).max()):.3e}"),
                     "tolerance_mm": 1e-4, "pass": abs(m_h - m_r) <= 1e-4}
                if gemm == "bf16":   # reduced precision: the delta IS the tolerance-study result
                    r.update({"tolerance_mm": None, "pass": None,
                              "note": "tolerance study (BASELINE config 3): bf16 operands of the layer GEMMs, attention's score and P.V products and the graph product; the fp32 bar is 1e-4 mm"})
                return r
            result["parity"] = parity(out_main, args.gemm)
            for g, v in variants.items():
                if g in ("fp32", "f16x3"):
                    v["parity"] = parity(v["_out"], g)
        c3 = variants.get("config3_bf16")
        if c3 is not None and args.eta == 0.0:
            c3["parity"] = config3_parity(args, x_all, tgt_all, c3["_out"], c3["_out_fp32"])
    for v in variants.values():
        v.pop("_out", None)
        v.pop("_out_fp32", None)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if use_dist:
        dist.destroy_process_group()
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus < 1:
        print("bench: --gpus must be >= 1", file=sys.stderr)
        return 2
    if args.gpus > 1 and "RANK" not in os.environ:
        return launch(args.gpus, argv)
    return rank_main(args)


if __name__ == "__main__":
    sys.exit(main())
