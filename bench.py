#!/usr/bin/env python3
"""bench.py — DiffPose DDIM sampler throughput on MI355X (BASELINE.json metric).

One "step" = one pass of the hot path over one batch: the K=50-step DDIM reverse
loop (reference common/utils_diff.py:46-68) over B=1024 frames per GPU (config
human36m_diffpose_uvxyz_cpn eval, H=1), inputs already resident in HBM, plus — for
N>1 — the RCCL all-gather of the final poses to every rank (frame-sharded, weak
scaling).  `value` is whole-job poses/s = frames processed by all ranks / time.

Also reported on the same JSON line:
  roofline      the sampler kernel's algorithmic FLOP rate (25,996,254 FLOP per
                pose-step × poses × K ÷ its average launch duration, measured with HIP events
                around that kernel on the stream it is launched on) vs the fp32 MFMA peak;
  cpu_baseline  the golden-pinned oracle (torch CPU, the reference's op sequence) timed on
                this host's cores on the first --cpu-frames frames of the same batch (rank 0,
                N=1 only);
  parity        MPJPE (mm) of the HIP result vs the oracle on those frames, and max |diff|;
  variants      the same measurement (warmup, timed steps, roofline, parity) in the other GEMM
                modes: the headline is fp32 MFMA (the reference's arithmetic); "f16x3" runs the
                layer GEMMs as three fp16-split MFMA products with fp32 accumulation; "bf16"
                rounds their operands to bf16 (BASELINE config 3's tolerance study).

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
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
          "bf16": "bf16 layer GEMMs (fp32 accumulate; LN/attention/graph/DDIM fp32): tolerance study"}
METRIC = "poses/sec (B=1024, 17j, K=50 DDIM) at 1/2/4/8 MI355X; MPJPE Δ vs ref"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1024, help="frames per GPU")
    ap.add_argument("--hyp", type=int, default=1, help="hypotheses per frame (test_times)")
    ap.add_argument("--K", type=int, default=50, help="DDIM steps (test_timesteps)")
    ap.add_argument("--T-test", type=int, default=50, help="test_num_diffusion_timesteps")
    ap.add_argument("--T", type=int, default=51, help="diffusion.num_diffusion_timesteps")
    ap.add_argument("--eta", type=float, default=0.0)
    ap.add_argument("--graph", action="store_true", help="replay the step from a captured hipGraph")
    ap.add_argument("--cpu-frames", type=int, default=1024)
    ap.add_argument("--cpu-repeats", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--gemm", choices=("fp32", "f16x3", "bf16"), default="fp32",
                    help="per-layer GEMM arithmetic of the headline (dpk_set_gemm_mode); fp32 is the reference's")
    ap.add_argument("--no-variants", dest="variants", action="store_false",
                    help="skip timing the other GEMM mode (reported under 'variants')")
    return ap.parse_args()


def host_cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def mpjpe_mm(out_uvxyz, targets, hyp):
    import numpy as np

    o = np.asarray(out_uvxyz, dtype=np.float64).reshape(hyp, -1, 17, 5).mean(0)
    xyz = o[:, :, 2:] - o[:, :1, 2:]
    return float(np.mean(np.linalg.norm(xyz - np.asarray(targets, np.float64), axis=-1)) * 1000.0)


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from diffpose_amd import dist as D
    from diffpose_amd.data import repeat_hypotheses, shard_frames, synthetic_batch
    from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict

    rank, world, local = D.world_info()
    if world != args.gpus:
        if rank == 0:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # under a launcher (torch.distributed.run sets RANK/MASTER_ADDR) the RCCL path runs at every
    # N, N=1 included, so per-GPU work is the same at every point of the scaling sweep
    use_dist = world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ)
    if use_dist:
        dist.init_process_group("nccl", device_id=dev)

    # ---- model, schedule, inputs (synthetic, seeded) ----
    model = HipGCNdiff(adj_mx_from_edges(), None, device=dev)
    model.load_state_dict(synthetic_state_dict())
    seq = make_seq("uniform", args.T_test, args.K)
    betas = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                               num_diffusion_timesteps=args.T)).float()
    model.set_schedule(seq, betas, args.eta)
    K = len(seq)
    B_total = args.frames * world
    x_all, tgt_all = synthetic_batch(B_total)
    lo, hi = shard_frames(B_total, world, rank)
    x_host = repeat_hypotheses(x_all[lo:hi], args.hyp)
    x = torch.from_numpy(x_host).to(dev)
    out = torch.empty_like(x)
    rows = x.shape[0]

    def step():
        model.sample(x, seq, betas, eta=args.eta, out=out)
        if use_dist:                             # the one data-path collective: final poses to every rank
            D.gather_frames(out, B_total, args.hyp)

    def measure(gemm):
        """Time exactly args.steps steps (barrier + sync both sides, max over ranks) in one GEMM mode."""
        model.set_gemm_mode(gemm)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        graph = None
        if args.graph:
            graph = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                step()                                   # warm the side stream
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize()
            with torch.cuda.graph(graph):
                step()
            run = graph.replay
        else:
            run = step
            model.profile(True)
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        if use_dist:
            dist.barrier()
        elapsed = D.max_over_ranks(time.perf_counter() - t0, device=dev)
        kernel_ms = model.kernel_times_ms() if graph is None else []
        model.profile(False)
        return elapsed, kernel_ms

    def roofline(gemm, kernel_ms):
        if not kernel_ms:
            return None
        avg_kernel_ms = float(np.mean(kernel_ms))
        achieved = W_ALG * rows * K / (avg_kernel_ms * 1e-3) / 1e12
        # f16x3: every fp32 product is three f16 MFMA passes, so the fp32-equivalent peak is 1/3 of f16's;
        # bf16: one pass at the dense bf16 peak (same rate as f16)
        peak = {"fp32": PEAK_FP32_MFMA, "f16x3": round(PEAK_F16_MFMA / 3, 1), "bf16": PEAK_F16_MFMA}[gemm]
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": None,
                "kernel": "dpk::sample_kernel<0, *, %d>" % {"fp32": 0, "f16x3": 1, "bf16": 2}[gemm],
                "avg_launch_ms": round(avg_kernel_ms, 4),
                "launches": len(kernel_ms), "flop_per_launch": W_ALG * rows * K,
                "per_unit": f"{W_ALG} FLOP per pose-step (SURVEY 8d) x {rows} poses x {K} steps"}
        tfile = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tfile):
            try:
                tr = json.load(open(tfile))
                key = f"frames{args.frames}_hyp{args.hyp}_K{K}" + ("" if gemm == "fp32" else "_" + gemm)
                if key in tr:
                    roof["traffic"] = tr[key]["hbm_bytes_per_launch"]
                    roof["traffic_source"] = tr[key]["source"]
            except (OSError, ValueError, KeyError):
                pass
        return roof

    # ---- timed region (headline mode), then the other GEMM mode as a variant on the same line ----
    elapsed, kernel_ms = measure(args.gemm)
    out_main = out.detach().cpu().numpy() if (world == 1 and rank == 0) else None
    variants = {}
    if args.variants:
        for g in ("fp32", "f16x3"):
            if g == args.gemm:
                continue
            e2, k2 = measure(g)
            variants[g] = {"value": round(B_total * args.steps / e2, 2), "ms_per_step": round(e2 / args.steps * 1e3, 4),
                           "roofline": roofline(g, k2),
                           "dtype": DTYPES[g]}
            if world == 1 and rank == 0:
                variants[g]["_out"] = out.detach().cpu().numpy()
        model.set_gemm_mode(args.gemm)

    frames_done = B_total * args.steps
    value = frames_done / elapsed
    ms_per_step = elapsed / args.steps * 1000.0
    roof = roofline(args.gemm, kernel_ms)

    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "poses/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPES[args.gemm],
        "data": "synthetic: seeded PCG64 Human3.6M-shaped uvxyz poses and GCNdiff weights (no H36M/checkpoints offline)",
        "config": {"workload": f"human36m_diffpose_uvxyz_cpn eval: {args.frames} frames/GPU x H={args.hyp}, "
                               f"K={K} DDIM (uniform skip over T'={args.T_test}, T={args.T}), eta={args.eta}",
                   "frames_per_gpu": args.frames, "hypotheses": args.hyp, "rows_per_gpu": rows, "K": K,
                   "parallelism": f"dp{world} frame-sharded" + (" + RCCL all_gather of final poses" if use_dist else ""),
                   "hipgraph": bool(args.graph), "gemm": args.gemm},
        "roofline": roof,
        "cpu_baseline": None,
    }
    if variants:
        result["variants"] = variants
    if args.hyp > 1:
        result["rows_per_s"] = round(value * args.hyp, 2)

    # ---- CPU baseline + parity (rank 0, N=1) ----
    if world == 1 and rank == 0 and not args.no_cpu:
        from oracle import gcndiff_oracle as O

        cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        cores = max(1, min(cores, os.cpu_count() or cores))
        torch.set_num_threads(cores)
        n_cpu = min(args.cpu_frames, args.frames)
        xc = torch.from_numpy(repeat_hypotheses(x_all[:n_cpu], args.hyp))
        P = O.params_to_torch(synthetic_state_dict())
        adj = O.adjacency()
        mask = torch.ones(1, 1, 17, dtype=torch.bool)
        best, ref = None, None
        for _ in range(max(1, args.cpu_repeats)):
            t0 = time.perf_counter()
            xs, _ = O.generalized_steps(xc, mask, seq, lambda a, m, t: O.gcndiff_forward(P, adj, a, m, t), betas,
                                        eta=0.0)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
            ref = xs[-1]
        result["cpu_baseline"] = {
            "value": round(n_cpu / best, 3), "unit": "poses/s", "cores": cores, "kind": "port",
            "sample": f"oracle generalized_steps+GCNdiff (torch CPU fp32, reference op order, golden-pinned) on the "
                      f"first {n_cpu} frames x H={args.hyp} of the same batch, K={K}, best of "
                      f"{max(1, args.cpu_repeats)}: {best:.2f} s; host '{host_cpu_model()}', "
                      f"{os.cpu_count()} logical CPUs, {cores} threads"}
        if args.eta == 0.0:
            idx = np.concatenate([np.arange(h * args.frames, h * args.frames + n_cpu) for h in range(args.hyp)])
            ref_np = ref.numpy()
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
                              "note": "tolerance study (BASELINE config 3): bf16 GEMM operands; the fp32 bar is 1e-4 mm"})
                return r
            result["parity"] = parity(out_main, args.gemm)
            for g, v in variants.items():
                v["parity"] = parity(v["_out"], g)
    for v in variants.values():
        v.pop("_out", None)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
