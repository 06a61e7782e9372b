"""Copy one tools/profile_r05.sh / profile_r06.sh run from gpurun_out/ into profiles/ with the summaries the docs cite.

  python tools/collect_profile.py TAG        # e.g. r05_v31, r06_v7
(profile_r06.sh's FETCH_SIZE / WRITE_SIZE passes are folded by tools/traffic_from_pmc.py.)

Per kernel trace (headline fp32, config-3 bf16, f16x3): the sampler kernel's per-dispatch durations
(rocprofv3 --kernel-trace), their mean over the timed dispatches (the last `steps` of them), the bench line
run under rocprofv3's own HIP-event average beside it, and the roofline fraction from the rocprof mean.
The SQ passes go through tools/sq_summary.py.  Bench lines, tests, smoke and phase traces are copied as is.
"""
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def trace_summary(tag, sub, bench_json, label):
    rows = [r for r in csv.DictReader(open(os.path.join(G, f"{tag}{sub}_prof", "run_kernel_trace.csv")))
            if "sample_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    b = last_json(bench_json)
    rf = b["roofline"]
    k = b["steps"]
    timed = ms[-k:]
    srt, tsrt = sorted(ms), sorted(timed)
    mean_t = sum(timed) / len(timed)
    flop = rf["flop_per_launch"]
    ach = flop / (mean_t * 1e-3) / 1e12
    out = [f"rocprofv3 --kernel-trace, {rows[0]['Kernel_Name']} ({label}), {len(ms)} dispatches "
           f"({len(ms) - k} warm-up + {k} timed): mean {sum(ms) / len(ms):.4f} ms, median {srt[len(srt) // 2]:.4f} ms, "
           f"min {srt[0]:.4f} ms, max {srt[-1]:.4f} ms; mean of the {k} timed dispatches {mean_t:.4f} ms, "
           f"median {tsrt[len(tsrt) // 2]:.4f} ms",
           "per-dispatch ms: " + ", ".join(f"{v:.4f}" for v in ms),
           f"bench.py line under rocprofv3 (same command): HIP-event avg_launch_ms {rf['avg_launch_ms']:.4f}, "
           f"median {rf['median_launch_ms']:.4f}",
           f"roofline from the rocprof timed mean: {flop / 1e12:.4f} TFLOP / {mean_t:.4f} ms = {ach:.1f} TF = "
           f"{ach / rf['peak']:.4f} of {rf['peak']} TF ({rf['bound']} bound; bench line frac {rf['frac']})"]
    return "\n".join(out) + "\n"


def main():
    tag = sys.argv[1]
    for name in ("bench.json", "bench_config3_bf16_k100.json", "bench_config5_share_2560rows.json",
                 "bench_under_rocprof.json", "c3_bench_under_rocprof.json", "f16x3_bench_under_rocprof.json",
                 "smoke.txt", "phase_trace_bf16.txt", "phase_trace_f16x3.txt"):
        shutil.copy(os.path.join(G, f"{tag}_{name}"), os.path.join(P, f"{tag}_{name}"))
    shutil.copy(os.path.join(G, f"{tag}_phase_trace.txt"), os.path.join(P, f"{tag}_phase_trace_fp32.txt"))
    shutil.copy(os.path.join(G, f"{tag}_gpu_tests.log"), os.path.join(P, f"{tag}_gpu_tests.txt"))
    for sub, bj, label in (("", "bench_under_rocprof.json", "headline fp32, BASELINE config 2, K=50"),
                           ("_c3", "c3_bench_under_rocprof.json", "BASELINE config 3, bf16 study, K=100"),
                           ("_f16x3", "f16x3_bench_under_rocprof.json", "config 2 in gemm mode f16x3, K=50")):
        shutil.copy(os.path.join(G, f"{tag}{sub}_prof", "run_kernel_stats.csv"),
                    os.path.join(P, f"{tag}{sub}_kernel_stats.csv"))
        with open(os.path.join(P, f"{tag}{sub}_kernel_trace_summary.txt"), "w") as f:
            f.write(trace_summary(tag, sub, os.path.join(G, f"{tag}_{bj}"), label))
    sq = []
    for sub, k, kern, label in (("_c3", 100, "sample_kernel<0", f"bf16 config 3 ({tag})"),
                                ("_f16x3", 50, "sample_kernel<0", f"f16x3 config 2 ({tag})")):
        for p in ("pmc_sq", "pmc_sq2"):
            shutil.copy(os.path.join(G, f"{tag}{sub}_{p}", "run_counter_collection.csv"),
                        os.path.join(P, f"{tag}{sub}_{p}.csv"))
        sq.append(subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), str(k),
                                  os.path.join(G, f"{tag}{sub}_pmc_sq"), os.path.join(G, f"{tag}{sub}_pmc_sq2"),
                                  kern, label], check=True, capture_output=True, text=True).stdout)
    open(os.path.join(P, f"{tag}_sq_summary.txt"), "w").write("".join(sq))
    print("".join(sq))
    for sub in ("", "_c3", "_f16x3"):
        print(open(os.path.join(P, f"{tag}{sub}_kernel_trace_summary.txt")).read().splitlines()[0][-200:])


if __name__ == "__main__":
    main()
