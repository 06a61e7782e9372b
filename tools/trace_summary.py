"""Summarise a rocprofv3 --kernel-trace run of bench.py for the sampler kernel (build container).

  python tools/trace_summary.py PROF_DIR BENCH_LINE_JSON [--warmup 2]
Prints the per-dispatch durations of the bench line's sampler kernel (dpk::sample_kernel<0, *, G>, G the
line's GEMM mode), the mean and median of the timed dispatches (the first `warmup` are bench.py's
untimed warm-up calls), the bench line's own HIP-event figures from the same profiled run, and the
roofline from the rocprof mean against the line's own peak.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("bench_json")
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    line = json.loads(open(a.bench_json).read().strip().splitlines()[-1])
    gm = {"fp32": 0, "f16x3": 1, "bf16": 2}[line["config"]["gemm"]]
    rows = []
    for f in glob.glob(os.path.join(a.prof_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if f"sample_kernel<0, true, {gm}, 0>" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
                             r["Kernel_Name"]))
    rows.sort()
    ms = [r[1] for r in rows]
    timed = ms[a.warmup:]
    rf = line["roofline"]
    peak = rf["peak"]
    flop = rf["flop_per_launch"]
    mean_t = statistics.mean(timed)
    print(f"rocprofv3 --kernel-trace, {rows[0][2]} ({line['config']['workload']}), {len(ms)} dispatches ({a.warmup} warm-up + "
          f"{len(timed)} timed): mean {statistics.mean(ms):.4f} ms, median {statistics.median(ms):.4f} ms, "
          f"min {min(ms):.4f} ms, max {max(ms):.4f} ms; mean of the {len(timed)} timed dispatches {mean_t:.4f} ms, "
          f"median {statistics.median(timed):.4f} ms")
    print("per-dispatch ms: " + ", ".join(f"{v:.4f}" for v in ms))
    print(f"bench.py line under rocprofv3 (same command): HIP-event avg_launch_ms {rf['avg_launch_ms']:.4f}, "
          f"median {rf['median_launch_ms']:.4f}")
    tf = flop / (mean_t * 1e-3) / 1e12
    print(f"roofline from the rocprof timed mean: {flop / 1e12:.4f} TFLOP / {mean_t:.4f} ms = {tf:.1f} TF = "
          f"{tf / peak:.4f} of {peak} TF ({line['config']['gemm']} bound; bench line frac {rf['frac']})")


if __name__ == "__main__":
    main()
