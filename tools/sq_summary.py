"""Per-SIMD, per-DDIM-step view of two rocprofv3 SQ passes of the sampler kernel.

  python tools/sq_summary.py K PASS1_DIR PASS2_DIR [kernel substring] [label]

PASS1: SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
PASS2: SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU
Counts are medians over the kernel's dispatches; instruction counts are divided by the 1,024 SIMDs (so a
layout with two waves per SIMD is compared per SIMD, not per wave), cycles by the 8 XCDs (GRBM_GUI_ACTIVE).
The wait counters are fractions of wave-cycles (both in the same units).
"""
import collections
import csv
import os
import sys

SIMDS = 1024


def load(d, kern):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if kern in r["Kernel_Name"]:
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (_, c), v in agg.items():
        per[c].append(v)
    return {c: sorted(v)[len(v) // 2] for c, v in per.items()}, {r for r, _ in agg}


def main():
    K = int(sys.argv[1])
    kern = sys.argv[4] if len(sys.argv) > 4 else "sample_kernel<0"
    label = sys.argv[5] if len(sys.argv) > 5 else ""
    a, da = load(sys.argv[2], kern)
    b, _ = load(sys.argv[3], kern)
    m = {**a, **b}
    cyc = m["GRBM_GUI_ACTIVE"] / 8 / K
    mfma_i = m["SQ_INSTS_MFMA"] / SIMDS / K
    valu_i = m["SQ_INSTS_VALU"] / SIMDS / K
    print(f"{label} K={K} dispatches={len(da)} waves={m['SQ_WAVES']:.0f} ({m['SQ_WAVES'] / SIMDS:.0f} per SIMD)")
    print(f"  cycles per step            {cyc / 1e3:8.1f}k")
    print(f"  MFMA pipe busy             {m['SQ_VALU_MFMA_BUSY_CYCLES'] / SIMDS / K / 1e3:8.1f}k  "
          f"({m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * SIMDS):.3f})")
    print(f"  MFMA instructions / SIMD   {mfma_i / 1e3:8.2f}k")
    print(f"  other VALU instr. / SIMD   {(valu_i - mfma_i) / 1e3:8.2f}k")
    print(f"  LDS instructions / SIMD    {m['SQ_INSTS_LDS'] / SIMDS / K / 1e3:8.2f}k")
    print(f"  issue stalls               {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.3f} of wave-cycles")
    print(f"  waits (waitcnt/barrier)    {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f} of wave-cycles")
    print(f"  wave-cycles per SIMD-cycle {m['SQ_WAVE_CYCLES'] * 4 / (m['GRBM_GUI_ACTIVE'] / 8 * SIMDS):.2f}"
          "  (SQ_WAVE_CYCLES in 4-cycle units: resident waves per SIMD)")


if __name__ == "__main__":
    main()
