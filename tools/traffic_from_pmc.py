"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes of the sampler kernel into profiles/traffic.json
(the bench line's roofline.traffic).  FETCH_SIZE is doubled per MI355X_MICROARCH.md's gfx950
correction (it counts half of the 16-B/lane streaming reads); both are KB per dispatch, the median over the
profiled dispatches (the first dispatch of a process can run with cold L2/MALL: round 5's fp32 pass read
32.6 MB for it against 11.3 MB for each later one).

  python tools/traffic_from_pmc.py KEY FETCH_DIR WRITE_DIR "SOURCE TEXT"
    KEY  rows{R}_K{K}[_gemm], the key bench.py looks up
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_median(d, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "sample_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for sample_kernel under {d}")
    vals.sort()
    return vals[len(vals) // 2]


def main():
    key, fdir, wdir, source = sys.argv[1:5]
    rows, k = key.split("_")[0][4:], key.split("_")[1][1:]
    fetch = kernel_median(fdir, "FETCH_SIZE")
    write = kernel_median(wdir, "WRITE_SIZE")
    path = os.path.join(ROOT, "profiles", "traffic.json")
    tr = json.load(open(path)) if os.path.exists(path) else {}
    old = tr.get(key, {})
    tr[key] = {"hbm_bytes_per_launch": int(round((2 * fetch + write) * 1024)), "fetch_size_kb_raw": fetch,
               "write_size_kb": write, "source": source,
               "algorithmic_bytes_per_launch": int(rows) * 680,
               "note": f"K={k}; weights (2.6 MB arena) re-read from L2/MALL by every XCD each launch; "
                       "HBM-side traffic ~ weight slices x 8 XCDs + the 680 B per pose of input and output"}
    for f in ("mfma_busy", "mfma_busy_source"):     # executed-work figures folded in separately are kept
        if f in old:
            tr[key][f] = old[f]
    json.dump(tr, open(path, "w"), indent=1)
    print(key, tr[key]["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
