"""Summarise a GPU run's parity-delta log (tests/conftest.record_delta, DPK_DELTA_LOG) as a table:
   python tools/deltas_summary.py gpurun_out/r04_t1_deltas.jsonl > profiles/r04_parity_deltas.txt
One row per check: the achieved delta, its bar and the margin (bar / delta)."""
import json
import sys


def main(path):
    rows = [json.loads(line) for line in open(path) if line.strip()]
    print(f"{len(rows)} parity checks, {sum(not r['pass'] for r in rows)} over their bar")
    print(f"{'check':78s} {'delta':>10s} {'bar':>9s} {'bar/delta':>9s}")
    for r in rows:
        ratio = r["tol"] / r["delta"] if r["delta"] > 0 else float("inf")
        print(f"{r['tag'][:78]:78s} {r['delta']:10.3e} {r['tol']:9.1e} {ratio:9.1f}")
    worst = {}
    for r in rows:
        k = r["tol"]
        worst[k] = max(worst.get(k, 0.0), r["delta"])
    print("largest delta per bar: " + ", ".join(f"bar {k:.0e}: {v:.3e}" for k, v in sorted(worst.items())))


if __name__ == "__main__":
    main(sys.argv[1])
