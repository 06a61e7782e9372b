# Paired A/B of the in-tree libdpk against ab/*.so on a gpurun box: bash tools/ab_round.sh TAG [REPS]
# (bench.py --no-cpu --no-variants --steps 20 per library, libraries interleaved per repetition)
TAG=${1:-r04_ab}; REPS=${2:-3}
O=gpurun_out; mkdir -p $O
for rep in $(seq 1 $REPS); do
  for lib in default ab/*.so; do
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 120 python3 bench.py --no-cpu --no-variants --steps 20 > $O/ab.json 2>/dev/null || exit 4
    python3 -c "import json,sys; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('AB $lib', d['value'], d['roofline']['avg_launch_ms'])" | tee -a $O/${TAG}.txt
  done
done
unset DPK_LIB
python3 - $O/${TAG}.txt <<'PY'
import sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    p = line.split()
    if p and p[0] == "AB":
        d[p[1]].append(float(p[3]))
base = sum(d["default"]) / len(d["default"])
for k, v in d.items():
    m = sum(v) / len(v)
    print(f"{k:28s} mean launch {m:.4f} ms over {len(v)}  vs default {100 * (base / m - 1):+.2f} %")
PY
