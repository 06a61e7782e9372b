# Co-resident 2-pose tiles (two workgroups per CU, DPK_CORES=1) against the 4-pose tiles, low-precision modes:
#   bash tools/r05_cores_ab.sh [lib.so ...]   ("default" = the in-tree library)
O=gpurun_out; mkdir -p $O
set -o pipefail
for rep in 1 2; do
for lib in "$@"; do
for c in 0 1; do
  if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
  DPK_CORES=$c timeout -k 10 120 python3 bench.py --config 3 --no-cpu --steps 10 > $O/ab.json 2>/dev/null || exit 1
  b=$(python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_ms'])")
  echo "$lib cores=$c bf16_c3 $b"
done
done
done
