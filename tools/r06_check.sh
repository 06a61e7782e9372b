# Round-6 check on a gpurun box (repo root):  bash tools/r06_check.sh TAG [tests] [lib1.so ...]
#   tests: every -m gpu test (parity deltas logged), smoke(), then the default bench line;
#   libs:  bitwise A/B of each library against the in-tree one (tools/bitwise_ab.py) and 2 interleaved
#          timing reps of config 2 fp32, config 3 bf16 and f16x3.
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
if [ "$1" = tests ]; then
  shift
  DPK_DELTA_LOG=$O/deltas.jsonl timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -3 $O/gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gpu_tests.log | head -20; exit 1; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
  timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -c 600 $O/bench.json
fi
[ $# -eq 0 ] && exit 0
unset DPK_LIB
timeout -k 10 240 python3 -u tools/bitwise_ab.py dump $O/default.npz > $O/dump_default.log 2>&1 || { tail -20 $O/dump_default.log; exit 1; }
for lib in "$@"; do
  n=$(basename $lib .so)
  DPK_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 240 python3 -u tools/bitwise_ab.py dump $O/$n.npz > $O/dump_$n.log 2>&1 || { tail -20 $O/dump_$n.log; exit 1; }
  python3 tools/bitwise_ab.py compare $O/default.npz $O/$n.npz > $O/cmp_$n.txt
  echo "== $n vs default: $(tail -1 $O/cmp_$n.txt)"
  grep -v "bitwise equal" $O/cmp_$n.txt | head -8
done
for rep in 1 2; do
  for lib in default "$@"; do
    n=$(basename $lib .so)
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
    for cfg in "--config 2" "--config 3" "--config 2 --gemm f16x3"; do
      timeout -k 10 120 python3 bench.py --no-cpu --no-variants --steps 20 $cfg > $O/ab.json 2>/dev/null || { echo "bench $n $cfg failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$rep $n', '$cfg'.replace(' ', ''), round(d['value']), d['roofline']['avg_launch_ms'])" | tee -a $O/timing.txt
    done
  done
done
echo done
