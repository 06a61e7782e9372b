# Round-4 check on a gpurun box: bash tools/r04_check.sh TAG [ab]
# every -m gpu test (achieved parity deltas logged to ${TAG}_deltas.jsonl), smoke(), the headline bench
# line, and (with "ab") a paired A/B of the in-tree library against ab/*.so.
TAG=${1:-r04}
O=gpurun_out; mkdir -p $O
rm -f $O/${TAG}_deltas.jsonl
DPK_DELTA_LOG=$O/${TAG}_deltas.jsonl timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -rP --timeout 240 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/${TAG}_gpu_tests.log | head -30; tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
grep -E "passed|failed" $O/${TAG}_gpu_tests.log | tail -1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${TAG}_smoke.txt 2>&1 || { tail -20 $O/${TAG}_smoke.txt; exit 2; }
tail -1 $O/${TAG}_smoke.txt
timeout -k 10 300 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -5 $O/${TAG}_bench.err; exit 3; }
cut -c1-400 $O/${TAG}_bench.json
if [ "$2" = ab ]; then
  for rep in 1 2 3; do
    for lib in default ab/*.so; do
      if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
      timeout -k 10 120 python3 bench.py --no-cpu --no-variants --steps 20 > $O/ab.json 2>/dev/null || exit 4
      python3 -c "import json,sys; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('AB $lib', d['value'], d['roofline']['avg_launch_ms'])" | tee -a $O/${TAG}_ab.txt
    done
  done
  unset DPK_LIB
fi
if [ "$3" = generic ] || [ "$2" = generic ]; then
  timeout -k 10 300 python3 tools/generic_bench.py > $O/${TAG}_generic_bench.txt 2>&1 || { tail -5 $O/${TAG}_generic_bench.txt; exit 5; }
  cat $O/${TAG}_generic_bench.txt
fi
echo done
