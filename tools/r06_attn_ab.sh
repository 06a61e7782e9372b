# Round 6 (verdict r05 item 4): bf16 attention variants on the GPU box.  For each library: the bf16 tolerance
# tests, the default bench line (its variants.config3_bf16 carries the parity study against the oracle on the
# whole 1,024-frame batch), then interleaved config-3 timing against the in-tree library.
#   bash tools/r06_attn_ab.sh TAG lib1.so ...
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
for lib in "$@"; do
  n=$(basename $lib .so)
  export DPK_LIB=$GRAFT_REPO_ROOT/$lib
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_tolerance.py tests/test_gpu_gemm_modes.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests_$n.log 2>&1 || { tail -20 $O/tests_$n.log; exit 1; }
  echo "$n tests: $(tail -1 $O/tests_$n.log)"
  timeout -k 10 400 python3 bench.py --cpu-repeats 1 > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().strip().splitlines()[-1]); c=d['variants']['config3_bf16']; print('$n', 'config3', c['value'], c['roofline']['frac'], c['parity']['bf16'], 'fp32', c['parity']['fp32'])"
done
for rep in 1 2 3; do
  for lib in default "$@"; do
    n=$(basename $lib .so)
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 120 python3 bench.py --no-cpu --no-variants --steps 20 --config 3 > $O/ab.json 2>/dev/null || { echo "bench $n failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$rep $n config3', round(d['value']), d['roofline']['avg_launch_ms'])" | tee -a $O/timing.txt
  done
done
echo done
