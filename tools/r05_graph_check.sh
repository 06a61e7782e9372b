# The half-width GraphNet products (gemm mode 1: DPK_F16_GRAPH 3-term fp16 split; mode 2: DPK_BF_GRAPH=2 bf16
# hi + lo L_g): the low-precision and parity tests on the in-tree build, then per library the config-3 bf16 line
# and the config-2 f16x3 line with their parity (128 frames against the CPU oracle) and timing.
#   bash tools/r05_graph_check.sh REPS lib...      ("default" = the in-tree library)
O=gpurun_out; mkdir -p $O
set -o pipefail
REPS=$1; shift
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_tolerance.py tests/test_gpu_gemm_modes.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $O/r05_graph_tests.log 2>&1
rc=$?; [ $rc = 0 ] || [ $rc = 1 ] || { tail -40 $O/r05_graph_tests.log; exit 1; }
grep -E "^(FAILED|E  )|passed|failed" $O/r05_graph_tests.log | head -20
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
    for m in "--config 3" "--gemm f16x3"; do
      timeout -k 10 120 python3 bench.py $m --cpu-frames 128 --cpu-repeats 1 --no-variants --steps 10 > $O/ab.json 2>/dev/null || exit 2
      python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); p=d['parity']; print('$lib', '$m', d['value'], d['roofline']['avg_launch_ms'], 'parity', p['frames'], 'dmpjpe_mm', p['mpjpe_delta_mm'], 'maxabs', p['max_abs_diff'])" || exit 3
    done
  done
done
