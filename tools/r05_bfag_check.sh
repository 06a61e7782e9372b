# gemm mode 2 (config 3's bf16 study) with attention (DPK_BF_ATTN) and the GraphNet products (DPK_BF_GRAPH) on
# bf16 MFMA: the bf16 tolerance tests and the f16x3 tests on the in-tree build, then per library (prev = both
# off, bfa = attention only, bfag = attention + graph, default = + Chebyshev) the config-3 line's parity (128 frames) and timing.
#   bash tools/r05_bfag_check.sh REPS lib...
O=gpurun_out; mkdir -p $O
set -o pipefail
REPS=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_tolerance.py tests/test_gpu_gemm_modes.py -q --timeout 120 --timeout-method thread > $O/r05_bfag_tests.log 2>&1
rc=$?; [ $rc = 0 ] || [ $rc = 1 ] || { tail -40 $O/r05_bfag_tests.log; exit 1; }     # 1: failed asserts (the study's bars), reported
grep -E "^(FAILED|E  )|passed|failed" $O/r05_bfag_tests.log | head -20
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 120 python3 bench.py --config 3 --cpu-frames 128 --cpu-repeats 1 --no-variants --steps 10 > $O/ab.json 2>/dev/null || exit 2
    python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); p=d['parity']; print('$lib', 'bf16_c3', d['value'], d['roofline']['avg_launch_ms'], 'parity', p['frames'], 'dmpjpe_mm', p['mpjpe_delta_mm'], 'maxabs', p['max_abs_diff'])" || exit 3
  done
done
