# 4-pose tiles on 8 waves (DPK_W8=1) against 4 waves, low-precision modes: parity subset, then A/B
O=gpurun_out; mkdir -p $O
set -o pipefail
DPK_W8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_tolerance.py tests/test_gpu_gemm_modes.py -x -q --timeout 120 --timeout-method thread > $O/r05_w8_tests.log 2>&1; tail -3 $O/r05_w8_tests.log
for rep in 1 2; do
for c in 0 1; do
  DPK_W8=$c timeout -k 10 120 python3 bench.py --config 3 --no-cpu --steps 10 > $O/ab.json 2>/dev/null || exit 1
  b=$(python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_ms'])")
  DPK_W8=$c timeout -k 10 120 python3 bench.py --gemm f16x3 --no-cpu --no-variants --steps 20 > $O/ab.json 2>/dev/null || exit 2
  f=$(python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_ms'])")
  echo "w8=$c bf16_c3 $b f16x3 $f"
done
done
