# Round-5 iteration check on a 1xMI355X gpurun box (repo root):
#   gpurun --timeout 900 -- 'bash tools/r05_iter.sh TAG [tests]'
# low-precision GEMM-mode parity tests, the config-3 and f16x3 bench lines, phase traces.
TAG=${1:-r05_it}
TESTS=${2:-"tests/test_gpu_gemm_modes.py tests/test_gpu_bf16_tolerance.py tests/test_gpu_weight_ranges.py"}
O=gpurun_out
mkdir -p $O
set -o pipefail
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1; rc=$?
tail -3 $O/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
step config3
timeout -k 10 200 python3 bench.py --config 3 --no-cpu > $O/${TAG}_bench_config3.json 2> $O/${TAG}_bench.err || exit 2
cut -c1-260 $O/${TAG}_bench_config3.json
step f16x3
timeout -k 10 200 python3 bench.py --gemm f16x3 --no-cpu --no-variants > $O/${TAG}_bench_f16x3.json 2>> $O/${TAG}_bench.err || exit 3
cut -c1-260 $O/${TAG}_bench_f16x3.json
step fp32
timeout -k 10 200 python3 bench.py --no-cpu --no-variants > $O/${TAG}_bench_fp32.json 2>> $O/${TAG}_bench.err || exit 4
cut -c1-260 $O/${TAG}_bench_fp32.json
step phase_trace
timeout -k 10 120 python3 tools/phase_trace.py --run --gemm f16x3 > $O/${TAG}_phase_trace_f16x3.txt 2>&1 || exit 5
timeout -k 10 120 python3 tools/phase_trace.py --run --gemm bf16 > $O/${TAG}_phase_trace_bf16.txt 2>&1 || exit 6
echo done
