# Round-3 GPU check, run from the repo root on a gpurun box:  bash tools/r03_check.sh TAG
# All -m gpu tests, the weight-range deltas (printed), then the headline bench line.
# Every GPU step has its own time limit; the chain stops at the first failure.
TAG=${1:-r03}
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { tail -40 $O/${TAG}_gpu_tests.log; exit 1; }
tail -2 $O/${TAG}_gpu_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_weight_ranges.py tests/test_gpu_config4.py -m gpu -q -s --timeout 240 --timeout-method thread > $O/${TAG}_weight_ranges.log 2>&1 || { tail -30 $O/${TAG}_weight_ranges.log; exit 2; }
grep -E "weight-range|config 4" $O/${TAG}_weight_ranges.log
timeout -k 10 300 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -5 $O/${TAG}_bench.err; exit 3; }
cut -c1-400 $O/${TAG}_bench.json
echo done
