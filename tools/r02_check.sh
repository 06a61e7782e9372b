# Round-2 GPU check: all -m gpu tests, then the bench lines (headline, config 5's per-GPU share,
# config 3).  Run from the repo root on a gpurun box:  bash tools/r02_check.sh TAG
TAG=${1:-r02}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
tail -2 $O/${TAG}_gpu_tests.log
timeout -k 10 300 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit 2
timeout -k 10 200 python bench.py --config 5 --total-frames 128 --no-cpu > $O/${TAG}_bench_c5_share.json 2> $O/${TAG}_bench_c5.err || exit 3
timeout -k 10 300 python bench.py --config 3 --cpu-frames 256 > $O/${TAG}_bench_c3.json 2> $O/${TAG}_bench_c3.err || exit 4
echo done
