# The hid-64 / 2-head persistent-sampler instance (dpkn, d_k 32, round 5): the generic-shape tests (both
# paths), the parity subset of the shipped shape, then tools/generic_bench.py.
#   bash tools/r05_dpkn_check.sh TAG
TAG=${1:-r05_dpkn}
O=gpurun_out; mkdir -p $O
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_generic_shapes.py -x -v --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
timeout -k 10 300 python3 tools/generic_bench.py > $O/${TAG}_generic_bench.txt 2>&1 || { tail -5 $O/${TAG}_generic_bench.txt; exit 2; }
cat $O/${TAG}_generic_bench.txt
