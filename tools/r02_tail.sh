# Tail-split check on a gpurun box: GPU tests, then config 5's per-GPU share with and without
# the 2-pose tail tiles, and the 1024-pose headline.
O=gpurun_out; mkdir -p $O; T=${1:-r02_b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -2 $O/${T}_gpu_tests.log
timeout -k 10 200 python bench.py --config 5 --total-frames 128 --no-cpu > $O/${T}_c5share.json 2>&1 || exit 2
DPK_TAIL_SPLIT=0 timeout -k 10 200 python bench.py --config 5 --total-frames 128 --no-cpu --no-variants > $O/${T}_c5share_nosplit.json 2>&1 || exit 3
timeout -k 10 200 python bench.py --no-cpu > $O/${T}_bench.json 2>&1 || exit 4
timeout -k 10 200 python bench.py --no-cpu --frames 512 --no-variants > $O/${T}_bench512.json 2>&1 || exit 5
echo done
