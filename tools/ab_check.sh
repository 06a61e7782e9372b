# Parity subset + A/B timing of the in-tree library against alternatives: bash tools/ab_check.sh TAG lib1.so ...
TAG=$1; shift
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_weight_ranges.py tests/test_gpu_pose_masks.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { tail -30 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
bash tools/ab_bench.sh "$@" || exit 4
echo done
