O=gpurun_out; mkdir -p $O
set -o pipefail
timeout -k 10 120 python3 tools/probe_user_object_release.py > $O/r05_user_object_probe.txt 2>&1; cat $O/r05_user_object_probe.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_generic_shapes.py -x -q --timeout 200 --timeout-method thread > $O/r05_wide_tests.log 2>&1; tail -15 $O/r05_wide_tests.log
timeout -k 10 300 python3 tools/generic_bench.py > $O/r05_generic_bench.txt 2>&1; cat $O/r05_generic_bench.txt
