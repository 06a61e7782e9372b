#!/bin/bash
# Parity suite on a variant library, then interleaved A/B against the in-tree one and round-3 v21.
#   bash tools/r03_variant_check.sh NAME [REPS]     (build/ab/NAME.so from tools/build_variant.sh)
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
NAME=$1; REPS=${2:-3}
export DPK_LIB=$GRAFT_REPO_ROOT/build/ab/$NAME.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pose_masks.py tests/test_gpu_weight_ranges.py tests/test_gpu_config4.py \
  tests/test_gpu_pose_metrics.py tests/test_gpu_num_layers.py > $O/r03_${NAME}_tests.txt 2>&1 || { tail -30 $O/r03_${NAME}_tests.txt; exit 1; }
tail -2 $O/r03_${NAME}_tests.txt
unset DPK_LIB
bash tools/ab3.sh $REPS default build/ab/$NAME.so | tee $O/r03_ab_${NAME}.txt
