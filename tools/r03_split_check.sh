# Step-split tail plan check on a gpurun box: bash tools/r03_split_check.sh TAG
# the plan's GPU tests, config 5's per-GPU share under plans 2 / 1 / 0, then an A/B of the
# headline bench against a saved library (build/ab/v21.so).
TAG=${1:-r03_split}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_streams_graphs.py tests/test_gpu_pose_masks.py -m gpu -x -v --timeout 240 --timeout-method thread -k "tail_round or step_split or flag_slots or capture or streams or mask" > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
tail -3 $O/${TAG}_tests.log
for plan in 2 1 0; do
  DPK_TAIL_SPLIT=$plan timeout -k 10 200 python bench.py --config 5 --total-frames 128 --no-cpu --no-variants > $O/${TAG}_c5share_plan$plan.json 2> $O/${TAG}_c5_plan$plan.err || { tail -5 $O/${TAG}_c5_plan$plan.err; exit 2; }
  python3 -c "import json; d=json.loads(open('$O/${TAG}_c5share_plan$plan.json').read().strip().splitlines()[-1]); print('plan $plan', d['value'], d['ms_per_step'], d.get('roofline',{}).get('avg_launch_ms'))"
done
timeout -k 10 200 python bench.py --no-cpu --no-variants > $O/${TAG}_full.json 2>/dev/null || exit 3
python3 -c "import json; d=json.loads(open('$O/${TAG}_full.json').read().strip().splitlines()[-1]); print('full', d['value'], d['ms_per_step'])"
bash tools/ab_bench.sh build/ab/v21.so || exit 4
echo done
