# A/B timing of alternative builds of libdpk on the GPU box: bash tools/ab_bench.sh lib1.so lib2.so ...
# (each run: bench.py --no-cpu --no-variants --steps 20; the in-tree library is "default")
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for rep in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$lib; fi
    timeout -k 10 120 python3 bench.py --no-cpu --no-variants --steps 20 > $O/ab.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$lib', d['value'], d['roofline']['avg_launch_ms'])"
  done
done
