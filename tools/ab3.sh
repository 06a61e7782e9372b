# Interleaved A/B timing of libdpk builds on the GPU box: bash tools/ab3.sh REPS lib1.so lib2.so ...
# ("default" = the in-tree library).  Each run: bench.py --no-cpu --no-variants --steps 20.
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
REPS=$1; shift
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 120 python3 bench.py --no-cpu --no-variants --steps 20 > $O/ab.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$lib', d['value'], d['roofline']['avg_launch_ms'])"
  done
done
