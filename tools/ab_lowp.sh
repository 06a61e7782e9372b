# Interleaved A/B timing of libdpk builds in the low-precision modes on the GPU box:
#   bash tools/ab_lowp.sh REPS lib1.so lib2.so ...   ("default" = the in-tree library)
# per lib: BASELINE config 3 (bf16, K=100) and the f16x3 variant at config 2, bench.py --no-cpu.
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
REPS=$1; shift
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 120 python3 bench.py --config 3 --no-cpu --steps 10 > $O/ab.json 2>/dev/null || exit 1
    b=$(python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_ms'])")
    timeout -k 10 120 python3 bench.py --gemm f16x3 --no-cpu --no-variants --steps 20 > $O/ab.json 2>/dev/null || exit 2
    f=$(python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_ms'])")
    echo "$lib bf16_c3 $b f16x3 $f"
  done
done
