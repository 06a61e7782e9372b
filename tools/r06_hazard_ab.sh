# Round 6, verdict r05 item 1 (GPU box): the MFMA-result pads (mfma_pad) and the two woven-epilogue variants that
# round 5 found wrong without them.  Bitwise A/B of every instance against round 5's library (build/ab/head.so),
# then interleaved timing of fp32 (config 2), bf16 (config 3, K=100) and f16x3.
#   bash tools/r06_hazard_ab.sh TAG lib1.so lib2.so ...      (the in-tree library is "default")
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
LIBS="build/ab/head.so default $*"
for lib in $LIBS; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
  timeout -k 10 240 python3 -u tools/bitwise_ab.py dump $O/$n.npz > $O/dump_$n.log 2>&1 || { echo "dump $n failed"; tail -20 $O/dump_$n.log; exit 1; }
  echo "dumped $n"
done
unset DPK_LIB
for lib in $LIBS; do
  n=$(basename $lib .so)
  [ "$n" = head ] && continue
  python3 tools/bitwise_ab.py compare $O/head.npz $O/$n.npz > $O/cmp_$n.txt
  echo "== $n vs head: $(tail -1 $O/cmp_$n.txt)"
  grep -v "bitwise equal" $O/cmp_$n.txt | head -12
done
for rep in 1 2; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    if [ "$lib" = default ]; then unset DPK_LIB; else export DPK_LIB=$GRAFT_REPO_ROOT/$lib; fi
    for cfg in "--config 2" "--config 3" "--config 2 --gemm f16x3"; do
      timeout -k 10 120 python3 bench.py --no-cpu --no-variants --steps 20 $cfg > $O/ab.json 2>/dev/null || { echo "bench $n $cfg failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$rep $n', '$cfg'.replace(' ', ''), round(d['value']), d['roofline']['avg_launch_ms'])" | tee -a $O/timing.txt
    done
  done
done
echo done
