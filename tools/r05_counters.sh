# Round-5 counter passes: HBM traffic (FETCH_SIZE / WRITE_SIZE) of the shipped build in every GEMM mode
# (config 3 bf16 K=100, config 2 fp32 and f16x3), and SQ passes of the two experimental tile layouts
# (co-resident 2-pose tiles DPK_CORES=1, 8-wave 4-pose tiles DPK_W8=1; build/ab/expt.so built with
# tools/build_variant.sh expt -DDPK_EXPT_TILES=1) against which the shipped tiles' passes are read.
#   bash tools/r05_counters.sh TAG
TAG=${1:-r05_cnt}
R=$GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
set -o pipefail
step() { echo "[$(date +%T)] $1"; }
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants"
step fetch_c3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/${TAG}_c3_pmc_fetch -o run -- $B --config 3 > /dev/null 2>&1 || exit 3
step write_c3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/${TAG}_c3_pmc_write -o run -- $B --config 3 > /dev/null 2>&1 || exit 4
step fetch_fp32
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/${TAG}_pmc_fetch -o run -- $B > /dev/null 2>&1 || exit 5
step write_fp32
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/${TAG}_pmc_write -o run -- $B > /dev/null 2>&1 || exit 6
step fetch_f16x3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/${TAG}_f16x3_pmc_fetch -o run -- $B --gemm f16x3 > /dev/null 2>&1 || exit 7
step write_f16x3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/${TAG}_f16x3_pmc_write -o run -- $B --gemm f16x3 > /dev/null 2>&1 || exit 8
export DPK_LIB=$R/build/ab/expt.so
SQ1="SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"
n=10
for v in CORES W8; do
  for g in c3 f16x3; do
    if [ $g = c3 ]; then A="--config 3"; else A="--gemm f16x3"; fi
    for p in 1 2; do
      if [ $p = 1 ]; then C=$SQ1; else C=$SQ2; fi
      step "${v}_${g}_sq$p"
      export DPK_$v=1
      timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/$O/${TAG}_${v,,}_${g}_pmc_sq$p -o run -- $B $A > /dev/null 2>&1 || exit $n
      unset DPK_$v
      n=$((n+1))
    done
  done
done
step done
