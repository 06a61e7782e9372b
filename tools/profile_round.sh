# Round profiling recipe, run on a 1xMI355X gpurun box from the repo root:
#   gpurun --timeout 1200 -- 'bash tools/profile_round.sh r01_v6 [extra bench args]'
# Writes gpurun_out/<tag>_*; copy the summaries that are judged into profiles/.
R=$GRAFT_REPO_ROOT
TAG=${1:-r01_vX}
shift
EXTRA="$*"
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python3 $R/bench.py $EXTRA > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit 1
cut -c1-300 $O/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-variants $EXTRA > $O/${TAG}_bench_under_rocprof.json 2>$O/${TAG}_prof.err || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants $EXTRA > /dev/null 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants $EXTRA > /dev/null 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/${TAG}_pmc_sq -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants $EXTRA > /dev/null 2>&1 || exit 5
echo done
