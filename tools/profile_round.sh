R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python3 $R/bench.py > $R/gpurun_out/r01_v5_bench.json 2> $R/gpurun_out/r01_v5_bench.err || exit 1
cut -c1-200 $R/gpurun_out/r01_v5_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_v5 -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/prof_v5_bench.json 2>$R/gpurun_out/prof_v5.err || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_v5 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_v5 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_sq_v5 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 5
echo done
