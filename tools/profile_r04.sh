# Round-4 profiling recipe (same passes as round 3), run on a 1xMI355X gpurun box from the repo root:
#   gpurun --timeout 1200 -- 'bash tools/profile_r04.sh r04_v24'
# Writes gpurun_out/<tag>_*; the judged summaries are copied into profiles/ afterwards.
# Every GPU step has its own time limit and the chain stops at the first failure.
TAG=${1:-r04_vX}
O=gpurun_out
mkdir -p $O
R=$(pwd)
set -o pipefail
step() { echo "== $1"; }
step bench
timeout -k 10 300 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit 1
cut -c1-200 $O/${TAG}_bench.json
step config5_share
timeout -k 10 200 python3 bench.py --config 5 --total-frames 128 --no-cpu > $O/${TAG}_bench_config5_share.json 2>> $O/${TAG}_bench.err || exit 2
step config5_full
timeout -k 10 200 python3 bench.py --config 5 --no-cpu --no-variants > $O/${TAG}_bench_config5_h20_1gpu.json 2>> $O/${TAG}_bench.err || exit 3
step config3
timeout -k 10 300 python3 bench.py --config 3 --cpu-frames 256 > $O/${TAG}_bench_config3_bf16_k100.json 2>> $O/${TAG}_bench.err || exit 4
step launcher_world1
timeout -k 10 200 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --no-cpu --no-variants > $O/${TAG}_bench_rccl_world1.json 2>> $O/${TAG}_bench.err || exit 5
cd /tmp && export TMPDIR=/tmp
step kernel_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/${TAG}_prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-variants > $R/$O/${TAG}_bench_under_rocprof.json 2> $R/$O/${TAG}_prof.err || exit 6
step pmc_fetch
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/${TAG}_pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 7
step pmc_write
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/${TAG}_pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 8
step pmc_sq
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/${TAG}_pmc_sq -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 9
step pmc_sq2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $R/$O/${TAG}_pmc_sq2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 10
step pmc_f16x3_fetch
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/${TAG}_f16x3_pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants --gemm f16x3 > /dev/null 2>&1 || exit 11
step pmc_f16x3_write
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/${TAG}_f16x3_pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-variants --gemm f16x3 > /dev/null 2>&1 || exit 12
cd $R
step phase_trace
timeout -k 10 120 python3 tools/phase_trace.py --run > $O/${TAG}_phase_trace.txt 2>&1 || exit 13
timeout -k 10 120 python3 tools/phase_trace.py --run --gemm f16x3 > $O/${TAG}_phase_trace_f16x3.txt 2>&1 || exit 14
echo done
