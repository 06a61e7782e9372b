# Round-5 low-precision profile (BASELINE config 3 = bf16 K=100, and the f16x3 variant), run on a
# 1xMI355X gpurun box from the repo root:
#   gpurun --timeout 900 -- 'bash tools/profile_r05_lowp.sh r05_base'
# Writes gpurun_out/<tag>_*; the judged summaries are copied into profiles/ afterwards.
# Every GPU step has its own time limit and the chain stops at the first failure.
TAG=${1:-r05_vX}
O=gpurun_out
mkdir -p $O
R=$(pwd)
set -o pipefail
step() { echo "== $1 $(date +%T)"; }
step config3
timeout -k 10 200 python3 bench.py --config 3 --no-cpu > $O/${TAG}_bench_config3.json 2> $O/${TAG}_bench.err || exit 1
cut -c1-300 $O/${TAG}_bench_config3.json
step f16x3
timeout -k 10 200 python3 bench.py --gemm f16x3 --no-cpu --no-variants > $O/${TAG}_bench_f16x3.json 2>> $O/${TAG}_bench.err || exit 2
cut -c1-300 $O/${TAG}_bench_f16x3.json
cd /tmp && export TMPDIR=/tmp
step kernel_trace_config3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/${TAG}_c3_prof -o run -- python3 $R/bench.py --config 3 --steps 10 --warmup 2 --no-cpu --no-variants > $R/$O/${TAG}_c3_bench_under_rocprof.json 2> $R/$O/${TAG}_c3_prof.err || exit 3
step pmc_sq_config3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/${TAG}_c3_pmc_sq -o run -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 4
step pmc_sq2_config3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $R/$O/${TAG}_c3_pmc_sq2 -o run -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 5
step pmc_sq3_config3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/$O/${TAG}_c3_pmc_sq3 -o run -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 6
cd $R
step phase_trace
timeout -k 10 120 python3 tools/phase_trace.py --run --gemm f16x3 > $O/${TAG}_phase_trace_f16x3.txt 2>&1 || exit 7
timeout -k 10 120 python3 tools/phase_trace.py --run --gemm bf16 > $O/${TAG}_phase_trace_bf16.txt 2>&1 || exit 8
echo done
