# Round-6 check + profile on a 1xMI355X gpurun box (repo root; the default bench line carries config 3 as
# variants.config3_bf16 since round 6, the separate config-3 line is kept for its whole-batch parity):
#   gpurun --timeout 1200 -- 'bash tools/profile_r06.sh r06_vX'
# GPU tests + smoke, bench lines (headline with the whole-batch CPU baseline, config 3, config 5 share,
# f16x3), rocprofv3 kernel traces (headline, config 3, f16x3) and SQ passes of the low-precision launches,
# FETCH_SIZE / WRITE_SIZE passes (headline and config 3, tools/traffic_from_pmc.py), phase traces.  Each GPU step has its own limit; the chain stops at the first failure.
TAG=${1:-r06_vX}
O=gpurun_out
mkdir -p $O
R=$(pwd)
set -o pipefail
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
tail -2 $O/${TAG}_gpu_tests.log
step smoke
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.txt 2>&1 || exit 2
tail -2 $O/${TAG}_smoke.txt
step bench
timeout -k 10 500 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit 3
cut -c1-300 $O/${TAG}_bench.json
step config3
timeout -k 10 300 python3 bench.py --config 3 --cpu-frames 256 --cpu-repeats 1 > $O/${TAG}_bench_config3_bf16_k100.json 2>> $O/${TAG}_bench.err || exit 4
step config5_share
timeout -k 10 200 python3 bench.py --config 5 --total-frames 128 --no-cpu > $O/${TAG}_bench_config5_share_2560rows.json 2>> $O/${TAG}_bench.err || exit 5
cd /tmp && export TMPDIR=/tmp
step kernel_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/${TAG}_prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-variants > $R/$O/${TAG}_bench_under_rocprof.json 2> $R/$O/${TAG}_prof.err || exit 6
step kernel_trace_config3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/${TAG}_c3_prof -o run -- python3 $R/bench.py --config 3 --steps 10 --warmup 2 --no-cpu --no-variants > $R/$O/${TAG}_c3_bench_under_rocprof.json 2> $R/$O/${TAG}_c3_prof.err || exit 7
step kernel_trace_f16x3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/${TAG}_f16x3_prof -o run -- python3 $R/bench.py --gemm f16x3 --steps 10 --warmup 2 --no-cpu --no-variants > $R/$O/${TAG}_f16x3_bench_under_rocprof.json 2> $R/$O/${TAG}_f16x3_prof.err || exit 8
step pmc_sq_config3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/${TAG}_c3_pmc_sq -o run -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 9
step pmc_sq2_config3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $R/$O/${TAG}_c3_pmc_sq2 -o run -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 10
step pmc_sq_f16x3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/${TAG}_f16x3_pmc_sq -o run -- python3 $R/bench.py --gemm f16x3 --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 11
step pmc_sq2_f16x3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $R/$O/${TAG}_f16x3_pmc_sq2 -o run -- python3 $R/bench.py --gemm f16x3 --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 12
for cfg in "fp32:" "c3:--config 3"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_${c}_$n
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/$O/${TAG}_${n}_pmc_$c -o run -- python3 $R/bench.py $a --steps 3 --warmup 1 --no-cpu --no-variants > /dev/null 2>&1 || exit 16
  done
done
cd $R
step phase_trace
timeout -k 10 120 python3 tools/phase_trace.py --run > $O/${TAG}_phase_trace.txt 2>&1 || exit 13
timeout -k 10 120 python3 tools/phase_trace.py --run --gemm f16x3 > $O/${TAG}_phase_trace_f16x3.txt 2>&1 || exit 14
timeout -k 10 120 python3 tools/phase_trace.py --run --gemm bf16 > $O/${TAG}_phase_trace_bf16.txt 2>&1 || exit 15
echo done
