# Kernel breakdown of the generic-shape path (hid 128 / 8 heads / 5 layers, B=1024, K=50) on a gpurun box:
#   gpurun -- 'bash tools/generic_profile.sh TAG'
TAG=${1:-r04_generic}
O=gpurun_out; mkdir -p $O; R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/${TAG}_prof -o run -- python3 $R/tools/generic_bench.py 128 8 5 > $R/$O/${TAG}_bench.txt 2> $R/$O/${TAG}_prof.err || { tail -5 $R/$O/${TAG}_prof.err; exit 1; }
cat $R/$O/${TAG}_bench.txt
f=$(ls $R/$O/${TAG}_prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $R/$O/${TAG}_prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -20
