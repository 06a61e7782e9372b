# Round-3 final check on a gpurun box: bash tools/r03_final.sh TAG
# every -m gpu test, smoke(), the headline bench line, config 5's share, the generic-path timing.
TAG=${1:-r03_final}
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { tail -40 $O/${TAG}_gpu_tests.log; exit 1; }
tail -2 $O/${TAG}_gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${TAG}_smoke.txt 2>&1 || { tail -20 $O/${TAG}_smoke.txt; exit 2; }
tail -1 $O/${TAG}_smoke.txt
timeout -k 10 300 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -5 $O/${TAG}_bench.err; exit 3; }
cut -c1-300 $O/${TAG}_bench.json
timeout -k 10 200 python3 bench.py --config 5 --total-frames 128 --no-cpu --no-variants > $O/${TAG}_c5share.json 2>> $O/${TAG}_bench.err || exit 4
python3 -c "import json; d=json.loads(open('$O/${TAG}_c5share.json').read().strip().splitlines()[-1]); print('config5 share rows/s', d.get('rows_per_s'), d['ms_per_step'])"
timeout -k 10 300 python3 tools/generic_bench.py > $O/${TAG}_generic_bench.txt 2>&1 || { tail -5 $O/${TAG}_generic_bench.txt; exit 5; }
cat $O/${TAG}_generic_bench.txt
echo done
