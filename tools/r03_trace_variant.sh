#!/bin/bash
# Phase trace of a traced variant library: DPK_* env as for its build.  bash tools/r03_trace_variant.sh NAME
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 200 python3 tools/phase_trace.py --run --so build/trace/trace_$1.so > $O/r03_trace_$1.txt 2>&1
