#!/bin/bash
# Build an alternative libdpk for A/B timing (tools/ab_bench.sh): tools/build_variant.sh NAME [-DFLAG=V ...]
# -> build/ab/NAME.so (same flags as diffpose-nw_amd/Makefile plus the given defines).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$ROOT/build/ab"
cd "$ROOT/diffpose-nw_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -mllvm -misched-cluster=0 -mllvm -amdgpu-disable-unclustered-high-rp-reschedule=1 \
    -I../include -Wno-unused-result "$@" csrc/dpk_kernels.hip csrc/dpk_metrics.hip csrc/dpk_gmm.hip \
    -o "$ROOT/build/ab/$NAME.so" 2>&1 | grep -v "hip-link" || true
test -f "$ROOT/build/ab/$NAME.so" && echo "built build/ab/$NAME.so $*"
