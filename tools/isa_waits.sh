# Device ISA of the fp32 sampler kernel (build container): per barrier-delimited phase, its MFMA and
# wide-store counts and every s_waitcnt on vmcnt (global loads) inside it.  A vmcnt wait in a VALU
# phase that reads no global data is a false dependency (see layer_norm's vpair note).
#   bash tools/isa_waits.sh [extra hipcc -D flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p /tmp/dpk_isa
cd "$ROOT/diffpose-nw_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
  -mllvm -misched-cluster=0 -mllvm -amdgpu-disable-unclustered-high-rp-reschedule=1 -I../include --cuda-device-only -S "$@" \
  -o /tmp/dpk_isa/dpk.s csrc/dpk_kernels.hip 2>&1 | grep -v hip-link || true
cd /tmp/dpk_isa
L0=$(grep -n '^_ZN3dpk13sample_kernelILi0ELb1ELi0EEEvN10dpk_shared10SampleArgsEPKfPKc:' dpk.s | cut -d: -f1)
awk -v s=$L0 'NR>=s{print} NR>s && /s_endpgm/{exit}' dpk.s > k.s
awk '/s_waitcnt.*vmcnt/{w=w" "NR":"$2"("$3")"} /v_mfma_f32_16x16x4/{m++} /ds_write_b128/{d++}
     /s_barrier/{printf "%6d BARRIER  phase before: mfma %4d  ds_write_b128 %3d  vmcnt waits:%s\n", NR, m, d, (length(w) > 300 ? substr(w,1,300)"..." : w); m=0; d=0; w=""}' k.s
echo "v_readlane $(grep -c v_readlane k.s)  v_accvgpr_read $(grep -c v_accvgpr_read k.s)  lines $(wc -l < k.s)"
