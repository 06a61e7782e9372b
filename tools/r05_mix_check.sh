# f16x3 lo halves by v_fma_mix (build/ab/mix.so, -DDPK_F16MIX=1): bitwise against the in-tree build on a
# 1,024-pose K=50 sample, the f16x3 parity tests on it, then interleaved A/B timing.
#   bash tools/r05_mix_check.sh
O=gpurun_out; mkdir -p $O
set -o pipefail
timeout -k 10 120 python3 tools/dump_sample.py $O/mix_ref.npy f16x3 || exit 1
DPK_LIB=$GRAFT_REPO_ROOT/build/ab/mix.so timeout -k 10 120 python3 tools/dump_sample.py $O/mix_new.npy f16x3 || exit 2
python3 -c "
import numpy as np; a=np.load('$O/mix_ref.npy'); b=np.load('$O/mix_new.npy')
print('mix vs default f16x3: bitwise', np.array_equal(a, b), 'max|d|', float(np.abs(a.astype(np.float64)-b).max()))" || exit 3
DPK_LIB=$GRAFT_REPO_ROOT/build/ab/mix.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_modes.py -x -q --timeout 120 --timeout-method thread > $O/r05_mix_tests.log 2>&1 || { tail -30 $O/r05_mix_tests.log; exit 4; }
tail -1 $O/r05_mix_tests.log
bash tools/ab_lowp.sh 2 default build/ab/mix.so || exit 5
