# fp32 headline A/B of two libdpk builds (interleaved) + the user-object release probe
O=gpurun_out; mkdir -p $O
timeout -k 10 120 python3 tools/probe_user_object_release.py > $O/r05_user_object_probe.txt 2>&1; cat $O/r05_user_object_probe.txt
timeout -k 10 600 bash tools/ab3.sh 3 "$@" > $O/r05_ab_fp32.txt 2>&1; cat $O/r05_ab_fp32.txt
