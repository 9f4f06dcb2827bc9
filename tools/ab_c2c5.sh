set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_norm_zone.py tests/test_mixed.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_new.log 2>&1; rc=$?; echo tests rc=$rc; tail -1 gpurun_out/gpu_new.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/c2_head_$k.log 2>&1 || exit $?
tail -1 gpurun_out/c2_head_$k.log | cut -c80-125
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_k.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/c2_k_$k.log 2>&1 || exit $?
tail -1 gpurun_out/c2_k_$k.log | cut -c80-125
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload c5 > gpurun_out/c5_head.log 2>&1 || exit $?
tail -1 gpurun_out/c5_head.log | cut -c80-125
