set -o pipefail
for k in 1 2 3; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/c2_head_$k.log 2>&1 || exit $?
tail -1 gpurun_out/c2_head_$k.log | cut -c80-125
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_k.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/c2_k_$k.log 2>&1 || exit $?
tail -1 gpurun_out/c2_k_$k.log | cut -c80-125
done
