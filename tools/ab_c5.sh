set -o pipefail
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload c5 --steps 1000 > gpurun_out/c5_new_$k.log 2>&1 || exit $?
tail -1 gpurun_out/c5_new_$k.log | cut -c80-130
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_satold.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload c5 --steps 1000 > gpurun_out/c5_old_$k.log 2>&1 || exit $?
tail -1 gpurun_out/c5_old_$k.log | cut -c80-130
done
