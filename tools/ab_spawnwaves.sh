set -o pipefail
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload c3 --steps 1000 > gpurun_out/c3_256.log 2>&1 || exit $?
tail -1 gpurun_out/c3_256.log | cut -c80-130
for w in 384 512; do
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_sw$w.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload c3 --steps 1000 > gpurun_out/c3_$w.log 2>&1 || exit $?
tail -1 gpurun_out/c3_$w.log | cut -c80-130
done
