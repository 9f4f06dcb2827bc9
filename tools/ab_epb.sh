set -o pipefail
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload c5 --steps 1000 > gpurun_out/c5_base.log 2>&1 || exit $?
tail -1 gpurun_out/c5_base.log | cut -c80-130
for w in 16 8; do
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_epb$w.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload c5 --steps 1000 > gpurun_out/c5_epb$w.log 2>&1 || exit $?
tail -1 gpurun_out/c5_epb$w.log | cut -c80-130
done
