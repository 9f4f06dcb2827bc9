set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k free_running > gpurun_out/gpu_fr.log 2>&1; rc=$?; tail -1 gpurun_out/gpu_fr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --workload c3 --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
echo $(tail -1 gpurun_out/bench_c3.log | cut -c90-150)
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c3 > gpurun_out/stamps.log 2>&1 || exit $?
grep -E "spawn waves|kernel A" gpurun_out/stamps.log
