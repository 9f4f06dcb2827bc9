set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mixed.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_new.log 2>&1; rc=$?; echo new rc=$rc; tail -2 gpurun_out/gpu_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_1.log | cut -c1-220
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c3 c5a c5b > gpurun_out/stamps.log 2>&1 || exit $?
cat gpurun_out/stamps.log
