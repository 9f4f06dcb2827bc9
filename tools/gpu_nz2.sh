set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_norm_zone.py tests/test_mixed.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_new.log 2>&1; rc=$?; echo new rc=$rc; tail -1 gpurun_out/gpu_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload c5 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log | cut -c80-135
