set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --workload c3 --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c3.log | cut -c1-200
timeout -k 10 200 python -u bench.py --steps 1000 --warmup 50 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-200
bash profiles/run_profile.sh ${1:-r02_f}
