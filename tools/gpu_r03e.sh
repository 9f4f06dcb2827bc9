# round 3 re-entry: rebuilt library (same sources as r03_d) -- full -m gpu suite, smoke, driver-style C2 bench
set -o pipefail
mkdir -p gpurun_out
CN_RESULTS_DIR=gpurun_out timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit $?
tail -1 gpurun_out/bench_driver.log | cut -c1-400
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c3.log | cut -c1-300
echo all done
