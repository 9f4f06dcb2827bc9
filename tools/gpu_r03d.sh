# round 3 end: full -m gpu suite, smoke, driver-style C2 bench (with cpu_baseline), C2 2000-step, C3, C5, C4
# benches, hash-matched profile of C2
set -o pipefail
mkdir -p gpurun_out
CN_RESULTS_DIR=gpurun_out timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit $?
tail -1 gpurun_out/bench_driver.log | cut -c1-300
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_2000.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/bench_c3.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 10 > gpurun_out/bench_c4.log 2>&1 || exit $?
timeout -k 10 1000 bash profiles/run_profile.sh r03_d > gpurun_out/prof.log 2>&1 || exit $?
echo all done
