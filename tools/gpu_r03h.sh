# round 3 end (sources of HEAD): full -m gpu suite, smoke, driver-style C2 bench, C4 bench, hash-matched C2
# profile passes, 2000-step C2, C3, C5 benches
set -o pipefail
mkdir -p gpurun_out
CN_RESULTS_DIR=gpurun_out timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/h_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/h_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/h_bench_driver.log 2>&1 || exit $?
tail -1 gpurun_out/h_bench_driver.log | cut -c1-200
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 10 > gpurun_out/h_bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/h_bench_c4.log | cut -c1-200
bash tools/gpu_r03g.sh r03_e
