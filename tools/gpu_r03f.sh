# fused spatial attention: full -m gpu suite, smoke, driver-style C2 bench, C4 bench, C4 per-op attribution
set -o pipefail
mkdir -p gpurun_out
CN_RESULTS_DIR=gpurun_out timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/f_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/f_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/f_bench_driver.log 2>&1 || exit $?
tail -1 gpurun_out/f_bench_driver.log | cut -c1-250
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 10 > gpurun_out/f_bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/f_bench_c4.log | cut -c1-200
timeout -k 10 300 python -u tools/prof_c4_ops.py > gpurun_out/f_c4_ops.log 2>&1 || exit $?
echo all done
