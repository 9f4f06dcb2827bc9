# round 6 final: full -m gpu suite, smoke, the driver's line, then the counter profiles of record
#   bash tools/gpu_r06_final.sh 1   -> suite, smoke, driver line, C2 profile (pmc_r06_i)
#   bash tools/gpu_r06_final.sh 2   -> C3 / C5 side-window profiles (pmc_r06_i_c3 / _c5)
set -o pipefail
O=gpurun_out/r06_final_i
mkdir -p $O
if [ "$1" = 1 ]; then
  CN_RESULTS_DIR=gpurun_out timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/f_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/f_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/f_smoke.log 2>&1 || exit $?
  tail -1 $O/f_smoke.log
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/f_bench_driver.log 2>&1 || exit $?
  python tools/line_summary.py $O/f_bench_driver.log
  bash profiles/run_profile.sh r06_i --gpus 1 --steps 20 --warmup 5 --no-side || exit $?
else
  bash profiles/run_profile.sh r06_i_c3 --workload c3 --steps 200 --warmup 100 --no-side || exit $?
  bash profiles/run_profile.sh r06_i_c5 --workload c5 --steps 200 --warmup 100 --no-side || exit $?
fi
