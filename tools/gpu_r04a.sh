# round 4 a: fdiv_lp full-range check, -m gpu suite, smoke, driver-style C2 line (with steady_state), C3 / C4
# lines, hash-matched profile of the driver's exact invocation
set -o pipefail
mkdir -p gpurun_out/r04
O=gpurun_out/r04
timeout -k 10 300 tools/bin/fdiv_lp_check 4 > $O/a_fdiv_lp_check.log 2>&1; rc=$?; cat $O/a_fdiv_lp_check.log; [ $rc -le 1 ] || exit $rc
CN_RESULTS_DIR=gpurun_out timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/a_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/a_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/a_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/a_bench_driver.log 2>&1 || exit $?
tail -1 $O/a_bench_driver.log | cut -c1-300
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/a_bench_c3.log 2>&1 || exit $?
tail -1 $O/a_bench_c3.log | cut -c1-300
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 6 > $O/a_bench_c4.log 2>&1 || exit $?
tail -1 $O/a_bench_c4.log | cut -c1-300
bash profiles/run_profile.sh r04_a > $O/a_prof.log 2>&1 || exit $?
echo all done
