# round 3 first call on the restored tree: full -m gpu suite, smoke, C2/C3 benches, hash-matched profile of C2
set -o pipefail
mkdir -p gpurun_out
CN_RESULTS_DIR=gpurun_out timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-600
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c3.log | cut -c1-300
timeout -k 10 1000 bash profiles/run_profile.sh r03_a > gpurun_out/prof.log 2>&1 || exit $?
echo all done
