set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_policy.py tests/test_learner.py tests/test_lidar.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c4 > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | cut -c1-200
grep "c4 update" gpurun_out/bench_c4.log | tail -2
