set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in c2 c5 c3; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload $w > gpurun_out/bench_$w.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$w.log | cut -c80-135
done
