# GPU: whole suite, smoke, C2 bench (with CPU baseline), C3/C5 benches, then the profile passes of the C2 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo pytest rc=$rc; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c80-135
for w in c3 c5; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload $w > gpurun_out/bench_$w.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$w.log | cut -c80-135
done
timeout -k 10 1000 bash profiles/run_profile.sh ${1:-r02_j} || exit $?
