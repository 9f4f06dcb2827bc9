# one GPU call: the named test files, then the C2 bench twice (variance)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$@" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_new.log 2>&1; rc=$?; echo new rc=$rc; tail -3 gpurun_out/gpu_new.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$k.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$k.log | cut -c1-200
done
