mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "philox or free_running" > gpurun_out/gpu_philox.log 2>&1; rc=$?
tail -25 gpurun_out/gpu_philox.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_mt.log 2>&1 || exit $?
tail -1 gpurun_out/bench_mt.log
timeout -k 10 200 python bench.py --no-cpu-baseline --rng philox > gpurun_out/bench_phx.log 2>&1 || exit $?
tail -1 gpurun_out/bench_phx.log
