# round 3 end (sources of HEAD): hash-matched C2 profile passes, 2000-step C2, C3, C5 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 bash profiles/run_profile.sh ${1:-r03_e} > gpurun_out/prof.log 2>&1 || exit $?
tail -2 gpurun_out/prof.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/g_bench_2000.log 2>&1 || exit $?
tail -1 gpurun_out/g_bench_2000.log | cut -c1-200
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/g_bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/g_bench_c3.log | cut -c1-200
timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/g_bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/g_bench_c5.log | cut -c1-200
echo all done
