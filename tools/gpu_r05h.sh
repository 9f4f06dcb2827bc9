# round 5: C2 window A/B (previous vs current library), C3 driver-style window, GPU suite
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
BENCH_ARGS="--steps 20 --warmup 5" bash tools/ab_c2.sh $O/ab_win2 crowdnav_dsrnn_amd/lib/variants/libcn_prev.so crowdnav_dsrnn_amd/lib/libcrowdnav_hip.so || exit $?
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_driver_style.log 2>&1 || exit $?
python tools/line_summary.py $O/c3_driver_style.log
CN_RESULTS_DIR=gpurun_out timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
