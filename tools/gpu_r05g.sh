# round 5: reset kernel draws the next spawns -- GPU suite, C3 driver-style window + steady line, C3 early timeline
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
CN_RESULTS_DIR=gpurun_out timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_driver_style.log 2>&1 || exit $?
python tools/line_summary.py $O/c3_driver_style.log
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_timeline.py 40 c3 > $O/timeline_c3.log 2>&1 || exit $?
grep -v amdgpu $O/timeline_c3.log | head -14
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit $?
python tools/line_summary.py $O/bench_driver.log
