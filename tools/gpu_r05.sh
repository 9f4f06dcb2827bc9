# round 5: full -m gpu suite, smoke, the driver's line (with its side windows and CPU baseline)
set -o pipefail
O=gpurun_out/r05
T=${1:-a}
mkdir -p $O
CN_RESULTS_DIR=gpurun_out timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/${T}_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
tail -1 $O/${T}_smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_bench_driver.log 2>&1 || exit $?
python tools/line_summary.py $O/${T}_bench_driver.log
if [ -n "$TIMELINE" ]; then
  CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 200 python -u tools/probe_timeline.py 400 c2 > $O/${T}_timeline_c2.log 2>&1 || exit $?
  tail -3 $O/${T}_timeline_c2.log
fi
