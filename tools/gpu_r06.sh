# round 6: full -m gpu suite, smoke, the driver's line (with its side windows and CPU baseline)
#   bash tools/gpu_r06.sh <tag>        -> gpurun_out/r06/<tag>_{tests,smoke,bench_driver}.log
set -o pipefail
O=gpurun_out/r06
T=${1:-a}
mkdir -p $O
CN_RESULTS_DIR=gpurun_out timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/${T}_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
tail -1 $O/${T}_smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_bench_driver.log 2>&1 || exit $?
python tools/line_summary.py $O/${T}_bench_driver.log
