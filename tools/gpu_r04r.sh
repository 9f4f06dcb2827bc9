# round 4 r: full -m gpu suite (incl. the new C4-shape and N = 25 DSRNN tests), smoke, C4 line
set -o pipefail
O=gpurun_out/r04
T=${1:-r}
mkdir -p $O
CN_RESULTS_DIR=gpurun_out timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed|c4_shape|N25|25\]" $O/${T}_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
tail -2 $O/${T}_smoke.log
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 6 > $O/${T}_bench_c4.log 2>&1 || exit $?
tail -1 $O/${T}_bench_c4.log | cut -c1-600
