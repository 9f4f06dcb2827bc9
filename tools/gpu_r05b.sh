# round 5, C3 rejection-loop work: GPU suite, C3 variants (goal-change cost, inline resets), C3 bench line;
# STAMPS=1 adds the stamps probe (per-pass cycles of the crowded loops; needs tools/build_stamps.sh first)
set -o pipefail
O=gpurun_out/r05b
T=${1:-a}
mkdir -p $O
CN_RESULTS_DIR=gpurun_out timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/${T}_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe_c3_variants.py > $O/${T}_c3_variants.log 2>&1 || exit $?
cat $O/${T}_c3_variants.log
timeout -k 10 300 python -u bench.py --workload c3 --steps 200 --warmup 100 --no-cpu-baseline > $O/${T}_bench_c3.log 2>&1 || exit $?
python tools/line_summary.py $O/${T}_bench_c3.log
if [ -n "$STAMPS" ]; then
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c3 > $O/${T}_stamps_c3.log 2>&1 || exit $?
grep -E "kernel A avg|crowded rejection|end pass|spawn waves" $O/${T}_stamps_c3.log
fi
