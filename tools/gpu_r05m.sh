# round 5: keyed spawn lists -- C3 determinism with parking on (150 runs), GPU suite
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 500 python -u tools/probe_c3_diverge2.py 150 400 10 600000 > $O/div150_park_keyed.log 2>&1 || exit $?
grep departs $O/div150_park_keyed.log | head -3; grep -c "== run 0" $O/div150_park_keyed.log
CN_SPAWN_BUDGET=600000 timeout -k 10 120 python -u tools/probe_c3_variants.py default > $O/c3_park.log 2>&1 || exit $?
CN_SPAWN_BUDGET=0 timeout -k 10 120 python -u tools/probe_c3_variants.py default > $O/c3_nopark.log 2>&1 || exit $?
grep "per launch" $O/c3_park.log $O/c3_nopark.log
CN_RESULTS_DIR=gpurun_out timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
