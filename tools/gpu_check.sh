#!/bin/bash
# GPU box check: parity tests, smoke, bench. Stops at the first GPU fault/abort/timeout
# (pytest exit 1 = test failures only, the later steps still run).
# usage: bash tools/gpu_check.sh [bench args...]
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench.log 2>&1 || exit $?
cat gpurun_out/bench.log | tail -1
exit $rc
