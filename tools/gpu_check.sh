set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
