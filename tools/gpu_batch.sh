set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_learner.py tests/test_evaluation.py -m gpu -v -s --timeout 150 --timeout-method thread > gpurun_out/gpu_new.log 2>&1; rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/gpu_new.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
