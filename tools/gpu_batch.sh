set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag_flips.py > gpurun_out/diag_flips.log 2>&1 || exit $?
cat gpurun_out/diag_flips.log
bash profiles/run_profile.sh r02_a
