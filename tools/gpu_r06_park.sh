# round 6: quad-path spawn parking -- its tests, then A/B/n against variants on C2 (steady, then the window)
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -p no:cacheprovider tests/test_gpu_parity.py tests/test_envs.py -k "parking or every_env or free_running or first_launches or step_seq or vecenv or ragged" -v --timeout 400 --timeout-method thread > $O/h_park_tests.log 2>&1; rc=$?; grep -E "passed|failed" $O/h_park_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r06_ab.sh 2 "$1"
