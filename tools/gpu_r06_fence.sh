# round 6: pending-slot fences off -- the spawn / parking / repeatability tests, then A/B/n against the fenced
# library on C3, C5 and C2 steady
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -p no:cacheprovider tests/test_gpu_parity.py tests/test_envs.py -k "parking or every_env or free_running or first_launches or step_seq or ragged or teacher_forced" -v --timeout 400 --timeout-method thread > $O/m_fence_tests.log 2>&1; rc=$?; grep -E "passed|failed" $O/m_fence_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
V="crowdnav_dsrnn_amd/lib/variants/libcn_fence1.so"
bash tools/abn.sh 3 "tree $V" --workload c3 --steps 200 --warmup 100 --no-side || exit $?
bash tools/abn.sh 3 "tree $V" --workload c5 --steps 200 --warmup 100 --no-side || exit $?
bash tools/abn.sh 3 "tree $V" --workload c2 --steps 2000 --warmup 100 --no-side --no-steady
