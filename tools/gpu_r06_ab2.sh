# round 6: parity subset, then A/B/n of the in-tree library against a variant on C2 steady, the C2 window, C3, C5
#   bash tools/gpu_r06_ab2.sh <rounds> <variant.so>
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -p no:cacheprovider tests/test_gpu_parity.py tests/test_envs.py tests/test_mixed.py -k "teacher_forced or every_env or free_running or first_launches or runs_repeat or vecenv or mixed or parking" -v --timeout 400 --timeout-method thread > $O/ab2_tests.log 2>&1; rc=$?; grep -E "passed|failed" $O/ab2_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
bash tools/abn.sh $1 "tree $2" --workload c2 --steps 2000 --warmup 100 --no-side --no-steady || exit $?
bash tools/abn.sh $1 "tree $2" --workload c2 --steps 20 --warmup 5 --no-side --no-steady || exit $?
bash tools/abn.sh $1 "tree $2" --workload c5 --steps 200 --warmup 100 --no-side || exit $?
bash tools/abn.sh $1 "tree $2" --workload c3 --steps 200 --warmup 100 --no-side
