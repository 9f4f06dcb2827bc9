# round 6: run-to-run determinism of the pending-slot handshake (tools/probe_c3_diverge2.py): runs that depart
# from run 0 of the same reset and actions, C3 (kd-tree path) and C2 (quad path) at two spawn budgets each
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
T=${1:-o}
timeout -k 10 900 python -u -m pytest -p no:cacheprovider tests/test_gpu_parity.py tests/test_envs.py -k "parking or every_env or free_running or first_launches or step_seq or ragged" -v --timeout 400 --timeout-method thread > $O/${T}_det_tests.log 2>&1; rc=$?; grep -E "passed|failed" $O/${T}_det_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
for cfg in "150 400 10 600000 c3" "100 400 10 300000 c3" "100 600 20 70000 c2" "100 600 20 20000 c2"; do
  set -- $cfg
  f=$O/${T}_div_$5_$4.log
  timeout -k 10 600 python -u tools/probe_c3_diverge2.py $cfg > $f 2>&1 || exit $?
  echo "$cfg: $(grep -c '== run 0' $f) equal, $(grep -c departs $f) departed"
done
