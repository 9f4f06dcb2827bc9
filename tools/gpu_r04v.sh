# round 4 v: sequence-GRU probe + GRU tests (+ optional C4 line)
set -o pipefail
O=gpurun_out/r04
T=${1:-v}
mkdir -p $O
timeout -k 10 300 python -u tools/probe_gru_seq.py > $O/${T}_probe.log 2>&1; rc=$?; cat $O/${T}_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_policy.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gru" > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/${T}_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
if [ "$2" = "c4" ]; then
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 6 > $O/${T}_bench_c4.log 2>&1 || exit $?
python -c "
import json
l=[x for x in open('$O/${T}_bench_c4.log') if x.startswith('{')][-1]; d=json.loads(l)
print('C4 %.1fk env-steps/s, %.1f ms/update, rollout %.4f s, ppo %.4f s, fused %.1f us, whole-update frac %.3f' % (d['value']/1e3, d['ms_per_step'], d['config']['rollout_s_per_update'], d['config']['ppo_s_per_update'], d['roofline']['avg_launch_us'], d['whole_update_roofline']['frac']))"
fi
