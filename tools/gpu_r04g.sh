# round 4 g: attention probe, policy / learner GPU tests, C4 line
set -o pipefail
O=gpurun_out/r04
T=${1:-g}
mkdir -p $O
timeout -k 10 120 python -u tools/probe_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 900 python -u -m pytest tests/test_policy.py tests/test_learner.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/${T}_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 6 > $O/${T}_bench_c4.log 2>&1 || exit $?
python -c "
import json
l=[x for x in open('$O/${T}_bench_c4.log') if x.startswith('{')][-1]; d=json.loads(l)
print('C4 %.1fk env-steps/s, %.1f ms/update, rollout %.4f s, ppo %.4f s, fused %.1f us (%.1f TF), whole-update frac %.3f' % (d['value']/1e3, d['ms_per_step'], d['config']['rollout_s_per_update'], d['config']['ppo_s_per_update'], d['roofline']['avg_launch_us'], d['roofline']['achieved'], d['whole_update_roofline']['frac']))"
