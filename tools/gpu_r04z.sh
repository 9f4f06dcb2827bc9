# round 4 z: GRU probe, policy / learner / lidar GPU tests, C4 line, C4 kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
T=${1:-z}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/probe_gru_seq.py > $O/${T}_probe.log 2>&1; rc=$?; grep -v amdgpu.ids $O/${T}_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_policy.py tests/test_learner.py tests/test_lidar.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/${T}_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 6 > $O/${T}_bench_c4.log 2>&1 || exit $?
python -c "
import json
l=[x for x in open('$O/${T}_bench_c4.log') if x.startswith('{')][-1]; d=json.loads(l)
print('C4 %.1fk env-steps/s, %.1f ms/update, rollout %.4f s, ppo %.4f s, fused %.1f us (%.1f TF), whole-update frac %.3f' % (d['value']/1e3, d['ms_per_step'], d['config']['rollout_s_per_update'], d['config']['ppo_s_per_update'], d['roofline']['avg_launch_us'], d['roofline']['achieved'], d['whole_update_roofline']['frac']))" || exit $?
if [ "$2" = "trace" ]; then
rm -rf $O/c4kt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -T -d $O/c4kt -o kt --output-format csv -- python3 $R/bench.py --workload c4 --no-cpu-baseline --steps 2 --warmup 2 > $O/${T}_c4kt.log 2>&1 || exit $?
echo traced
fi
