# round 4 final: full -m gpu suite, smoke, the driver's line (with its CPU baseline), C3 / C5 / C4 lines
set -o pipefail
O=gpurun_out/r04
T=${1:-f}
mkdir -p $O
CN_RESULTS_DIR=gpurun_out timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" $O/${T}_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
tail -1 $O/${T}_smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_bench_driver.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_c3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_c5.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 6 > $O/${T}_bench_c4.log 2>&1 || exit $?
for w in driver c3 c5; do python -c "
import json
l=[x for x in open('$O/${T}_bench_$w.log') if x.startswith('{')][-1]; d=json.loads(l); s=d.get('steady_state',{})
print('$w', 'window %.2fM (%.2f us kernel)' % (d['value']/1e6, d['config']['step_kernel_ms']*1e3), 'steady %.2fM (%.2f us kernel, resets %s)' % (s.get('value',0)/1e6, s.get('step_kernel_ms',0)*1e3, s.get('resets')))
" || exit $?; done
python -c "
import json
l=[x for x in open('$O/${T}_bench_c4.log') if x.startswith('{')][-1]; d=json.loads(l)
print('C4 %.1fk env-steps/s, %.1f ms/update, rollout %.4f s, ppo %.4f s, fused %.1f us (%.1f TF), whole-update frac %.3f' % (d['value']/1e3, d['ms_per_step'], d['config']['rollout_s_per_update'], d['config']['ppo_s_per_update'], d['roofline']['avg_launch_us'], d['roofline']['achieved'], d['whole_update_roofline']['frac']))"
