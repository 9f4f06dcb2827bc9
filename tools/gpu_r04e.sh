# round 4 e: env-kernel change check: GPU parity suite (env), C3 / C2 / C5 lines
set -o pipefail
O=gpurun_out/r04
T=${1:-e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_policy_factory.py tests/test_mixed.py tests/test_orca_known_answers.py tests/test_envs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_c3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_c5.log 2>&1 || exit $?
for w in c3 c2 c5; do python -c "
import json,sys
l=[x for x in open('$O/${T}_bench_$w.log') if x.startswith('{')][-1]; d=json.loads(l); s=d.get('steady_state',{})
print('$w', 'window %.2fM (%.2f us kernel)' % (d['value']/1e6, d['config']['step_kernel_ms']*1e3), 'steady %.2fM (%.2f us kernel, resets %s)' % (s.get('value',0)/1e6, s.get('step_kernel_ms',0)*1e3, s.get('resets')))
"; done
