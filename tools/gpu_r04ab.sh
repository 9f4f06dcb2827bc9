# round 4 ab: C2 line (window + steady) of the main library vs variant libraries, alternating
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
for rep in 1 2; do
  for v in main "$@"; do
    if [ "$v" = main ]; then L=""; else L=crowdnav_dsrnn_amd/lib/variants/libcrowdnav_hip_$v.so; fi
    CN_LIB_PATH=$L timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/ab_${v}_$rep.log 2>&1 || exit $?
    python -c "
import json
l=[x for x in open('$O/ab_${v}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l); s=d['steady_state']
print('%-8s rep $rep: window %.2fM (%.2f us kernel, %.2f us/step)  steady %.2fM (%.2f us kernel)' % ('$v', d['value']/1e6, d['config']['step_kernel_ms']*1e3, d['ms_per_step']*1e3, s['value']/1e6, s['step_kernel_ms']*1e3))" || exit $?
  done
done
