#!/bin/bash
# step-kernel time vs env count (C2 shape): is the kernel latency- or issue-bound?
for E in 256 512 1024 1536 2048 3072 4096 5120 6144 8192 16384; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --envs $E --steps 500 --warmup 100 > gpurun_out/sweep_$E.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$E.log').read().strip().splitlines()[-1]); print($E, d['config']['step_kernel_ms']*1e3, d['value'])"
done
