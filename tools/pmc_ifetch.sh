# one PMC pass: instruction-cache traffic of the C2 step kernel (SQC -> L2 instruction requests, I$ misses)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/prof_ifetch
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_TC_INST_REQ SQC_ICACHE_MISSES -T -d $R/gpurun_out/prof_ifetch/if -o if --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $R/gpurun_out/prof_ifetch/bench.log 2>&1 || exit $?
echo done
