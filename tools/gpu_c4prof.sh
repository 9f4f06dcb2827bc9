# GPU: C4 bench line (+ MFMA roofline), rocprofv3 kernel trace of a short C4 run, then the C2 profile passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c4 > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | cut -c1-300
R=$(pwd)
mkdir -p gpurun_out/prof_c4
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/prof_c4/kt -o kt --output-format csv -- python3 $R/bench.py --workload c4 --steps 2 --warmup 1 > $R/gpurun_out/prof_c4/bench.log 2>&1 ) || exit $?
echo c4 trace done
timeout -k 10 1000 bash profiles/run_profile.sh ${1:-r02_i} || exit $?
