# C4 bench repeated (run-to-run spread of the update time)
set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 10 > gpurun_out/rep_c4_$k.log 2>&1 || exit $?
  tail -1 gpurun_out/rep_c4_$k.log | cut -c1-200
done
