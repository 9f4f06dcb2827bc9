# A/B of the in-tree library against tools/bin/libcn_base.so on one workload, alternating runs
#   bash tools/ab.sh <runs> [bench args...]
set -o pipefail
mkdir -p gpurun_out
R=${1:-3}; shift
for k in $(seq 1 $R); do
CN_LIB_PATH=tools/bin/libcn_base.so timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_base_$k.log 2>&1 || exit $?
echo "base $(tail -1 gpurun_out/ab_base_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_new_$k.log 2>&1 || exit $?
echo "new  $(tail -1 gpurun_out/ab_new_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
