set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload c4 > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"]); print(d["roofline"]); print(d["whole_update_roofline"])'
