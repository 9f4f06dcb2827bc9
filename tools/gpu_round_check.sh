# Round-end check of HEAD's library on one GPU (run from the repo root via gpurun):
#   bash tools/gpu_round_check.sh <tag>
# GPU suite, smoke, C2 (default + driver-style window), C3, C5, C4 benches, then the rocprofv3 passes of
# profiles/run_profile.sh; every step under its own time limit, stopping at the first failure.
set -o pipefail
T=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c3 > gpurun_out/${T}_bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 > gpurun_out/${T}_bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c4 > gpurun_out/${T}_bench_c4.log 2>&1 || exit 1
bash profiles/run_profile.sh ${T} > gpurun_out/${T}_profile.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver_style.log 2>&1 || exit 1
