set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/n_gputest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/n_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/n_bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c3 > gpurun_out/n_bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 > gpurun_out/n_bench_c5.log 2>&1 || exit 1
bash profiles/run_profile.sh r02_n > gpurun_out/n_profile.log 2>&1 || exit 1
