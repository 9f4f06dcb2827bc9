# round-3 GPU call: full -m gpu suite, smoke, C2 bench, C2 stamps (diagnostic lib), C3 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-400
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c2 > gpurun_out/stamps.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c3.log | cut -c1-300
