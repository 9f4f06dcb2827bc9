set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_learner.py -m gpu -k "graph or c4_shape" > gpurun_out/r05b/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05b/bench_graph1.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --launch host --no-side --no-cpu-baseline > gpurun_out/r05b/bench_host1.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-side --no-cpu-baseline > gpurun_out/r05b/bench_graph2.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --launch host --no-side --no-cpu-baseline > gpurun_out/r05b/bench_host2.log 2>&1 || exit 1
