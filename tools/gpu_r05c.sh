set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_envs.py -m gpu -k "step_seq" > gpurun_out/r05c/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05c/bench_seq1.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --launch host --no-side --no-cpu-baseline > gpurun_out/r05c/bench_host1.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-side --no-cpu-baseline > gpurun_out/r05c/bench_seq2.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --launch host --no-side --no-cpu-baseline > gpurun_out/r05c/bench_host2.log 2>&1 || exit 1
