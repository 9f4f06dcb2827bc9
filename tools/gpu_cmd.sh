set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_orca_known_answers.py tests/test_gpu_parity.py tests/test_policy_factory.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh 3
bash tools/ab.sh 2 --workload c3 --steps 300 --warmup 30
