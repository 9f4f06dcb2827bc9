set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_orca_known_answers.py tests/test_gpu_parity.py tests/test_policy_factory.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh 2 --workload c3 --steps 300 --warmup 30
CN_LIB_PATH=tools/bin/libcn_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c2 > gpurun_out/stamps.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/prof_c4_ops.py > gpurun_out/c4_ops.log 2>&1 || exit $?
