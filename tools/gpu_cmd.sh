set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
bash tools/abn.sh 2 "tools/bin/libcn_base.so tree" || exit $?
bash tools/abn.sh 2 "tools/bin/libcn_base.so tree" --steps 20 --warmup 5 || exit $?
bash tools/abn.sh 1 "tools/bin/libcn_base.so tree" --workload c3 --steps 300 --warmup 30 || exit $?
