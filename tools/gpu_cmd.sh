set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
L="tools/bin/libcn_base.so tree tools/bin/libcn_w2.so tools/bin/libcn_w3.so tools/bin/libcn_w4.so"
bash tools/abn.sh 2 "$L" --steps 20 --warmup 5 || exit $?
bash tools/abn.sh 1 "$L" || exit $?
