set -o pipefail
mkdir -p gpurun_out
bash tools/abn.sh 5 "tools/bin/libcn_base.so tree" --steps 20 --warmup 5 || exit $?
