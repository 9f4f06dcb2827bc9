set -o pipefail
mkdir -p gpurun_out
bash tools/abn.sh 2 "tools/bin/libcn_base.so tree tools/bin/libcn_d.so"
bash tools/abn.sh 1 "tools/bin/libcn_base.so tree" --workload c3 --steps 300 --warmup 30
