set -o pipefail
mkdir -p gpurun_out
true
bash tools/ab.sh 2
bash tools/ab.sh 1 --workload c3 --steps 300 --warmup 30
bash tools/ab.sh 1 --workload c5
