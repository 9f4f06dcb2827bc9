# round 6: A/B/n of variant libraries against the in-tree one on C2 (steady 2000 launches, then the driver's window)
#   bash tools/gpu_r06_ab.sh <rounds> "<lib...>"
set -o pipefail
bash tools/abn.sh $1 "tree $2" --workload c2 --steps 2000 --warmup 100 --no-side --no-steady || exit $?
bash tools/abn.sh $1 "tree $2" --workload c2 --steps 20 --warmup 5 --no-side --no-steady
