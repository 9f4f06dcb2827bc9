# A/B/n: bench.py with each library in turn (CN_LIB_PATH; "tree" = the in-tree library), R rounds
#   bash tools/abn.sh <rounds> "<lib1> <lib2> ..." [bench args...]
set -o pipefail
mkdir -p gpurun_out
R=$1; LIBS=$2; shift 2
for k in $(seq 1 $R); do
  for L in $LIBS; do
    tag=$(basename $L .so)
    if [ "$L" = tree ]; then env_lib=""; else env_lib="CN_LIB_PATH=$L"; fi
    env $env_lib timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/abn_${tag}_$k.log 2>&1 || exit $?
    echo "$tag $(tail -1 gpurun_out/abn_${tag}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
