# A/B of C2 library variants, alternating: [BENCH_ARGS=...] bash tools/ab_c2.sh OUTDIR lib1.so lib2.so ...
set -o pipefail
O=$1; shift
mkdir -p $O
for r in 1 2; do for L in "$@"; do
  n=$(basename $L .so)
  CN_LIB_PATH=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-side $BENCH_ARGS > $O/${n}_$r.log 2>&1 || exit $?
  echo "$n: $(python tools/line_summary.py $O/${n}_$r.log | head -2 | tr '\n' ' ')"
done; done
