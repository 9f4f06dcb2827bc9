# A/B of C3 library variants (tools/probe_c3_variants.py default, alternating): bash tools/ab_c3.sh OUT lib1.so lib2.so ...
set -o pipefail
OUT=$1; shift
mkdir -p $(dirname $OUT)
for r in 1 2; do for L in "$@"; do
  CN_LIB_PATH=$L timeout -k 10 120 python -u tools/probe_c3_variants.py default >> $OUT 2>&1 || exit $?
done; done
grep "per launch" $OUT
