#!/bin/bash
# rocprofv3 collection for the bench workload (run on the GPU box via gpurun from the repo root):
#   bash profiles/run_profile.sh <tag>
# 1) kernel trace + stats (per-kernel average durations), 2) FETCH_SIZE pass, 3) WRITE_SIZE pass
# (separate --pmc passes: FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2 — MI355X_MICROARCH.md).
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 400 --warmup 40 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $OUT/kt -o kt --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o fetch --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o write --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_write.log 2>&1
python3 $R/profiles/summarize.py $OUT $TAG
