#!/bin/bash
# SQ/SQC counter passes for the step kernel (diagnostic; separate --pmc passes, no trace domains):
#   bash profiles/run_sq.sh <tag>
set -e
TAG=${1:-sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 200 --warmup 20 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/p1 -o p1 --output-format csv -- python3 $R/bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VSKIPPED -d $OUT/p2 -o p2 --output-format csv -- python3 $R/bench.py $ARGS > $OUT/p2.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "cn_step" not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print("  %-28s per-launch mean %.4g  (%d launches)" % (c, sum(v) / len(v), len(v)))
PY
