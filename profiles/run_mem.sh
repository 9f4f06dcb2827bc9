#!/bin/bash
# TCP/UTCL1 counter passes for the step kernel (diagnostic): bash profiles/run_mem.sh <tag>
set -e
TAG=${1:-mem}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/mem_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 200 --warmup 20 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_TRANSLATION_MISS -d $OUT/p1 -o p1 --output-format csv -- python3 $R/bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TCP_TCP_LATENCY TCP_TA_TCP_STATE_READ -d $OUT/p2 -o p2 --output-format csv -- python3 $R/bench.py $ARGS > $OUT/p2.log 2>&1
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
