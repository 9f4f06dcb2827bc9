#!/bin/bash
# HBM traffic of the fused GRU step (probe binary, B = 20,480, H = 256): FETCH_SIZE and WRITE_SIZE passes.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_gf_bytes
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o fetch --output-format csv -- $R/tools/bin/gf_base 20480 256 20 > $OUT/fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o write --output-format csv -- $R/tools/bin/gf_base 20480 256 20 > $OUT/write.log 2>&1
echo done
