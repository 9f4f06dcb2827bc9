#!/bin/bash
# One SQ counter pass over the fused GRU step probes (tools/gru_fused_probe.hip builds in tools/bin/).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_gf
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in base noepi; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -T -d $OUT/$v -o sq --output-format csv -- $R/tools/bin/gf_$v 20480 256 20 > $OUT/$v.log 2>&1
done
echo done
