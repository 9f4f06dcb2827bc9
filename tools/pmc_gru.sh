# SQ counters of the GRU sequence kernels at C4's edge-pair shape (tools/probe_gru_seq.py pair), one pass each
#   bash tools/pmc_gru.sh <tag> [library path, e.g. a variant under crowdnav_dsrnn_amd/lib/variants]
set -o pipefail
TAG=$1; LIB=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gru_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export CN_LIB_PATH=$R/$LIB
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $R/tools/probe_gru_seq.py pair > $OUT/kt.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/sq -o sq --output-format csv -- python3 $R/tools/probe_gru_seq.py pair > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum -d $OUT/tcc -o tcc --output-format csv -- python3 $R/tools/probe_gru_seq.py pair > $OUT/tcc.log 2>&1 || exit 1
echo done $TAG
