# diagnostic: libraries with cn_gru.hip compile-time variants (tools/probe_gru_seq.py via CN_LIB_PATH)
#   bash tools/build_gru_variants.sh name "-DGF_WPC=3 ..." [name "-D..."] ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
V=$R/crowdnav_dsrnn_amd/lib/variants
mkdir -p $V
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result"
[ -f $V/engine.o ] || hipcc $F -mllvm -disable-machine-licm -c -o $V/engine.o $R/crowdnav_dsrnn_amd/csrc/cn_engine.hip
while [ $# -ge 2 ]; do
  n=$1; d=$2; shift 2
  hipcc $F $d -c -o $V/gru_$n.o $R/crowdnav_dsrnn_amd/csrc/cn_gru.hip -Rpass-analysis=kernel-resource-usage 2>&1 \
    | grep -A12 "fused_kernel" | grep -E " VGPRs:|VGPRs Spill" | sed "s/.*remark: *//" | tr '\n' ' '; echo " <- $n"
  hipcc --offload-arch=gfx950 -shared -fPIC -o $V/libcrowdnav_hip_$n.so $V/engine.o $V/gru_$n.o
  rm -f $V/gru_$n.o
done
