# diagnostic: the engine library as of a git revision, for A/B runs through CN_LIB_PATH (tools/ab_c2.sh, abn.sh)
#   bash tools/build_rev_variant.sh <rev> <name>   -> crowdnav_dsrnn_amd/lib/variants/libcn_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
V=$R/crowdnav_dsrnn_amd/lib/variants
T=$(mktemp -d /tmp/cnrev.XXXXXX)
mkdir -p $V $T/crowdnav_dsrnn_amd/csrc $T/include
for f in crowdnav_dsrnn_amd/csrc/cn_engine.hip crowdnav_dsrnn_amd/csrc/cn_gru.hip crowdnav_dsrnn_amd/csrc/cn_math.h \
         include/crowdnav.h include/crowdnav_state.h; do
  git -C $R show $1:$f > $T/$f
done
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -DCN_SRC_HASH=\"rev-$1\""
hipcc $F -mllvm -disable-machine-licm -c -o $T/e.o $T/crowdnav_dsrnn_amd/csrc/cn_engine.hip &
hipcc $F -c -o $T/g.o $T/crowdnav_dsrnn_amd/csrc/cn_gru.hip
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o $V/libcn_$2.so $T/e.o $T/g.o
rm -rf $T
echo $V/libcn_$2.so
