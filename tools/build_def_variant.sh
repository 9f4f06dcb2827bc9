# diagnostic: the engine library of the working tree with extra defines, for A/B runs through CN_LIB_PATH
#   bash tools/build_def_variant.sh <name> "<-Dflags...>"   -> crowdnav_dsrnn_amd/lib/variants/libcn_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
V=$R/crowdnav_dsrnn_amd/lib/variants
T=$(mktemp -d /tmp/cndef.XXXXXX)
mkdir -p $V
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -DCN_SRC_HASH=\"def-$1\" $2"
hipcc $F -mllvm -disable-machine-licm -c -o $T/e.o $R/crowdnav_dsrnn_amd/csrc/cn_engine.hip &
hipcc $F -c -o $T/g.o $R/crowdnav_dsrnn_amd/csrc/cn_gru.hip
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o $V/libcn_$1.so $T/e.o $T/g.o
rm -rf $T
echo $V/libcn_$1.so
