# diagnostic library with in-kernel s_memtime stamps (tools/probe_stamps.py), same flags as build.py
R=$(cd "$(dirname "$0")/.." && pwd)
H=$(cd $R && python -c 'from crowdnav_dsrnn_amd import build; print(build.source_hash())')
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -mllvm -disable-machine-licm -DCN_STAMPS \
  -DCN_SRC_HASH=\"$H\" -o $R/crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so $R/crowdnav_dsrnn_amd/csrc/cn_engine.hip $R/crowdnav_dsrnn_amd/csrc/cn_gru.hip
