# round 6: stamps probes (phase breakdown, grid timeline) of the in-tree sources (tools/build_stamps.sh first)
#   bash tools/gpu_r06_stamps.sh <tag> <variant...>
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
T=$1; shift
for v in "$@"; do
  CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py $v > $O/${T}_stamps_$v.log 2>&1 || exit $?
  grep -v amdgpu $O/${T}_stamps_$v.log | head -60
done
