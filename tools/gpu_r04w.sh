# round 4 w: GRU kernel variants (tools/build_gru_variants.sh) timed by tools/probe_gru_seq.py
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
for v in "$@"; do
  echo "== $v"
  CN_LIB_PATH=crowdnav_dsrnn_amd/lib/variants/libcrowdnav_hip_$v.so timeout -k 10 120 python -u tools/probe_gru_seq.py > $O/w_$v.log 2>&1; rc=$?; grep -v amdgpu.ids $O/w_$v.log; [ $rc -eq 0 ] || exit $rc
done
