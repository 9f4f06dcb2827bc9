set -o pipefail
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c3 > gpurun_out/stamps.log 2>&1 || exit $?
grep -E "kernel A|total median|rng work|policy|visib|resets|spawn waves|crowded" gpurun_out/stamps.log
