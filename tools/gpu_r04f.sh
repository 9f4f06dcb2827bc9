# round 4 f: env-kernel change check (parity suite, C3 / C2 / C5 lines) + C3 stamps
set -o pipefail
T=${1:-f}
bash tools/gpu_r04e.sh $T || exit $?
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c3 > gpurun_out/r04/${T}_stamps_c3.log 2>&1 || exit $?
grep -E "kernel A|total median|visib|policy|rng work|wave0|kd walk|grid|step  start|spawn start" gpurun_out/r04/${T}_stamps_c3.log
