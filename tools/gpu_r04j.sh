# round 4 j: env-kernel change check + C3 variants + C3 stamps (default / no goal changes)
set -o pipefail
T=${1:-j}
bash tools/gpu_r04e.sh $T || exit $?
timeout -k 10 300 python -u tools/probe_c3_variants.py > gpurun_out/r04/${T}_c3_variants.log 2>&1 || exit $?
cat gpurun_out/r04/${T}_c3_variants.log
for v in c3 c3nogoal; do
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py $v > gpurun_out/r04/${T}_stamps_$v.log 2>&1 || exit $?
grep -E "kernel A|total median|visib|policy|rng work|wave0|step  start|slowest|end pass|random pass" gpurun_out/r04/${T}_stamps_$v.log
done
