# round 4 p: env-kernel change check (parity suite, C3 / C2 / C5 lines), C3 goal-change variants, and the
# hash-matched profile of the driver's invocation (per-window traffic)
set -o pipefail
T=${1:-p}
bash tools/gpu_r04e.sh $T || exit $?
timeout -k 10 300 python -u tools/probe_c3_variants.py > gpurun_out/r04/${T}_c3_variants.log 2>&1 || exit $?
cat gpurun_out/r04/${T}_c3_variants.log
bash profiles/run_profile.sh r04_$T > gpurun_out/r04/${T}_prof.log 2>&1 || exit $?
echo profile done
