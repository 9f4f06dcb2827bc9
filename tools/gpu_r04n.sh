# round 4 n: env-kernel change check (parity suite, C3 / C2 / C5 lines) + hash-matched profile of the
# driver's invocation (per-window traffic)
set -o pipefail
T=${1:-n}
bash tools/gpu_r04e.sh $T || exit $?
bash profiles/run_profile.sh r04_$T > gpurun_out/r04/${T}_prof.log 2>&1 || exit $?
echo profile done
