# round 4 s: kernel trace of C4 updates (timeline: busy / idle per update, per-kernel totals)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -T -d $O/c4kt -o kt --output-format csv -- python3 $R/bench.py --workload c4 --no-cpu-baseline --steps 2 --warmup 2 > $O/s_c4kt.log 2>&1 || exit $?
echo traced
