# round 3: new GPU tests (kd ORCA predict, forced spawn parking, full-size C3), then a C2 kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_policy_factory.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "parking or full_size_c3" > gpurun_out/gpu_new.log 2>&1; rc=$?; echo new rc=$rc; grep -E "passed|failed|PASS|FAIL" gpurun_out/gpu_new.log | tail -8; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/kt_c2 -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 400 --warmup 40 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/kt_c2.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
f=$(ls gpurun_out/kt_c2/*/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(ls gpurun_out/kt_c2/*kernel_trace.csv | head -1)
python3 tools/launch_hist.py $f cn_step_kernel 20
