# round 4 b: C3 diagnostics (phase stamps, SQ counters of the C3 step kernel) + C2 driver-style line after the
# host-overhead trim of CrowdNavEngine.step
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b_bench_driver.log 2>&1 || exit $?
tail -1 $O/b_bench_driver.log | cut -c1-400
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c3 > $O/b_stamps_c3.log 2>&1 || exit $?
cat $O/b_stamps_c3.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/$O/c3kt -o kt --output-format csv -- python3 $R/bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/b_c3_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -T -d $R/$O/c3sq1 -o sq1 --output-format csv -- python3 $R/bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/b_c3_sq1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SMEM SQ_INSTS_VSKIPPED -T -d $R/$O/c3sq2 -o sq2 --output-format csv -- python3 $R/bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/b_c3_sq2.log 2>&1 || exit $?
echo all done
