#!/bin/bash
# rocprofv3 collection for a bench workload (run on the GPU box via gpurun from the repo root):
#   bash profiles/run_profile.sh <tag> [bench.py args...]
# Default args = the driver's own invocation (bench.py --gpus 1 --steps 20 --warmup 5), whose line carries
# the main window (launches 6-25 after cn_reset) and the steady_state window (launches 126-2125);
# summarize.py splits every figure by those windows. The counter passes add --no-cpu-baseline (the CPU leg
# runs after all GPU work and launches nothing), the kernel-trace pass runs the command unchanged.
# Passes (each its own run, no trace domain beside --pmc; MI355X_MICROARCH.md § rocprofv3 PMC slots):
#   kt     --kernel-trace --stats (per-kernel average durations)
#   fetch  --pmc FETCH_SIZE   (3 TCC slots)
#   write  --pmc WRITE_SIZE   (2 TCC slots)
#   sq1    8 SQ counters (instruction mix, wave cycles, waits) + GRBM_GUI_ACTIVE
#   sq2    8 SQ counters (f64 / transcendental / branch detail)
#   tcc    L2 hit / miss and the fabric's DRAM read / write requests
# Output under gpurun_out/prof_<tag>/ (merged back by gpurun); summarise on the CPU side with
#   python profiles/summarize.py gpurun_out/prof_<tag> <tag>
set -e
TAG=${1:-r02}
shift || true
ARGS="${*:---gpus 1 --steps 20 --warmup 5}"
PARGS="$ARGS --no-cpu-baseline"
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, '$R'); from crowdnav_dsrnn_amd import _lib; print(_lib.lib().cn_version().decode())" > $OUT/lib_version.txt
echo "$ARGS" > $OUT/bench_args.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt -o kt --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o fetch --output-format csv -- python3 $R/bench.py $PARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o write --output-format csv -- python3 $R/bench.py $PARGS > $OUT/bench_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -T -d $OUT/sq1 -o sq1 --output-format csv -- python3 $R/bench.py $PARGS > $OUT/bench_sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SMEM SQ_INSTS_VSKIPPED -T -d $OUT/sq2 -o sq2 --output-format csv -- python3 $R/bench.py $PARGS > $OUT/bench_sq2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum -T -d $OUT/tcc -o tcc --output-format csv -- python3 $R/bench.py $PARGS > $OUT/bench_tcc.log 2>&1
# calibration of FETCH_SIZE / WRITE_SIZE on this kernel's 8-B-per-lane access shape (tools/calib_pmc.py)
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/calfetch -o calfetch --output-format csv -- python3 $R/tools/calib_pmc.py > $OUT/calib_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/calwrite -o calwrite --output-format csv -- python3 $R/tools/calib_pmc.py > $OUT/calib_write.log 2>&1
echo profile $TAG done
