# round 5: reset-key A/B (C2 steady + C3), C2 spawn counters, C3 driver-style window, driver line, C3 divergence catcher, C2 stamps
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
bash tools/ab_c2.sh $O/ab_c2 crowdnav_dsrnn_amd/lib/variants/libcn_head.so crowdnav_dsrnn_amd/lib/libcrowdnav_hip.so || exit $?
bash tools/ab_c3.sh $O/ab_c3.log crowdnav_dsrnn_amd/lib/variants/libcn_head.so crowdnav_dsrnn_amd/lib/libcrowdnav_hip.so || exit $?
timeout -k 10 120 python -u tools/probe_c2_inline.py > $O/c2_inline.log 2>&1 || exit $?
grep -v amdgpu $O/c2_inline.log
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_driver_style.log 2>&1 || exit $?
python tools/line_summary.py $O/c3_driver_style.log
timeout -k 10 400 python -u tools/probe_c3_diverge2.py 14 400 10 > $O/div2.log 2>&1 || exit $?
grep -v amdgpu $O/div2.log | tail -16
CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py c2w c2_301 > $O/stamps_c2.log 2>&1 || exit $?
grep -E "kernel A avg|total median|rng work|policy|slowest|resets \(|goal items" $O/stamps_c2.log
