# round 6: norm-zone predicate tests + the parity suite's C5 / mixed tests, then A/B of the in-tree library
# against the previous commit's (tools/build_rev_variant.sh HEAD head) on C5, C2 steady and C3
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -p no:cacheprovider tests/test_norm_zone.py tests/test_mixed.py tests/test_gpu_parity.py -k "norm or mixed or c5 or social" -v --timeout 300 --timeout-method thread > $O/b_nz_tests.log 2>&1; rc=$?; grep -E "passed|failed" $O/b_nz_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
bash tools/abn.sh 2 "tree crowdnav_dsrnn_amd/lib/variants/libcn_head.so" --workload c5 --steps 200 --warmup 100 --no-side || exit $?
bash tools/abn.sh 2 "tree crowdnav_dsrnn_amd/lib/variants/libcn_head.so" --workload c2 --steps 2000 --warmup 100 --no-side || exit $?
bash tools/abn.sh 1 "tree crowdnav_dsrnn_amd/lib/variants/libcn_head.so" --workload c3 --steps 200 --warmup 100 --no-side
