# round 6: A/B/n of the in-tree library against the round-5 fenced handshake (libcn_fence1) on C3, C5, C2 steady
set -o pipefail
V="crowdnav_dsrnn_amd/lib/variants/libcn_fence1.so"
bash tools/abn.sh $1 "tree $V" --workload c3 --steps 200 --warmup 100 --no-side || exit $?
bash tools/abn.sh $1 "tree $V" --workload c5 --steps 200 --warmup 100 --no-side || exit $?
bash tools/abn.sh $1 "tree $V" --workload c2 --steps 2000 --warmup 100 --no-side --no-steady
