# stamps of the step kernel from the -DCN_STAMPS build (tools/bin/libcn_stamps.so, built beforehand)
set -o pipefail
mkdir -p gpurun_out
CN_LIB_PATH=tools/bin/libcn_stamps.so timeout -k 10 300 python -u tools/probe_stamps.py ${STAMP_VARIANTS:-c2} > gpurun_out/stamps.log 2>&1 || exit $?
echo done
