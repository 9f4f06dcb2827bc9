mkdir -p gpurun_out/r06
timeout -k 10 700 python -u _prefix/run.py > gpurun_out/r06/a_prefix_race.log 2>&1
rc=$?
echo "prefix rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest -p no:cacheprovider tests/test_gpu_parity.py -k every_env -v --timeout 400 --timeout-method thread > gpurun_out/r06/a_fixed_race.log 2>&1
rc=$?
echo "fixed rc=$rc"
exit $rc
