timeout -k 10 1000 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/r5t_tier.log 2>&1
rc=$?; tail -3 gpurun_out/r5t_tier.log; grep -E "FAILED|state not carried" gpurun_out/r5t_tier.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu.sh driver r5t_driver
