mkdir -p gpurun_out/r5u
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_rebalance.py tests/test_session_migration.py > gpurun_out/r5u/mig.log 2>&1
rc=$?; grep -E "capture\]|PASS|FAIL|Error" gpurun_out/r5u/mig.log | head -40; exit $rc
