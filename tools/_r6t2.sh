# move tests with the capture-thread stall bound
bash tools/gpu.sh tests r6t2 tests/test_rebalance.py || exit $?
