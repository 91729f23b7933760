# HEVC GPU tests on the in-tree build, then k_hevc_bins A/B: packed 64-bit bin stores vs 16-bit
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hevc_gpu.py tests/test_ratecontrol.py > gpurun_out/r5h_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r5h_tests.log; [ $rc -eq 0 ] || exit $rc
for v in binref binpk binref binpk; do
  SK_NATIVE_LIB=$PWD/tools/ab/libsk_$v.so bash tools/gpu.sh prof r5h_$v --encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
  echo "$v $(grep -E 'k_hevc_bins ' gpurun_out/r5h_$v/kernels.md | cut -d'|' -f2,4,6,8 | tr '\n' ' ')"
done
