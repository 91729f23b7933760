# AV1 GPU tests on the in-tree build (k_av1_inter and k_av1_tokens at 3 waves/SIMD), then k_av1_tokens at 4
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_av1_gpu.py tests/test_av1_entropy.py > gpurun_out/r5ab_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r5ab_tests.log; [ $rc -eq 0 ] || exit $rc
for v in w3t3 w3t4 w3t3 w3t4; do
  SK_NATIVE_LIB=$PWD/tools/ab/libsk_$v.so bash tools/gpu.sh prof r5ab_$v --encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
  echo "$v $(grep -E 'k_av1_inter |k_av1_tokens ' gpurun_out/r5ab_$v/kernels.md | cut -d'|' -f2,4,6 | tr '\n' ' ') $(tail -1 gpurun_out/r5ab_$v/prof.log | grep -o '"value": [0-9.]*')"
done
