# k_hevc_bins CUs per wave A/B (SK_HEVC_BINS_LPW), HEVC 4K CRF bench block
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hevc_gpu.py > gpurun_out/r5h_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r5h_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 64 32 16 8 64 16; do
  SK_HEVC_BINS_LPW=$v bash tools/gpu.sh prof r5h_l$v --encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
  echo "lpw $v $(grep -E 'k_hevc_bins ' gpurun_out/r5h_l$v/kernels.md | cut -d'|' -f2,4,6,8 | tr '\n' ' ') $(tail -1 gpurun_out/r5h_l$v/prof.log | grep -o '"value": [0-9.]*')"
done
