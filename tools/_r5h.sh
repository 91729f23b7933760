# k_hevc_sao_stats occupancy A/B (5 = default / 6 / 8 waves per SIMD), HEVC 4K CRF
for v in ss5 ss6 ss8 ss5 ss6 ss8; do
  SK_NATIVE_LIB=$PWD/tools/ab/libsk_$v.so bash tools/gpu.sh prof r5h_$v --encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
  echo "$v $(grep -E 'k_hevc_sao_stats ' gpurun_out/r5h_$v/kernels.md | cut -d'|' -f2,4,6,8 | tr '\n' ' ')"
done
