# HEVC parity after the binariser rework, then the 4K CRF kernel table at 32 / 16 units per wave
A="--encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0"
bash tools/gpu.sh tests r6a_t tests/test_hevc_gpu.py || exit $?
bash tools/gpu.sh prof r6a_l32 $A > /dev/null || exit $?
SK_HEVC_BINS_LPW=16 bash tools/gpu.sh prof r6a_l16 $A > /dev/null || exit $?
for v in l32 l16; do
  echo "$v $(grep -E 'k_hevc_bins ' gpurun_out/r6a_$v/kernels.md | cut -d'|' -f2,4,6,7,8 | tr '\n' ' ')"
  tail -1 gpurun_out/r6a_$v/prof.log | cut -c1-400
done
