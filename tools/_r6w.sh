# k_pc_model chain-segment length A/B (SK_HEVC_PC_SEG) at 4K, then the 8K extras
for seg in 32 64 128; do
  export SK_HEVC_PC_SEG=$seg
  bash tools/gpu.sh prof r6w_$seg --encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 30 --warmup 6 --pool 8 \
      --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0 > /dev/null || exit $?
  echo "seg $seg"; grep -E "k_pc_model|k_pc_rmap " gpurun_out/r6w_$seg/kernels.md | cut -d'|' -f2-8
done
unset SK_HEVC_PC_SEG
bash tools/_r6v.sh
