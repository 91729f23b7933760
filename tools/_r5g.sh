# k_code_inter occupancy A/B on the H.264 headline config (4 / 5 / 6 waves per SIMD)
for v in ci4 ci5 ci6 ci4 ci5 ci6; do
  SK_NATIVE_LIB=$PWD/tools/ab/libsk_$v.so bash tools/gpu.sh prof r5g_$v --steps 40 --warmup 5 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
  echo "$v $(grep -E 'k_code_inter ' gpurun_out/r5g_$v/kernels.md | cut -d'|' -f2,4,6 | tr '\n' ' ') $(tail -1 gpurun_out/r5g_$v/prof.log | grep -o '"value": [0-9.]*')"
done
for v in ci4 ci5 ci4 ci5; do
  SK_NATIVE_LIB=$PWD/tools/ab/libsk_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 2>/dev/null | tail -1 | grep -o '"value": [0-9.]*' | sed "s/^/$v bench /"
done
