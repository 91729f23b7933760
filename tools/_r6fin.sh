# final tree: full GPU tier + smoke()
bash tools/gpu.sh tests r6fin_tier || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6fin_tier/smoke.log 2>&1 || { tail -20 gpurun_out/r6fin_tier/smoke.log; exit 1; }
tail -3 gpurun_out/r6fin_tier/smoke.log
