# e2e knee attribution: 56 and 64 sessions (8 per server process, x264enc) with CPU sampling
mkdir -p gpurun_out/r6s
timeout -k 10 400 python -u tools/bench_e2e.py --sweep 56,64 --encoder x264enc --sessions-per-proc 8 --client-procs 8 \
    --sample-cpu --log-dir gpurun_out/r6s/logs > gpurun_out/r6s/out.txt 2>&1 || { tail -20 gpurun_out/r6s/out.txt; exit 1; }
tail -60 gpurun_out/r6s/out.txt | cut -c1-2000
