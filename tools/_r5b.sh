# A/B of the H.264 headline across round-3/4 commits: every tree runs the driver's bench
# configuration (no e2e / 4K extras), interleaved, three repetitions, one box.
ROOT=$(pwd); mkdir -p gpurun_out/r5b
for rep in 1 2 3; do
  for t in HEAD ab_9002773 ab_9b83cda ab_901ff5b ab_bb5e2b7 ab_aee4e20; do
    if [ $t = HEAD ]; then d=.; extra="--e2e-av1 none"; else d=$t; extra=""; fi
    ( cd $d && timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --e2e-sessions 0 --extra-4k 0 $extra \
        > $ROOT/gpurun_out/r5b/${t}_$rep.json 2> $ROOT/gpurun_out/r5b/${t}_$rep.err ) || { echo "$t rep $rep failed: $?"; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/r5b/${t}_$rep.json').read().strip().splitlines()[-1]); print('$t', $rep, d['value'], d['p50_encode_latency_ms'], d['p99_encode_latency_ms'])"
  done
done
bash tools/gpu.sh prof r5b_h264prof --gpus 1 --steps 20 --warmup 5 --e2e-sessions 0 --extra-4k 0 --e2e-av1 none
