# H.264 headline: two frames in flight per session and more hardware queues, interleaved A/B
mkdir -p gpurun_out/r5s
B="--gpus 1 --steps 20 --warmup 5 --e2e-sessions 0 --extra-4k 0 --e2e-av1 none"
for rep in 1 2 3; do
  for v in base if2 q8 if2q8; do
    case $v in
      base) E="";; if2) E="SK_CAPTURE_INFLIGHT=2";; q8) E="GPU_MAX_HW_QUEUES=8";; if2q8) E="SK_CAPTURE_INFLIGHT=2 GPU_MAX_HW_QUEUES=8";;
    esac
    env $E timeout -k 10 200 python -u bench.py $B > gpurun_out/r5s/${v}_$rep.json 2> gpurun_out/r5s/${v}_$rep.err || { echo "$v $rep failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r5s/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', $rep, d['value'], d['p50_encode_latency_ms'], d['p99_encode_latency_ms'], d['config']['frames_in_flight'])"
  done
done
A="--encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0"
bash tools/gpu_steps.sh \
 "tests r5s_tests tests/test_av1_gpu.py" \
 "prof r5s_av1prof $A" \
 "py r5s_rd1080 tools/rd_codecs.py --backend hip --width 1920 --height 1080 --frames 20 --content motion,desktop --json gpurun_out/r5s_rd1080/rd.json" \
 "profpy r5s_av1key tools/key_latency.py --codec av1 --frames 24"
