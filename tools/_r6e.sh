# parity (H.264 auto deblock, HEVC 4x4 serial binarisation, AV1 qp floor), HEVC 4K key-frame
# kernel profile, then the headline with automatic deblocking (its cost at CRF 25)
bash tools/gpu.sh tests r6e2_t tests/test_h264_gpu.py tests/test_hevc_gpu.py tests/test_ratecontrol.py || exit $?
bash tools/gpu.sh profpy r6e2_key tools/key_latency.py --codec hevc --width 3840 --height 2160 --frames 24 --period 4 > /dev/null || exit $?
head -24 gpurun_out/r6e2_key/kernels.md | cut -d'|' -f2-8; tail -4 gpurun_out/r6e2_key/out.txt
bash tools/gpu.sh bench r6e2_b --steps 20 --warmup 5 --e2e-sessions 0 --e2e-av1 none --extra-4k 1 --extra-8k 0 > /dev/null || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6e2_b/bench.jsonl").read().strip().splitlines()[-1])
print(d["value"], d["p50_encode_latency_ms"], d["config"].get("deblock"))
for k in ("hevc_4k", "hevc_4k_cbr", "av1_4k"):
    v = d.get(k, {})
    print(k, v.get("fps"), v.get("p50_encode_latency_ms"), v.get("p99_encode_latency_ms"), v.get("keyframe", {}).get("latency_ms"), v.get("kib_per_frame"), v.get("paced", {}).get("p99_encode_latency_ms"))
PY
