# HEVC 4x4 transforms through DPP (quad broadcasts / row rotates): parity, 4K key-frame profile, extras
bash tools/gpu.sh tests r6y_t tests/test_hevc_gpu.py tests/test_hevc_sao.py tests/test_hevc_subpel.py || exit $?
bash tools/gpu.sh profpy r6y_key tools/key_latency.py --codec hevc --width 3840 --height 2160 --frames 24 --period 4 > /dev/null || exit $?
grep -E "k_hevc_intra_seg|k_hevc_bins|k_hevc_intra_prep|k_hevc_inter " gpurun_out/r6y_key/kernels.md | cut -d'|' -f2-8; tail -2 gpurun_out/r6y_key/out.txt
bash tools/gpu.sh bench r6y_b --steps 20 --warmup 5 --e2e-sessions 0 --e2e-av1 none > /dev/null || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6y_b/bench.jsonl").read().strip().splitlines()[-1])
print(d["value"], d["p50_encode_latency_ms"])
for k in ("hevc_4k", "hevc_4k_cbr", "av1_4k", "hevc_8k", "hevc_8k_cbr", "av1_8k"):
    v = d.get(k, {})
    print(k, v.get("fps"), v.get("p50_encode_latency_ms"), v.get("p99_encode_latency_ms"), v.get("keyframe", {}).get("latency_ms"), v.get("kib_per_frame"), v.get("paced", {}).get("p99_encode_latency_ms"))
PY
