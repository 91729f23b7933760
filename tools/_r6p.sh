# HEVC parity with 5-CTB key-frame segments at 4K, HEVC 4K kernel table + PMC passes, bench extras
A="--encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0"
bash tools/gpu.sh tests r6p_t tests/test_hevc_gpu.py || exit $?
bash tools/gpu.sh prof r6p_p $A > /dev/null || exit $?
head -22 gpurun_out/r6p_p/kernels.md | cut -d'|' -f2-8
[ -n "$PMC" ] && { bash tools/gpu.sh pmc r6p_pmc $A > /dev/null || exit $?; }
[ -n "$PMC" ] && head -30 gpurun_out/r6p_pmc/pmc.md
bash tools/gpu.sh bench r6p_b --steps 20 --warmup 5 --e2e-sessions 0 --e2e-av1 none > /dev/null || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6p_b/bench.jsonl").read().strip().splitlines()[-1])
print(d["value"], d["p50_encode_latency_ms"])
for k in ("hevc_4k", "hevc_4k_cbr", "av1_4k", "hevc_8k", "av1_8k"):
    v = d.get(k, {})
    print(k, v.get("fps"), v.get("p50_encode_latency_ms"), v.get("p99_encode_latency_ms"), v.get("keyframe", {}).get("latency_ms"), v.get("kib_per_frame"), v.get("paced", {}).get("p99_encode_latency_ms"))
PY
