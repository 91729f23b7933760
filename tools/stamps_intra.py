"""Diagnostic: per-segment cycle shares of the H.264 intra wavefront kernel.

Needs the stamps library: SK_STAMPS_BUILD=1 python -m selkies_gstreamer_amd.ops.build
(-> _lib/libselkies_native_stamps.so); this script selects it and sets SK_STAMPS=1."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SK_STAMPS"] = "1"
os.environ["SK_NATIVE_LIB"] = os.path.join(ROOT, "selkies_gstreamer_amd", "_lib", "libselkies_native_stamps.so")
sys.path.insert(0, ROOT)
from selkies_gstreamer_amd.ops.native import H264Encoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
W, H = 1920, 1080
src = SyntheticDesktop(W, H, "motion")
enc = H264Encoder(W, H, stripe_height=64, backend="hip")
for t in range(3):
    enc.request_keyframe()
    enc.encode(src.frame(t), t)
raw = enc.debug_buffer("stamps", np.uint64).astype(np.int64)
st = raw[:1024].reshape(64, 16)
span = raw[1024:1024 + 34].reshape(17, 2)
dur = (span[:, 1] - span[:, 0]) / 100.0
print("per-slice k_code_intra span us:", dur.round(1).tolist())
hw = raw[1024 + 128:1024 + 133]
print("block 0 waves: simd", ((hw >> 4) & 3).tolist(), "wave slot", (hw & 15).tolist(), "cu", ((hw >> 8) & 15).tolist())
cyc = raw[1024 + 64:1024 + 64 + 34].reshape(17, 2)
print("per-slice memtime cycles:", cyc[:, 0].tolist())
print("per-slice implied MHz:", (cyc[:, 0] / np.maximum(dur, 1e-3)).round(0).tolist())
print("per-slice XCC/SE/CU/SIMD:", [(int(h >> 20) & 15, int(h >> 13) & 7, int(h >> 8) & 15, int(h >> 4) & 3) for h in cyc[:, 1]])
print("stamped block: kernel start -> step 0:", st[0, 0] - raw[1024 + 200], "cycles; last stamped step -> end:",
      raw[1024 + 201] - st[62, 8], "; steps 0..62 span", st[62, 8] - st[0, 0])
print("stamped block: start->loop", raw[1024 + 202] - raw[1024 + 200], "loop->end", raw[1024 + 201] - raw[1024 + 202],
      "steps", raw[1024 + 203], "first stamp - loop start", st[0, 0] - raw[1024 + 202])
print("slice start offsets us:", ((span[:, 0] - span[:, 0].min()) / 100.0).round(1).tolist())
# points: 0 start, 2 pred done, 3 fwd transform done, 9 quant lanes in, 10 dc, 11 analysis,
# 12 crude bound, 4 quant loop done, 5 recon done, 6 code_mb done, 7 edges done, 8 after barrier
seg = [("pred", 0, 2), ("fwd", 2, 3), ("q_in", 3, 9), ("q_dc", 9, 10), ("q_analysis", 10, 11),
       ("q_crude", 11, 12), ("q_tail", 12, 4), ("recon", 4, 5), ("copy", 5, 6), ("store+edges", 6, 7),
       ("barrier", 7, 8)]
rows = []
for step in range(0, 63):
    r = st[step]
    if r[0] == 0 or r[8] == 0:
        continue
    rows.append([r[b] - r[a] for _, a, b in seg] + [r[8] - r[0], r[15] & 0xffff])
rows = np.array(rows)
med = np.median(rows, axis=0)
for (n, _, _), v in zip(seg, med[:-2]):
    print(f"{n:12s} {v:8.0f}")
print(f"{'step total':12s} {med[-2]:8.0f}   quant iterations (median) {med[-1]:.0f}")
print("median step-to-step cycles:", np.median(st[1:63, 8] - st[0:62, 8]))
print("step-to-step cycles:", (st[1:63, 8] - st[0:62, 8]).tolist())
print("after-barrier stamps (relative):", (st[:30, 8] - st[0, 8]).tolist())
print("barrier wait per step:", (st[:63, 8] - st[:63, 7]).tolist())
tot = rows[:, -2]
print("per-step total cycles:", tot.tolist())
print("crude bound per step:", (st[:63, 14]).tolist())
