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
print("slice start offsets us:", ((span[:, 0] - span[:, 0].min()) / 100.0).round(1).tolist())
# points: 0 start, 2 pred done, 3 fwd transform done, 9 quant lanes in, 10 dc, 11 analysis,
# 12 crude bound, 4 quant loop done, 5 recon done, 6 code_mb done, 7 edges done, 8 after barrier
seg = [("pred", 0, 2), ("fwd", 2, 3), ("q_in", 3, 9), ("q_dc", 9, 10), ("q_analysis", 10, 11),
       ("q_crude", 11, 12), ("q_tail", 12, 4), ("recon", 4, 5), ("copy", 5, 6), ("store+edges", 6, 7),
       ("barrier", 7, 8)]
rows = []
for step in range(10, 60):
    r = st[step]
    rows.append([r[b] - r[a] for _, a, b in seg] + [r[8] - r[0], r[15] & 0xffff])
rows = np.array(rows)
med = np.median(rows, axis=0)
for (n, _, _), v in zip(seg, med[:-2]):
    print(f"{n:12s} {v:8.0f}")
print(f"{'step total':12s} {med[-2]:8.0f}   quant iterations (median) {med[-1]:.0f}")
print("median step-to-step cycles:", np.median(st[11:60, 8] - st[10:59, 8]))
