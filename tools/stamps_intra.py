"""Diagnostic: per-segment cycle shares of the intra wavefront kernel (needs a
library built with SK_STAMPS_BUILD=1 and SK_STAMPS=1 at run time)."""
import os, sys
import numpy as np
os.environ["SK_STAMPS"] = "1"
sys.path.insert(0, ".")
from selkies_gstreamer_amd.ops.native import H264Encoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
W, H = 1920, 1080
src = SyntheticDesktop(W, H, "motion")
enc = H264Encoder(W, H, stripe_height=64, backend="hip")
for t in range(3):
    enc.request_keyframe()
    enc.encode(src.frame(t), t)
st = enc.debug_buffer("stamps", np.uint64).reshape(64, 16).astype(np.int64)
names = ["start", "lumamode", "chromamode", "code_mb:in", "quantloop", "recon", "coefcopy", "edges/end"]
for step in (10, 11, 12, 30, 31):
    r = st[step]
    d = [r[i + 1] - r[i] for i in range(7)] + [r[8] - r[0]]
    print(step, dict(zip(["mode_l", "mode_c", "prep", "quant", "recon", "copy", "edges", "step_total"], d)))
for step in (10, 11, 12, 30):
    r = st[step]
    print(step, "q-in->quant", r[9] - r[3], "dc", r[10] - r[9], "analysis", r[11] - r[10], "crude", r[12] - r[11],
          "crude_bits", r[14], "iters", r[15] & 0xffff, "bound", r[15] >> 32)
print("median step cycles (s_memtime ticks):", np.median(st[10:60, 8] - st[9:59, 8]))
