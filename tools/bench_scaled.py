#!/usr/bin/env python3
"""Capture at one size, stream at another (K2 resample fused into K1): fps of a
4K capture encoded as 1080p vs native 1080p, one session."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selkies_gstreamer_amd.ops.native import H264Encoder, PinnedBuffer  # noqa: E402
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop  # noqa: E402


def run(sw, sh, dw, dh, steps=100, warmup=10):
    src = SyntheticDesktop(sw, sh, kind="motion")
    pool = PinnedBuffer((4, sh, sw, 4))
    for i in range(4):
        src.frame(i, out=pool.array[i])
    enc = H264Encoder(dw, dh, stripe_height=64, backend="hip", use_paint_over=False, src_width=sw, src_height=sh)
    lat = []
    for t in range(warmup + steps):
        a = time.perf_counter()
        enc.encode(pool.array[t % 4], t)
        if t >= warmup:
            lat.append(time.perf_counter() - a)
    enc.close()
    pool.close()
    lat = np.array(lat)
    return {"capture": f"{sw}x{sh}", "stream": f"{dw}x{dh}", "fps": round(len(lat) / lat.sum(), 1),
            "p50_ms": round(float(np.median(lat)) * 1e3, 3)}


if __name__ == "__main__":
    for cfg in ((1920, 1080, 1920, 1080), (3840, 2160, 1920, 1080), (2560, 1440, 1920, 1080), (1920, 1080, 1280, 720)):
        print(json.dumps(run(*cfg)), flush=True)
