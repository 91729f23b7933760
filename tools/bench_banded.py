#!/usr/bin/env python3
"""8K (or any size) single-session encode, one band vs N bands (parallel/banded.py).

    python tools/bench_banded.py --width 7680 --height 4320 --bands 1 2 4 --devices 0

On a multi-GPU node pass --devices 0 1 2 3 ... (band i runs on devices[i % len]);
on one GPU the bands share the device (concurrent streams, split H2D).
Prints one JSON line per band count.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from selkies_gstreamer_amd.ops.native import PinnedBuffer  # noqa: E402
from selkies_gstreamer_amd.parallel.banded import BandedH264Encoder  # noqa: E402
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--bands", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--devices", type=int, nargs="+", default=[0])
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--content", default="motion")
    args = ap.parse_args()
    W, H = args.width, args.height
    src = SyntheticDesktop(W, H, kind=args.content)
    pool = PinnedBuffer((args.pool, H, W, 4))
    for i in range(args.pool):
        src.frame(i, out=pool.array[i])
    for nb in args.bands:
        devs = [args.devices[i % len(args.devices)] for i in range(nb)]
        enc = BandedH264Encoder(W, H, devs, stripe_height=64, backend="hip", use_paint_over=False)
        lat = []
        nbytes = 0
        for t in range(args.warmup + args.steps):
            a = time.perf_counter()
            pk = enc.encode(pool.array[t % args.pool], t)
            dt = time.perf_counter() - a
            if t >= args.warmup:
                lat.append(dt)
                nbytes += sum(len(p.data) for p in pk)
        enc.close()
        lat = np.array(lat)
        print(json.dumps({"resolution": f"{W}x{H}", "bands": nb, "devices": devs, "fps": round(len(lat) / lat.sum(), 1),
                          "p50_ms": round(float(np.median(lat)) * 1e3, 3),
                          "p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 3),
                          "kib_per_frame": round(nbytes / len(lat) / 1024, 1)}), flush=True)
    pool.close()


if __name__ == "__main__":
    main()
