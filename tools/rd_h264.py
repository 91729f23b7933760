#!/usr/bin/env python3
"""Rate-distortion report of the H.264 encoder: bits per frame vs luma PSNR (decoded
with the independent test decoder, models/h264/decoder.py) over QP and AQ settings,
on the synthetic desktop and moving-desktop content. CPU reference backend (the HIP
backend is bit-identical, tests/test_h264_gpu.py).

usage: python tools/rd_h264.py [--width 640 --height 368 --frames 8] > profiles/r2_rd_h264.md
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selkies_gstreamer_amd.ops.native import H264Encoder          # noqa: E402
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop  # noqa: E402
from tests.h264_util import StripeDecoder, bgrx_to_y709, psnr      # noqa: E402


def run(W, H, kind, qp, aq, frames):
    enc = H264Encoder(W, H, qp=qp, paint_qp=qp, use_paint_over=False, aq_strength=aq, backend="cpu")
    dec = StripeDecoder(W, H)
    src = SyntheticDesktop(W, H, kind=kind, seed=7)
    bits, ps = [], []
    for t in range(frames):
        f = src.frame(t)
        pk = enc.encode(f, t)
        bits.append(8 * sum(len(p.data) - 10 for p in pk))
        for p in pk:
            dec.feed(p.data)
        ps.append(psnr(dec.Y, bgrx_to_y709(f)[:H, :W]))
    enc.close()
    return bits, ps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=368)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--qps", default="18,25,32,38")
    ap.add_argument("--aqs", default="0,1.0")
    a = ap.parse_args()
    print(f"# H.264 rate-distortion ({a.width}x{a.height}, {a.frames} frames: IDR + P, CPU reference = HIP bitstream)\n")
    print("bits = payload bits per frame (IDR / mean P); PSNR = luma PSNR of the decoded frame vs the "
          "BT.709 limited-range source luma (independent decoder), mean over frames.\n")
    for kind in ("desktop", "motion"):
        print(f"## {kind}\n")
        print("| QP | AQ | IDR kbit | P kbit (mean) | total kbit | PSNR dB (mean) | PSNR IDR |")
        print("|---|---|---|---|---|---|---|")
        for qp in [int(x) for x in a.qps.split(",")]:
            for aq in [float(x) for x in a.aqs.split(",")]:
                bits, ps = run(a.width, a.height, kind, qp, aq, a.frames)
                print(f"| {qp} | {aq:.1f} | {bits[0] / 1e3:.1f} | {np.mean(bits[1:]) / 1e3:.1f} | {sum(bits) / 1e3:.1f} | "
                      f"{np.mean(ps):.2f} | {ps[0]:.2f} |", flush=True)
        print()


if __name__ == "__main__":
    main()
