"""Rate-distortion of the three encoders on the same synthetic content: H.264
(Constrained Baseline, full-frame pictures), HEVC Main and AV1 Main, each swept over
constant QPs, bytes vs luma PSNR of the reconstruction against the source, and the
Bjontegaard delta rate (BD-rate) of HEVC and AV1 against H.264.

    python tools/rd_codecs.py --width 640 --height 360 --frames 30 [--backend cpu|hip] [--json out.json]

The GPU encoders are bit-exact with the CPU references, so both backends give the same
table; the CPU one is just slower. Prints a markdown table.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

QPS = (22, 27, 32, 37, 42)


def _planes(enc, w, h):
    sy = (w + 15) // 16 * 16
    ref = enc.debug_buffer("ref_y").reshape(-1, sy)[:h, :w].astype(np.float64)
    src = enc.debug_buffer("src_y").reshape(-1, sy)[:h, :w].astype(np.float64)
    return ref, src


def run_point(codec, qp, w, h, frames, kind, backend):
    from selkies_gstreamer_amd.ops.native import H264Encoder
    from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
    src = SyntheticDesktop(w, h, kind=kind)
    enc = H264Encoder(w, h, fullframe=True, codec=codec, backend=backend, qp=qp, paint_qp=qp, use_paint_over=False,
                      fps=60.0, rate_control="cqp")
    nbytes, mse = 0, []
    for t in range(frames):
        pk = enc.encode(src.frame(t), t)
        nbytes += sum(len(p.data) - 10 for p in pk)
        ref, s = _planes(enc, w, h)
        mse.append(np.mean((ref - s) ** 2))
    enc.close()
    m = float(np.mean(mse))
    return {"qp": qp, "bytes": nbytes, "psnr": 99.0 if m == 0 else 10 * np.log10(255.0 ** 2 / m)}


def bd_rate(anchor, test):
    """Bjontegaard delta rate (%) of `test` against `anchor`: cubic fits of log rate over
    PSNR, averaged over the overlapping PSNR interval."""
    pa, ra = np.array([p["psnr"] for p in anchor]), np.log([p["bytes"] for p in anchor])
    pt, rt = np.array([p["psnr"] for p in test]), np.log([p["bytes"] for p in test])
    lo, hi = max(pa.min(), pt.min()), min(pa.max(), pt.max())
    if hi <= lo:
        return float("nan")
    fa, ft = np.polyfit(pa, ra, 3), np.polyfit(pt, rt, 3)
    ia, it = np.polyint(fa), np.polyint(ft)
    da = (np.polyval(ia, hi) - np.polyval(ia, lo)) / (hi - lo)
    dt = (np.polyval(it, hi) - np.polyval(it, lo)) / (hi - lo)
    return float((np.exp(dt - da) - 1) * 100)


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=360)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--backend", default="cpu", choices=("cpu", "hip"))
    ap.add_argument("--content", default="motion,desktop")
    ap.add_argument("--json", default="")
    ap.add_argument("--vs", default="", metavar="TABLE.md",
                    help="an earlier run's markdown table (e.g. profiles/r5_rd_codecs_1080p.md): also print each "
                         "codec's BD-rate against the same codec there")
    ap.add_argument("--ab", default="", metavar="CODEC:ENV",
                    help="A/B one encoder tool: CODEC with ENV=0 (tool off) against the default (on), "
                         "e.g. av1:SK_AV1_PALETTE; prints the tool's BD-rate")
    a = ap.parse_args()
    if a.ab:
        codec, env = a.ab.split(":")
        res = {}
        for kind in a.content.split(","):
            os.environ[env] = "0"
            off = [run_point(codec, q, a.width, a.height, a.frames, kind, a.backend) for q in QPS]
            os.environ.pop(env)
            on = [run_point(codec, q, a.width, a.height, a.frames, kind, a.backend) for q in QPS]
            res[kind] = {"off": off, "on": on, "bd_rate_pct": bd_rate(off, on)}
        if a.json:
            with open(a.json, "w") as f:
                json.dump(res, f)
        print(f"# {codec} with {env} on vs off, {a.width}x{a.height}, {a.frames} frames per point, "
              f"QP {', '.join(map(str, QPS))}, backend {a.backend}\n")
        print("| content | QP | off bytes/frame | off Y-PSNR | on bytes/frame | on Y-PSNR |")
        print("|---|---|---|---|---|---|")
        for kind, r in res.items():
            for p0, p1 in zip(r["off"], r["on"]):
                print(f"| {kind} | {p0['qp']} | {p0['bytes'] / a.frames:.0f} | {p0['psnr']:.2f} | "
                      f"{p1['bytes'] / a.frames:.0f} | {p1['psnr']:.2f} |")
        print("\nBD-rate of the tool (on against off, equal Y-PSNR; negative = fewer bytes):\n")
        for kind, r in res.items():
            print(f"- {kind}: {r['bd_rate_pct']:+.1f} %")
        return
    out = {}
    for kind in a.content.split(","):
        out[kind] = {}
        for c in ("h264", "hevc", "av1"):
            out[kind][c] = []
            for q in QPS:
                out[kind][c].append(run_point(c, q, a.width, a.height, a.frames, kind, a.backend))
                print(f"# {kind} {c} QP {q}: {out[kind][c][-1]}", file=sys.stderr, flush=True)   # progress
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f)
    print(f"# Rate-distortion, {a.width}x{a.height}, {a.frames} frames per point, constant QP "
          f"{', '.join(map(str, QPS))} (AV1: the QP's qindex), backend {a.backend}\n")
    print("| content | codec | QP | bytes/frame | Y-PSNR dB |")
    print("|---|---|---|---|---|")
    for kind, cs in out.items():
        for c, pts in cs.items():
            for p in pts:
                print(f"| {kind} | {c} | {p['qp']} | {p['bytes'] / a.frames:.0f} | {p['psnr']:.2f} |")
    print("\nBD-rate against H.264 at equal Y-PSNR (negative = fewer bytes):\n")
    print("| content | HEVC | AV1 |")
    print("|---|---|---|")
    for kind, cs in out.items():
        print(f"| {kind} | {bd_rate(cs['h264'], cs['hevc']):+.1f} % | {bd_rate(cs['h264'], cs['av1']):+.1f} % |")
    if a.vs:
        old = read_table(a.vs, a.frames)
        print(f"\nBD-rate against the same codec in `{a.vs}` (negative = fewer bytes at equal Y-PSNR):\n")
        print("| content | H.264 | HEVC | AV1 |")
        print("|---|---|---|---|")
        for kind, cs in out.items():
            cells = [f"{bd_rate(old[kind][c], cs[c]):+.1f} %" if old.get(kind, {}).get(c) else "-"
                     for c in ("h264", "hevc", "av1")]
            print(f"| {kind} | " + " | ".join(cells) + " |")


def read_table(path, frames):
    """Rows `| content | codec | QP | bytes/frame | Y-PSNR dB |` of an earlier run's table."""
    out = {}
    for line in open(path):
        f = [x.strip() for x in line.strip().strip("|").split("|")]
        if len(f) == 5 and f[1] in ("h264", "hevc", "av1") and f[2].isdigit():
            out.setdefault(f[0], {}).setdefault(f[1], []).append(
                {"qp": int(f[2]), "bytes": float(f[3]) * frames, "psnr": float(f[4])})
    return out


if __name__ == "__main__":
    main()
