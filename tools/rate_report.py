"""Rate-control report (markdown) from a directory of tools/rc_trace.py JSON traces
(tools/gpu.sh rate TAG writes them)."""
import json
import sys
from pathlib import Path

import numpy as np


def main(d: str) -> None:
    rows, notes = [], []
    for f in sorted(Path(d).glob("*.json")):
        r = json.loads(f.read_text())
        t = r["trace"]
        b = np.asarray(t["bytes"], float)
        k = np.asarray(t["key"], bool)
        q = np.asarray(t["qp"])
        budget = r["target_kbps"] * 1000 / r["fps"] / 8 if r["mode"] == "cbr" else None
        nk = b[~k]
        rows.append(
            f"| {r.get('codec', 'h264')} | {r['mode'].upper()} | {r['content']} | {r['target_kbps'] if r['mode'] == 'cbr' else '-'} | "
            f"{r['mean_kbps']:.0f} | {r.get('rate_ratio', '-') if budget else '-'} | "
            f"{(nk.max() / budget) if budget else float('nan'):.2f} | {r.get('nonkey_over_1p5', '-') if budget else '-'} | "
            f"{int(k.sum())} | {r.get('max_key_budgets', '-') if budget else '-'} | {r['qp_min']}-{r['qp_max']} "
            f"(mean {r['qp_mean']}) | {r['redos']} |")
        if budget:
            w = [f"{np.mean(b[i:i + 60]) / budget:.2f}" for i in range(0, len(b), 60)]
            notes.append(f"- {r.get('codec', 'h264')} {r['content']} {r['target_kbps']} kbit/s, mean size per second (x budget): " + " ".join(w))
    print("# K10 rate control on the MI355X (HIP encoders)\n")
    print("600 frames of 1920x1080 at 60 fps per run, `tools/rc_trace.py --backend hip` via `tools/gpu.sh rate`, "
          "synthetic content (`utils/synthetic.py`: motion = scrolling text + moving window, desktop = mostly "
          "static with typing bursts). Sizes are delivered packet bytes (stripe headers included); the "
          "controller budgets the payload. H.264: striped session (64-px stripes, 1.5-frame VBV, overflow guard); "
          "HEVC: full frame, slices of 64-px rows; AV1: full frame, tiles, 120 ms buffer (svtav1enc's "
          "buf-optimal-sz), no guard.\n")
    print("| codec | mode | content | target kbit/s | mean kbit/s | mean / target | max non-key frame (x budget) | "
          "non-key frames > 1.5x | key packets | max key frame (x budget) | QP | guard re-codes |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(r)
    print("\nPer-second means (CBR):\n")
    for n in notes:
        print(n)


if __name__ == "__main__":
    main(sys.argv[1])
