#!/usr/bin/env python3
"""Per-range summary (markdown) of the roctx ranges (csrc/runtime/trace.h) in a
rocprofv3 --marker-trace database.

    python tools/roctx_summary.py gpurun_out/<dir>/run_results.db
"""
import json
import sqlite3
import sys

import numpy as np


def main(path: str) -> None:
    db = sqlite3.connect(path)
    ranges: dict = {}
    for ext, s, e in db.execute("select extdata, start, end from regions"):
        try:
            name = json.loads(ext).get("message", "?")
        except (TypeError, ValueError):
            name = "?"
        ranges.setdefault(name, []).append((e - s) / 1e3)
    print("| range | count | median us | p90 us | max us |")
    print("|---|---|---|---|---|")
    for name, v in sorted(ranges.items()):
        a = np.array(v)
        print(f"| {name} | {len(a)} | {np.median(a):.1f} | {np.percentile(a, 90):.1f} | {a.max():.1f} |")


if __name__ == "__main__":
    main(sys.argv[1])
