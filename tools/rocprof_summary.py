#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (``*_results.db``) as a markdown
table (per-kernel calls, total/median/p90 durations, share, VGPRs, LDS, scratch).

usage: python tools/rocprof_summary.py gpurun_out/prof/run_results.db > profiles/x.md
"""
import collections
import sqlite3
import sys

import numpy as np


def main(path: str):
    c = sqlite3.connect(path)
    rows = list(c.execute(
        "select name, duration, grid_x, workgroup_x, scratch_size, vgpr_count, lds_size from kernels"))
    d = collections.defaultdict(list)
    meta = {}
    for n, du, gx, wx, sc, vg, lds in rows:
        k = n.split("(")[0].split("::")[-1]
        d[k].append(du / 1000.0)
        meta[k] = (gx // max(wx, 1), wx, sc, vg, lds)
    # shares exclude the start-up warm-up (k_touch_pages faults in the session buffers
    # once, before the first frame; docs/design: it is not per-frame work)
    warm = {"k_touch_pages"}
    total = sum(sum(v) for k, v in d.items() if k not in warm)
    print(f"source: `{path}`  \n")
    if warm & set(d):
        print(f"shares are of the per-frame work: {', '.join(sorted(warm & set(d)))} (start-up warm-up, "
              f"{sum(sum(d[k]) for k in warm & set(d)) / 1000:.2f} ms) is listed but not counted\n")
    print("| kernel | calls | total ms | share | median us | p90 us | max us | blocks | wg | vgpr | lds B | scratch B/lane |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v = np.asarray(v)
        g, w, sc, vg, lds = meta[k]
        share = "-" if k in warm else f"{100 * v.sum() / total:.1f}%"
        print(f"| {k} | {len(v)} | {v.sum() / 1000:.2f} | {share} | {np.median(v):.1f} | "
              f"{np.percentile(v, 90):.1f} | {v.max():.1f} | {g} | {w} | {vg} | {lds} | {sc} |")


if __name__ == "__main__":
    main(sys.argv[1])
