#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (counter_collection.csv, one directory per
pass) into per-kernel hardware metrics: VALU busy / utilisation, MFMA busy,
occupancy, LDS bank-conflict cycles per LDS instruction, HBM/L2 bytes and the
achieved bandwidth.

usage: python tools/pmc_summary.py gpurun_out/pmc/h264_p1 gpurun_out/pmc/h264_p2 ... [--top 12]
"""
import argparse
import collections
import csv
import glob
import os

CU_NUM, SIMD_NUM = 256, 1024


def load(dirs):
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(list)
    calls = collections.defaultdict(set)
    for d in dirs:
        path = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
        seen = set()
        for row in csv.DictReader(open(path)):
            k = row["Kernel_Name"].split("(")[0].split("::")[-1]
            if k.startswith("void "):
                k = k[5:]
            sums[k][row["Counter_Name"]] += float(row["Counter_Value"])
            key = (d, row["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                calls[k].add(key)
                if d == dirs[0]:
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return sums, dur, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=14)
    a = ap.parse_args()
    sums, dur, calls = load(a.dirs)
    order = sorted(dur, key=lambda k: -sum(dur[k]))[: a.top]
    print("| kernel | calls | us/call | VALU busy % | VALU util % | MFMA busy % | occupancy % | LDS conflict cyc/LDS instr | "
          "fetch KB/call | write KB/call | GB/s | L2 hit % | VALU / SALU / LDS / VMEM instr per wave |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for k in order:
        s = sums[k]
        n = len(dur[k])
        us = sum(dur[k]) / max(n, 1)
        g = s.get("GRBM_GUI_ACTIVE", 0) or 1
        f = lambda x: f"{x:.1f}"
        valu = 100 * s.get("SQ_ACTIVE_INST_VALU", 0) / CU_NUM / g
        valu_u = 100 * s.get("SQ_THREAD_CYCLES_VALU", 0) / max(s.get("SQ_ACTIVE_INST_VALU", 0) * 64, 1)
        mfma = 100 * s.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (g * SIMD_NUM)
        occ = 400 * s.get("SQ_WAVE_CYCLES", 0) / g / CU_NUM / 32
        lds = s.get("SQ_LDS_BANK_CONFLICT", 0) / max(s.get("SQ_INSTS_LDS", 0), 1)
        npass = max(n, 1)
        fetch = s.get("FETCH_SIZE", 0) / npass
        write = s.get("WRITE_SIZE", 0) / npass
        bw = (fetch + write) * 1024 / (us * 1e3) if us else 0
        hit = 100 * s.get("TCC_HIT", 0) / max(s.get("TCC_HIT", 0) + s.get("TCC_MISS", 0), 1)
        waves = max(s.get("SQ_WAVES", 0), 1)   # same pass as the VALU / SALU counts
        ipw = "/".join(f"{s.get(c, 0) / waves:.0f}" for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU"))
        ipw += "/" + "/".join(f"{s.get(c, 0) / waves:.0f}" for c in ("SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"))
        print(f"| {k} | {n} | {us:.1f} | {f(valu)} | {f(valu_u)} | {f(mfma)} | {f(occ)} | {lds:.2f} | {fetch:.0f} | "
              f"{write:.0f} | {bw:.1f} | {f(hit)} | {ipw} |")


if __name__ == "__main__":
    main()
