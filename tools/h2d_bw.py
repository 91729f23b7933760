#!/usr/bin/env python3
"""Pinned host -> device copy bandwidth (the bound of the host-capture pipeline:
every 1080p BGRx frame is 8.3 MB over PCIe). One and several concurrent streams."""
import json
import time

import torch


def run(streams: int, mb: float = 8.2944, iters: int = 200):
    n = int(mb * 1e6)
    hs = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(streams)]
    ds = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(streams)]
    ss = [torch.cuda.Stream() for _ in range(streams)]
    for _ in range(5):
        for h, d, s in zip(hs, ds, ss):
            with torch.cuda.stream(s):
                d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        for h, d, s in zip(hs, ds, ss):
            with torch.cuda.stream(s):
                d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    return streams * iters * n / dt / 1e9


if __name__ == "__main__":
    for s in (1, 2, 4, 8):
        print(json.dumps({"h2d_streams": s, "GBps": round(run(s), 1)}), flush=True)
