"""Diagnostic: the HIP chunk-parallel CABAC state (cu_t / cu_r / tail per unit chunk)
against the host model (CPU encoder with SK_HEVC_PCABAC=1) on one frame sequence."""
import os
import sys
import numpy as np
sys.path.insert(0, '.')
from selkies_gstreamer_amd.ops.native import HevcEncoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop

W, H = int(sys.argv[1]), int(sys.argv[2])
kind = sys.argv[3] if len(sys.argv) > 3 else "desktop"
frames = int(sys.argv[4]) if len(sys.argv) > 4 else 2
gpu = HevcEncoder(W, H, backend="hip", device=0)
os.environ["SK_HEVC_PCABAC"] = "1"
cpu = HevcEncoder(W, H, backend="cpu")
src = SyntheticDesktop(W, H, kind=kind)
W16 = (W + 15) // 16
for t in range(frames):
    f = src.frame(t)
    pg, pc = gpu.encode(f, t), cpu.encode(f, t)
    d = np.frombuffer(cpu.debug_buffer("pc_dbg", np.uint8), np.uint32).reshape(-1, 3)
    ct = np.frombuffer(gpu.debug_buffer("cu_t", np.uint8), np.uint32)
    cr = np.frombuffer(gpu.debug_buffer("cu_r", np.uint8), np.uint16)
    tl = np.frombuffer(gpu.debug_buffer("tail", np.uint8), np.uint8).reshape(-1, 2)
    tlv = tl[:, 0].astype(np.uint32) | (tl[:, 1].astype(np.uint32) << 8)
    eq = [p.data for p in pg] == [p.data for p in pc]
    bad_t = np.nonzero(ct != d[:, 0])[0]
    bad_r = np.nonzero(cr != d[:, 1])[0]
    bad_tl = np.nonzero(tlv != d[:, 2])[0]
    print(f"frame {t}: packets equal {eq}; cu_t diffs {len(bad_t)}, cu_r diffs {len(bad_r)}, tail diffs {len(bad_tl)}", flush=True)
    for name, bad, g, c in (("t", bad_t, ct, d[:, 0]), ("r", bad_r, cr, d[:, 1]), ("tail", bad_tl, tlv, d[:, 2])):
        for i in bad[:5]:
            print(f"  {name} unit {i} ({i % W16}, {i // W16}): gpu {g[i]} host {c[i]}")
    if not eq:   # the substreams of the first differing slice NAL, GPU (pre emulation prevention) vs CPU
        from selkies_gstreamer_amd.models.hevc.decoder import split_annexb, unescape
        ng, nc = split_annexb(pg[0].data[10:]), split_annexb(pc[0].data[10:])
        k = next(i for i, (a, b) in enumerate(zip(ng, nc)) if a != b)
        sub = np.frombuffer(gpu.debug_buffer("sub", np.uint8), np.uint8)
        size = np.frombuffer(gpu.debug_buffer("sub_size", np.uint8), np.int32)
        rb = np.frombuffer(gpu.debug_buffer("row_bits", np.uint8), np.uint32)
        cw, stride = (W16 + 1) // 2, len(sub) // ((H + 31) // 32)
        cpu_rbsp = unescape(nc[k][2:])
        # the slice's last CTB row is the one whose substream ends the NAL: find it by size
        K = len(size) // ((H + 31) // 32)
        print("  cpu nal", k, "rbsp len", len(cpu_rbsp), "tail", cpu_rbsp[-8:].hex())
        for r in (2 * k, 2 * k + 1):
            sz = int(size[r * K])
            print("  gpu row", r, "size", sz, "T", int(rb[r * K]), "tail", bytes(sub[r * stride + max(0, sz - 8):r * stride + sz]).hex())
        for r in range((H + 31) // 32):
            sz = int(size[r * K])
            g = bytes(sub[r * stride:r * stride + sz])
            if sz > 4 and cpu_rbsp.endswith(g[:-1]) and g != cpu_rbsp[-len(g):]:
                c = cpu_rbsp[-len(g):]
                d = [i for i in range(len(g)) if g[i] != c[i]]
                print(f"  nal {k}: CTB row {r} T {rb[r * K]} size {sz} differing bytes {d[:8]} gpu {[g[i] for i in d[:4]]} cpu {[c[i] for i in d[:4]]}")
                last = [u for u in range(2 * r * W16, min(2 * r + 2, (H + 15) // 16) * W16)]
                print("   T&7", rb[r * K] & 7, "(T+1)>>3", (rb[r * K] + 1) >> 3, "tail of last unit",
                      tlv[(2 * r + 1) * W16 + W16 - 1] if 2 * r + 1 < (H + 15) // 16 else None, "tail hex", hex(int(tlv[(2 * r + 1) * W16 + W16 - 1])))
