"""Shared helpers for the H.264 encoder tests: synthetic desktop-like frames,
decoding of 0x04 stripe packets and PSNR."""
from __future__ import annotations

import numpy as np

from selkies_gstreamer_amd.models.h264.decoder import H264Decoder


def synthetic_frames(w: int, h: int, n: int, seed: int = 0, kind: str = "desktop"):
    """Yields n BGRx frames: 'desktop' = gradient background + moving window +
    scrolling text-like band; 'noise' = uniform random pixels."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    text = rng.integers(0, 2, (h * 2, w), dtype=np.uint8) * 200
    for t in range(n):
        if kind == "noise":
            yield rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
            continue
        f = np.zeros((h, w, 4), np.uint8)
        f[..., 0] = (xx // 2 + 40) % 256
        f[..., 1] = (yy // 2 + 60) % 256
        f[..., 2] = 90
        q = h // 4
        sc = (3 * t) % h
        f[q:2 * q, :, 0] = text[sc + q: sc + 2 * q, :]
        f[q:2 * q, :, 1] = text[sc + q: sc + 2 * q, :]
        wx = (5 * t) % max(1, w - w // 3)
        f[h // 2: h // 2 + q, wx: wx + w // 3, :3] = (200, 120, 30)
        f[h // 2 + 4: h // 2 + 8, wx + 4: wx + w // 3 - 4, :3] = rng.integers(0, 255, 3)
        yield f


class StripeDecoder:
    """Decodes 0x04 stripe packets into a full frame (one decoder per stripe y,
    as the browser client does, selkies-core.js:2956-3007)."""

    def __init__(self, w: int, h: int):
        self.w, self.h = w, h
        self.decs: dict[int, H264Decoder] = {}
        self.Y = np.zeros((h, w), np.uint8)
        self.U = np.zeros((h // 2, w // 2), np.uint8)
        self.V = np.zeros((h // 2, w // 2), np.uint8)

    def feed(self, packet: bytes):
        assert packet[0] == 0x04
        key = packet[1]
        y = int.from_bytes(packet[4:6], "big")
        pw = int.from_bytes(packet[6:8], "big")
        ph = int.from_bytes(packet[8:10], "big")
        if key:
            self.decs[y] = H264Decoder()
        dec = self.decs[y]
        frames = dec.decode(packet[10:])
        assert len(frames) == 1, "one picture per packet"
        Y, U, V = frames[0]
        assert Y.shape == (ph, pw)
        self.Y[y:y + ph] = Y
        self.U[y // 2:(y + ph) // 2] = U
        self.V[y // 2:(y + ph) // 2] = V
        return dec


def bgrx_to_y709(f: np.ndarray) -> np.ndarray:
    r, g, b = f[..., 2].astype(np.int64), f[..., 1].astype(np.int64), f[..., 0].astype(np.int64)
    return ((47 * r + 157 * g + 16 * b + 128) >> 8) + 16


def psnr(a: np.ndarray, b: np.ndarray) -> float:
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)
