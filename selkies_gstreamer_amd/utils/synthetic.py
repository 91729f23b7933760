"""Synthetic X11-like framebuffer content (BGRx, 4 bytes/pixel).

Used by the benchmark, the synthetic capture source (when no X display is
available) and tests. Three kinds:

* ``motion``  - an actively moving desktop: the whole page scrolls vertically
  every frame (every stripe changes), windows move, and a video-like window
  shows random pixels. This is the "actively moving screen" load the reference
  quotes its 60 fps claim for (docs/component.md:312).
* ``desktop`` - mostly static desktop with one moving window and a scrolling
  text band (typical office use; most stripes are skipped by damage tracking).
* ``noise``   - uniform random pixels in every frame (worst case).
"""
from __future__ import annotations

import numpy as np


class SyntheticDesktop:
    def __init__(self, width: int, height: int, kind: str = "motion", seed: int = 0):
        if kind not in ("motion", "desktop", "noise"):
            raise ValueError(f"unknown synthetic content kind {kind!r}")
        self.w, self.h, self.kind = width, height, kind
        self.rng = np.random.default_rng(seed)
        H2 = height * 3
        yy, xx = np.mgrid[0:H2, 0:width]
        page = np.empty((H2, width, 4), np.uint8)
        page[..., 0] = (200 + 40 * np.sin(xx / 97.0) + 10 * np.cos(yy / 53.0)).clip(0, 255)
        page[..., 1] = (210 + 30 * np.cos(yy / 71.0)).clip(0, 255)
        page[..., 2] = (220 + 25 * np.sin((xx + yy) / 131.0)).clip(0, 255)
        page[..., 3] = 255
        # text-like glyph rows: 12 px lines of random 7x9 "glyphs"
        for ty in range(8, H2 - 16, 18):
            ncol = width // 8
            glyphs = self.rng.random((ncol,)) < 0.7
            bitmap = (self.rng.random((9, ncol * 8)) < 0.35) & np.repeat(glyphs, 8)[None, :]
            bitmap[:, 7::8] = False
            sl = page[ty:ty + 9, : ncol * 8]
            sl[bitmap] = (30, 30, 40, 255)
        self.page = page
        self.video = self.rng.integers(0, 256, (max(16, height // 6), max(16, width // 6), 4), np.uint8)

    def frame(self, t: int, out: np.ndarray | None = None) -> np.ndarray:
        w, h = self.w, self.h
        if out is None:
            out = np.empty((h, w, 4), np.uint8)
        if self.kind == "noise":
            out[...] = self.rng.integers(0, 256, (h, w, 4), np.uint8)
            return out
        H2 = self.page.shape[0]
        scroll = (3 * t) % (H2 - h) if self.kind == "motion" else 0
        out[...] = self.page[scroll:scroll + h]
        if self.kind == "desktop":
            band = slice(h // 5, h // 5 + h // 8)
            s2 = (2 * t) % (H2 - h)
            out[band] = self.page[s2 + h // 5: s2 + h // 5 + h // 8]
        # moving windows with title bars
        for k, (ww, hh, sp) in enumerate(((w // 3, h // 3, 4), (w // 4, h // 4, 7))):
            if self.kind == "desktop" and k == 1:
                continue
            x0 = (sp * t + k * w // 2) % max(1, w - ww)
            y0 = (h // 3 + k * h // 5 + (t * (k + 1)) % 40) % max(1, h - hh)
            out[y0:y0 + hh, x0:x0 + ww] = (236, 236, 236, 255)
            out[y0:y0 + 18, x0:x0 + ww] = (180, 110, 40, 255)
            out[y0 + 30:y0 + 30 + 9, x0 + 10:x0 + ww - 10: 2] = (20, 20, 20, 255)
        if self.kind == "motion":
            vh, vw = self.video.shape[:2]
            vy, vx = h - vh - 20, w - vw - 20
            if vy > 0 and vx > 0:
                self.video = np.roll(self.video, 5, axis=1)
                self.video[:, :5] = self.rng.integers(0, 256, (vh, 5, 4), np.uint8)
                out[vy:vy + vh, vx:vx + vw] = self.video
        return out
