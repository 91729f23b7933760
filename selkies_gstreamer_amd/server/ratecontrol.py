"""Bitrate -> QP rate control for the H.264 encoder.

The reference's WebRTC mode runs its hardware/x264 encoders in CBR with a VBV
of 1.5 frame intervals (legacy/gstwebrtc_app.py:101-105, 345, 500, 633) and
lets the client or GCC change ``video_bitrate`` at runtime (``vb,<kbps>``,
webrtc_input.py:615; rtpgccbwe, gstwebrtc_app.py:1555-1572). The HIP encoder
is QP-driven per frame, so CBR becomes a frame-level feedback loop on QP:

* H.264 bits scale roughly by 2^(-dQP/6), so an overshoot of ``r`` = actual /
  target asks for ``+6*log2(r)`` QP (bounded steps, fast up);
* undershoot lowers QP one step at a time and only while frames are large
  enough to mean real motion — a static desktop (paint-over, skipped stripes)
  must not drive QP to the floor and then burst when motion resumes;
* the paint-over QP tracks the motion QP minus a fixed refinement offset;
* a VBV-like guard: a frame larger than ``vbv_frames`` frame budgets raises QP
  immediately (a keyframe is exempt).
"""
from __future__ import annotations

import math
from typing import Optional


class RateController:
    def __init__(self, target_bps: int, fps: float, qp_init: int = 25, qp_min: int = 12, qp_max: int = 46,
                 paint_offset: int = 7, window_frames: int = 15, vbv_frames: float = 1.5):
        self.target_bps = int(target_bps)
        self.fps = float(fps)
        self.qp = int(qp_init)
        self.qp_min, self.qp_max = qp_min, qp_max
        self.paint_offset = paint_offset
        self.window = window_frames
        self.vbv_frames = vbv_frames
        self._bytes = 0
        self._frames = 0

    def set_target(self, bps: int) -> None:
        self.target_bps = max(100_000, int(bps))

    def set_fps(self, fps: float) -> None:
        self.fps = max(1.0, float(fps))

    @property
    def paint_qp(self) -> int:
        return max(self.qp_min, self.qp - self.paint_offset)

    def _clamp(self, q: int) -> int:
        return max(self.qp_min, min(self.qp_max, q))

    def on_frame(self, nbytes: int, keyframe: bool = False) -> Optional[int]:
        """Feed one encoded frame; returns the new QP when it changed, else None."""
        budget = self.target_bps / 8.0 / self.fps
        old = self.qp
        if not keyframe and nbytes > self.vbv_frames * budget * 2:
            self.qp = self._clamp(self.qp + 2)
        self._bytes += nbytes
        self._frames += 1
        if self._frames >= self.window:
            actual = self._bytes * 8.0 * self.fps / self._frames
            r = actual / max(1.0, self.target_bps)
            if r > 1.1:
                self.qp = self._clamp(self.qp + max(1, min(6, round(6 * math.log2(r)))))
            elif r < 0.7 and self._bytes / self._frames > 0.25 * budget:
                self.qp = self._clamp(self.qp - 1)
            self._bytes = self._frames = 0
        return self.qp if self.qp != old else None
