"""GPU placement of streaming sessions on a multi-GPU MI355X node.

The reference runs one session per container and leaves GPU choice to the
operator (``--dri_node`` / ``--gpu_id``). Here one node serves
many desktop sessions: every session (display) is one independent encode
pipeline (session-parallel "dp"), so placement is a bin-packing problem over
GPUs. A 1080p60 H.264 session costs ~16 ms/s of GPU time on one MI355X
(profiles/), so a GPU holds dozens; placement spreads sessions least-loaded
first, respecting a per-GPU cap, and keeps a session's displays together
(their captures share one X screen and one upload stream).
"""
from __future__ import annotations

import glob
import os
import threading
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class GpuSlot:
    index: int
    sessions: set = field(default_factory=set)
    weight: float = 0.0          # sum of session weights (e.g. pixels x fps / 1080p60)
    external_load: float = 0.0   # 0..1 busy fraction reported by the driver


def session_weight(width: int, height: int, fps: float) -> float:
    """Relative encode cost of a session vs 1920x1080@60."""
    return (width * height * fps) / (1920 * 1080 * 60)


class SessionPlacer:
    """Thread-safe least-loaded placement with a per-GPU capacity (in 1080p60 units)."""

    def __init__(self, num_gpus: int, capacity_per_gpu: float = 48.0, first_gpu: int = 0):
        if num_gpus < 1:
            raise ValueError("need at least one GPU")
        self.slots = [GpuSlot(first_gpu + i) for i in range(num_gpus)]
        self.capacity = capacity_per_gpu
        self.where: dict = {}
        self._mu = threading.Lock()

    def _score(self, s: GpuSlot) -> float:
        return s.weight / self.capacity + s.external_load

    def acquire(self, session_id: str, weight: float = 1.0) -> Optional[int]:
        """GPU index for a new session, or None if every GPU is full."""
        with self._mu:
            if session_id in self.where:
                return self.where[session_id][0]
            best = None
            for s in self.slots:
                if s.weight + weight > self.capacity:
                    continue
                if best is None or self._score(s) < self._score(best):
                    best = s
            if best is None:
                return None
            best.sessions.add(session_id)
            best.weight += weight
            self.where[session_id] = (best.index, weight)
            return best.index

    def release(self, session_id: str) -> None:
        with self._mu:
            item = self.where.pop(session_id, None)
            if item is None:
                return
            idx, w = item
            for s in self.slots:
                if s.index == idx:
                    s.sessions.discard(session_id)
                    s.weight = max(0.0, s.weight - w)

    def update_external_load(self, loads: dict) -> None:
        with self._mu:
            for s in self.slots:
                if s.index in loads:
                    s.external_load = float(loads[s.index])

    def snapshot(self) -> list[dict]:
        with self._mu:
            return [{"gpu": s.index, "sessions": sorted(s.sessions), "weight": round(s.weight, 3),
                     "load": s.external_load} for s in self.slots]


def visible_gpu_count() -> int:
    """HIP devices visible to this process (HIP_VISIBLE_DEVICES aware), 0 without a GPU."""
    try:
        from selkies_gstreamer_amd.ops import native
        return native.hip_device_count()
    except Exception:
        return 0


def amdgpu_loads() -> dict:
    """{card index: busy fraction} from the amdgpu sysfs counters."""
    out = {}
    cards = sorted(d for d in glob.glob("/sys/class/drm/card*/device")
                   if os.path.exists(os.path.join(d, "gpu_busy_percent")))
    for i, d in enumerate(cards):
        try:
            with open(os.path.join(d, "gpu_busy_percent")) as f:
                out[i] = int(f.read().strip()) / 100.0
        except (OSError, ValueError):
            pass
    return out
