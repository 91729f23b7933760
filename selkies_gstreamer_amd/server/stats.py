"""System / GPU / network statistics sent to clients every 5 s.

Message shapes follow the reference (selkies.py:2966-3083): ``system_stats``
(cpu_percent, mem_total, mem_used), ``gpu_stats`` (gpu_id, load 0..1,
memory_total, memory_used in bytes), ``network_stats`` (bandwidth_mbps,
latency_ms). The reference reads NVIDIA GPUs through GPUtil/nvidia-smi; here
the GPU numbers come from the amdgpu driver's sysfs counters
(``gpu_busy_percent``, ``mem_info_vram_*``) with ``amd-smi`` as fallback, so the
MI355X that runs the encoder is what the stats panel shows.
"""
from __future__ import annotations

import asyncio
import glob
import json
import logging
import os
import shutil
import subprocess
import time
from datetime import datetime
from typing import Optional

log = logging.getLogger("stats")

try:
    import psutil
except ImportError:  # pragma: no cover
    psutil = None


def system_stats() -> dict:
    if psutil is not None:
        cpu = psutil.cpu_percent()
        vm = psutil.virtual_memory()
        total, used = vm.total, vm.used
    else:
        cpu, total, used = 0.0, 0, 0
    return {"type": "system_stats", "timestamp": datetime.now().isoformat(), "cpu_percent": cpu,
            "mem_total": total, "mem_used": used}


def _amdgpu_cards() -> list[str]:
    cards = []
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        if os.path.exists(os.path.join(dev, "mem_info_vram_total")):
            cards.append(dev)
    return cards


def _read_int(path: str) -> Optional[int]:
    try:
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return None


def gpu_stats(gpu_id: int = 0) -> Optional[dict]:
    """amdgpu sysfs first, amd-smi second; None if no AMD GPU is visible."""
    cards = _amdgpu_cards()
    if gpu_id < len(cards):
        dev = cards[gpu_id]
        busy = _read_int(os.path.join(dev, "gpu_busy_percent"))
        total = _read_int(os.path.join(dev, "mem_info_vram_total"))
        used = _read_int(os.path.join(dev, "mem_info_vram_used"))
        if total:
            return {"type": "gpu_stats", "timestamp": datetime.now().isoformat(), "gpu_id": gpu_id,
                    "load": (busy or 0) / 100.0, "memory_total": total, "memory_used": used or 0}
    return _amd_smi_stats(gpu_id)


def _amd_smi_stats(gpu_id: int) -> Optional[dict]:
    exe = shutil.which("amd-smi")
    if not exe:
        return None
    try:
        out = subprocess.run([exe, "metric", "-g", str(gpu_id), "-u", "-m", "--json"], capture_output=True,
                             timeout=5, text=True)
        data = json.loads(out.stdout)
    except (OSError, subprocess.TimeoutExpired, ValueError):
        return None
    if isinstance(data, list):
        data = data[0] if data else {}
    usage = data.get("usage", {})
    mem = data.get("mem_usage", {})

    def val(d, k):
        v = d.get(k)
        if isinstance(v, dict):
            v = v.get("value")
        try:
            return float(v)
        except (TypeError, ValueError):
            return 0.0
    mib = 1024 * 1024
    return {"type": "gpu_stats", "timestamp": datetime.now().isoformat(), "gpu_id": gpu_id,
            "load": val(usage, "gfx_activity") / 100.0,
            "memory_total": int(val(mem, "total_vram") * mib), "memory_used": int(val(mem, "used_vram") * mib)}


class BandwidthMeter:
    """Bytes-sent accumulator -> Mbit/s per interval (server-wide)."""

    def __init__(self, clock=time.monotonic):
        self.clock = clock
        self.bytes = 0
        self.t0 = clock()

    def add(self, n: int):
        self.bytes += n

    def sample(self) -> float:
        now = self.clock()
        dt = now - self.t0
        mbps = self.bytes * 8 / dt / 1e6 if dt > 0 else 0.0
        self.bytes, self.t0 = 0, now
        return mbps


def network_stats(mbps: float, latency_ms: float) -> dict:
    return {"type": "network_stats", "timestamp": datetime.now().isoformat(),
            "bandwidth_mbps": round(mbps, 2), "latency_ms": round(latency_ms, 1)}


class StatsPublisher:
    """Per-connection collectors + sender (cancel() on disconnect)."""

    def __init__(self, send, meter: BandwidthMeter, latency_fn, gpu_id: int = 0, interval: float = 5.0):
        self.send, self.meter, self.latency_fn = send, meter, latency_fn
        self.gpu_id, self.interval = gpu_id, interval
        self.shared: dict = {}
        self.tasks: list[asyncio.Task] = []

    def start(self):
        self.tasks = [asyncio.create_task(self._collect_system()), asyncio.create_task(self._collect_net()),
                      asyncio.create_task(self._sender())]
        if _amdgpu_cards() or shutil.which("amd-smi"):
            self.tasks.append(asyncio.create_task(self._collect_gpu()))

    async def cancel(self):
        for t in self.tasks:
            t.cancel()
        for t in self.tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        self.tasks = []

    async def _collect_system(self):
        while True:
            self.shared["system"] = system_stats()
            await asyncio.sleep(1.0)

    async def _collect_gpu(self):
        loop = asyncio.get_running_loop()
        while True:
            s = await loop.run_in_executor(None, gpu_stats, self.gpu_id)
            if s is None:
                return
            self.shared["gpu"] = s
            await asyncio.sleep(1.0)

    async def _collect_net(self):
        while True:
            await asyncio.sleep(2.0)
            self.shared["network"] = network_stats(self.meter.sample(), self.latency_fn())

    async def _sender(self):
        while True:
            await asyncio.sleep(self.interval)
            for key in ("system", "gpu", "network"):
                msg = self.shared.pop(key, None)
                if msg is not None:
                    if not await self.send(json.dumps(msg)):
                        return
