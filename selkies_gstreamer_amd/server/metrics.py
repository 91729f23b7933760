"""Prometheus metrics (reference legacy/metrics.py:39-253).

Same gauge names as the reference (``fps``, ``gpu_utilization``, ``latency``,
histogram ``fps_hist`` with buckets 0/20/40/60, info ``webrtc_statistics``)
plus encoder-side gauges from the native capture sessions
(``selkies_encode_ms``, ``selkies_frames_total``, ``selkies_bytes_total``,
``selkies_clients``). Served at ``/metrics`` on the data server port (the
reference starts a separate HTTP server; one port is simpler behind a proxy).
Client WebRTC stats can be appended to a CSV file like the reference does.
"""
from __future__ import annotations

import csv
import json
import logging
import os
from typing import Optional

from aiohttp import web

log = logging.getLogger("metrics")

try:
    from prometheus_client import CollectorRegistry, Gauge, Histogram, Info, generate_latest, CONTENT_TYPE_LATEST
    HAVE_PROM = True
except ImportError:  # pragma: no cover
    HAVE_PROM = False


class _EncodeHistogram:
    """Prometheus histogram of per-frame encode time per display, from the native
    capture session's bucket counters (no per-frame Python work)."""

    def __init__(self, metrics: "Metrics"):
        self.m = metrics

    def describe(self):
        return []

    def collect(self):
        from prometheus_client.core import HistogramMetricFamily
        fam = HistogramMetricFamily("selkies_encode_seconds", "Per-frame encode time (capture -> packets)",
                                    labels=["display"])
        for did, module in list(self.m.captures.items()):
            try:
                st = module.stats()
                les, counts = st["encode_ms_buckets"], st["encode_ms_counts"]
            except Exception:
                continue
            cum, buckets = 0, []
            for le, c in zip(les, counts):
                cum += c
                buckets.append(("+Inf" if le == float("inf") else str(le / 1e3), cum))
            fam.add_metric([did], buckets, sum_value=st["encode_ms_mean"] * st["frames"] / 1e3)
        yield fam


class Metrics:
    def __init__(self, server=None, csv_path: Optional[str] = None):
        self.server = server
        self.captures: dict = {}
        self.csv_path = csv_path
        self.registry = CollectorRegistry() if HAVE_PROM else None
        if HAVE_PROM:
            r = self.registry
            self.fps = Gauge("fps", "Frames per second observed by the client", registry=r)
            self.fps_hist = Histogram("fps_hist", "Histogram of FPS observed by the client",
                                      buckets=(0, 20, 40, 60), registry=r)
            self.gpu_utilization = Gauge("gpu_utilization", "Utilization percentage reported by the GPU",
                                         registry=r)
            self.latency = Gauge("latency", "Latency observed by the client (ms)", registry=r)
            self.webrtc_statistics = Info("webrtc_statistics", "Client WebRTC/stream statistics", registry=r)
            self.encode_ms = Gauge("selkies_encode_ms", "Mean encode time per frame (ms)", ["display"], registry=r)
            self.frames = Gauge("selkies_frames_total", "Frames encoded", ["display"], registry=r)
            self.bytes = Gauge("selkies_bytes_total", "Bytes produced by the encoder", ["display"], registry=r)
            self.clients = Gauge("selkies_clients", "Connected websocket clients", registry=r)
            r.register(_EncodeHistogram(self))

    # capture lifecycle hooks (called by DataStreamingServer)
    def capture_started(self, did: str, module):
        self.captures[did] = module

    def capture_stopped(self, did: str):
        self.captures.pop(did, None)

    def set_fps(self, fps: float):
        if HAVE_PROM:
            self.fps.set(fps)
            self.fps_hist.observe(fps)

    def set_latency(self, ms: float):
        if HAVE_PROM:
            self.latency.set(ms)

    def set_gpu_utilization(self, pct: float):
        if HAVE_PROM:
            self.gpu_utilization.set(pct)

    def set_webrtc_stats(self, kind: str, payload: str):
        """``_stats_video`` / ``_stats_audio`` JSON from the client -> Info + optional CSV."""
        try:
            stats = json.loads(payload)
        except ValueError:
            return
        flat = {f"{kind}_{k}": str(v) for k, v in (stats.items() if isinstance(stats, dict) else [])}
        if HAVE_PROM and flat:
            self.webrtc_statistics.info(flat)
        if self.csv_path and flat:
            self._append_csv(flat)

    def _append_csv(self, row: dict):
        exists = os.path.exists(self.csv_path)
        header = list(row)
        if exists:
            with open(self.csv_path, newline="") as f:
                old = next(csv.reader(f), [])
            if set(header) - set(old):  # schema grew: rewrite with the union of columns
                with open(self.csv_path, newline="") as f:
                    rows = list(csv.DictReader(f))
                header = old + [h for h in header if h not in old]
                with open(self.csv_path, "w", newline="") as f:
                    w = csv.DictWriter(f, fieldnames=header)
                    w.writeheader()
                    w.writerows(rows)
            else:
                header = old
        with open(self.csv_path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=header)
            if not exists:
                w.writeheader()
            w.writerow(row)

    def refresh(self):
        if not HAVE_PROM:
            return
        for did, module in list(self.captures.items()):
            try:
                st = module.stats()
            except Exception:
                continue
            self.encode_ms.labels(did).set(st["encode_ms_mean"])
            self.frames.labels(did).set(st["frames"])
            self.bytes.labels(did).set(st["bytes"])
        if self.server is not None:
            self.clients.set(len(self.server.clients))

    async def handler(self, request):
        if not HAVE_PROM:
            raise web.HTTPNotFound()
        self.refresh()
        return web.Response(body=generate_latest(self.registry), headers={"Content-Type": CONTENT_TYPE_LATEST})
