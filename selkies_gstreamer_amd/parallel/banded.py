"""Spatial parallelism for one session: a frame's stripes split across GPUs.

SURVEY §5.7 maps the reference's scaling axes (resolution up to 7680x4320,
stripe decomposition, selkies.py:266-267, selkies-core.js:2956-2985) onto the
node: an 8K desktop is one session, but its stripes are independent H.264
streams (each stripe has its own SPS/PPS, reference picture and controller
state — the client runs one decoder per stripe y), so contiguous bands of
stripes can be encoded on different GPUs with no halo exchange and no
cross-GPU reference traffic at all. What does cross the boundary is the frame
itself: each GPU uploads only its band's rows over its own PCIe link (an 8K
BGRx frame is 133 MB; one link moves it in ~2.5 ms, eight links in ~0.3 ms),
and the packets are merged on the host in stripe order.

One thread drives all bands: every band is *submitted* (upload + one graph
launch, asynchronous) before any is *finished*, so the GPUs work concurrently.
Bands that share a device use that device's shared copy stream: their uploads
run back to back in band order at full PCIe rate and each band's kernels start
as soon as its own rows have landed — on a single GPU this overlaps most of the
frame upload with encoding (lower latency than one encoder of the whole frame). Output is byte-identical to a
single-GPU encoder of the whole frame except for the 0x04 header's stripe y,
which is rebased to the full frame (tests/test_parallel_banded.py).
"""
from __future__ import annotations

import struct
from typing import Sequence

import numpy as np

from ..ops.native import H264Encoder, Packet


def split_bands(height: int, stripe_height: int, parts: int) -> list[tuple[int, int]]:
    """Row ranges [y0, y1) of `parts` bands made of whole stripes, sizes as equal as possible."""
    n = (height + stripe_height - 1) // stripe_height
    parts = max(1, min(parts, n))
    bounds = [round(i * n / parts) for i in range(parts + 1)]
    return [(b0 * stripe_height, min(height, b1 * stripe_height)) for b0, b1 in zip(bounds, bounds[1:])]


def rebase_packet(p: Packet, y0: int) -> Packet:
    """Shifts a band-local 0x04 stripe packet to full-frame coordinates."""
    if y0 == 0:
        return p
    data = bytearray(p.data)
    struct.pack_into(">H", data, 4, p.y + y0)
    return Packet(bytes(data), p.y + y0, p.w, p.h, p.key)


class BandedH264Encoder:
    """Striped H.264 for one frame on several devices (or several encoders on one).

    ``devices``: HIP device per band (may repeat). Keyword arguments go to every
    band's :class:`H264Encoder`; ``fullframe`` is not supported (a single picture
    would need cross-band motion compensation and in-order slice assembly)."""

    def __init__(self, width: int, height: int, devices: Sequence[int], *, stripe_height: int = 64,
                 backend: str = "hip", **kw):
        if kw.get("fullframe"):
            raise ValueError("banded encoding needs striped mode (independent stripe streams)")
        self.width, self.height = width, height
        self.bands = split_bands(height, stripe_height, len(devices))
        shared = {d for d in devices if list(devices).count(d) > 1}
        self.encoders = [H264Encoder(width, y1 - y0, stripe_height=stripe_height, device=dev, backend=backend,
                                     shared_copy=dev in shared, **kw)
                         for (y0, y1), dev in zip(self.bands, devices)]

    def encode(self, bgrx: np.ndarray, frame_id: int = 0) -> list[Packet]:
        if bgrx.shape[0] != self.height:
            raise ValueError("frame height does not match the encoder")
        if not bgrx.flags["C_CONTIGUOUS"]:
            bgrx = np.ascontiguousarray(bgrx)
        for enc, (y0, y1) in zip(self.encoders, self.bands):
            enc.submit(bgrx[y0:y1], frame_id)   # row views: no copy
        out: list[Packet] = []
        for enc, (y0, _) in zip(self.encoders, self.bands):
            out.extend(rebase_packet(p, y0) for p in enc.finish())
        return out

    def request_keyframe(self) -> None:
        for e in self.encoders:
            e.request_keyframe()

    def set_qp(self, qp: int, paint_qp: int = 0) -> None:
        for e in self.encoders:
            e.set_qp(qp, paint_qp)

    def close(self) -> None:
        for e in self.encoders:
            e.close()
