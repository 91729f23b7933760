"""One session's frame encoded across ranks: one process per GPU, bands over RCCL.

The multi-process form of :mod:`.banded` (which drives several devices from one
thread). Rank 0 owns the session: it has the captured frame and the websocket
clients. Every step

1. rank 0 broadcasts a small control tensor (frame id, keyframe request, QP), so the
   whole encoder behaves as one session driven from rank 0 (reference: one
   pipeline per display, selkies.py:266-267; keyframe on client connect/PLI);
2. the frame's bands (contiguous whole stripes, :func:`.banded.split_bands`) are
   scattered from rank 0's GPU to the other GPUs with ONE ``dist.scatter`` — on
   MI355X that is RCCL over xGMI, device to device, no host staging;
3. each rank encodes its band from device memory (``H264Encoder.upload_ptr``: a
   D2D copy into the encoder's input buffer) on its own GPU;
4. the band packets come back to rank 0 in ONE gather per step
   (:func:`.fanout.gather_bytes`), their stripe y rebased to the full frame.

Stripes are independent H.264 streams (own SPS/PPS, reference and controller), so
the output is byte-identical to one encoder of the whole frame except for the
0x04 header's y, and no halo or reference data ever crosses a GPU boundary. Per
step the xGMI traffic is the frame once (scatter) plus the packets once (gather).

CPU rehearsal: gloo backend with CPU tensors and the CPU encoder
(tests/test_dist_banded.py, world size 2 and 3).
"""
from __future__ import annotations

import struct
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..ops.native import H264Encoder, Packet
from .banded import rebase_packet, split_bands
from .fanout import gather_bytes

_REC = struct.Struct("<HHHBI")   # y, w, h, key, len


def _pack(packets: list[Packet]) -> bytes:
    parts = [struct.pack("<I", len(packets))]
    for p in packets:
        parts.append(_REC.pack(p.y, p.w, p.h, int(p.key), len(p.data)))
        parts.append(p.data)
    return b"".join(parts)


def _unpack(blob: bytes) -> list[Packet]:
    (n,) = struct.unpack_from("<I", blob, 0)
    off, out = 4, []
    for _ in range(n):
        y, w, h, key, ln = _REC.unpack_from(blob, off)
        off += _REC.size
        out.append(Packet(bytes(blob[off:off + ln]), y, w, h, bool(key)))
        off += ln
    return out


class DistBandedEncoder:
    """Striped H.264 of one WxH session with band r on rank r (collective: every rank
    calls :meth:`encode` each step; only rank 0's ``frame`` is read).

    ``frame`` on rank 0: a uint8 tensor (H, W, 4) on this rank's device (``cuda`` for
    RCCL, CPU for gloo) or a numpy array (copied to the device). Returns the packets
    of the whole frame on rank 0, ``None`` on the other ranks.

    The constructor is collective over the DEFAULT group when ``group`` is an RCCL group
    and no ``control_group`` is given: it creates the gloo twin with ``dist.new_group``,
    which every process of the job must call in the same order. With a sub-group, create
    its gloo twin on all ranks yourself and pass it as ``control_group``."""

    def __init__(self, width: int, height: int, *, stripe_height: int = 64, group=None, backend: str = "hip",
                 control_group=None, **kw):
        if kw.get("fullframe"):
            raise ValueError("distributed bands need striped mode (independent stripe streams)")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.width, self.height = width, height
        self.bands = split_bands(height, stripe_height, self.world)
        if len(self.bands) != self.world:
            raise ValueError(f"{height} rows make only {len(self.bands)} bands of whole stripes for {self.world} ranks")
        self.rows = max(y1 - y0 for y0, y1 in self.bands)   # scatter needs equal chunks: pad to the tallest
        self.nccl = dist.get_backend(group) == "nccl"
        self.device = torch.device("cuda", torch.cuda.current_device()) if self.nccl else torch.device("cpu")
        y0, y1 = self.bands[self.rank]
        dev_index = self.device.index if self.nccl else 0
        self.enc = H264Encoder(width, y1 - y0, stripe_height=stripe_height, backend=backend, device=dev_index, **kw)
        self.recv = torch.empty((self.rows, width, 4), dtype=torch.uint8, device=self.device)
        self.stage = (torch.zeros((self.world, self.rows, width, 4), dtype=torch.uint8, device=self.device)
                      if self.rank == 0 else None)
        # control plane on the host: a gloo twin of an RCCL group, so reading the
        # broadcast values never synchronises a GPU stream
        if control_group is not None:
            self._cgroup = control_group
        elif not self.nccl:
            self._cgroup = group
        elif group is None:
            self._cgroup = dist.new_group(ranks=self._ranks(group), backend="gloo")
        else:   # new_group over a sub-group's ranks would hang the ranks outside it
            raise ValueError("an RCCL sub-group needs control_group= (its gloo twin, created on every rank)")
        self._ctrl = torch.zeros(3, dtype=torch.int64)
        self._key = False
        self._qp = 0
        self.steps = 0

    @staticmethod
    def _ranks(group) -> list[int]:
        if group is None:
            return list(range(dist.get_world_size()))
        return dist.get_process_group_ranks(group)

    # -- control (rank 0; applied on every rank at the next step) ---------------------
    def request_keyframe(self) -> None:
        self._key = True

    def set_qp(self, qp: int) -> None:
        self._qp = int(qp)

    def _control(self, frame_id: int) -> int:
        if self.rank == 0:
            self._ctrl[0], self._ctrl[1], self._ctrl[2] = frame_id, int(self._key), self._qp
            self._key, self._qp = False, 0
        dist.broadcast(self._ctrl, src=self._ranks(self.group)[0], group=self._cgroup)
        fid, key, qp = (int(v) for v in self._ctrl.tolist())
        if key:
            self.enc.request_keyframe()
        if qp > 0:
            self.enc.set_qp(qp)
        return fid

    def _scatter(self, frame) -> None:
        chunks = None
        if self.rank == 0:
            if isinstance(frame, np.ndarray):
                frame = torch.from_numpy(np.ascontiguousarray(frame)).to(self.device)
            if tuple(frame.shape) != (self.height, self.width, 4):
                raise ValueError("frame shape does not match the session")
            for r, (y0, y1) in enumerate(self.bands):
                self.stage[r, : y1 - y0].copy_(frame[y0:y1], non_blocking=True)
            chunks = list(self.stage.unbind(0))
        dist.scatter(self.recv, chunks, src=self._ranks(self.group)[0], group=self.group)

    def encode(self, frame=None, frame_id: int = 0) -> Optional[list[Packet]]:
        fid = self._control(frame_id)
        self._scatter(frame)
        y0, y1 = self.bands[self.rank]
        band = self.recv[: y1 - y0]
        if self.nccl:
            # the encoder's copy waits on the device for what RCCL wrote on torch's stream
            # (an event, not a host synchronisation)
            self.enc.upload_ptr(band.data_ptr(), self.width * 4, fid, keepalive=band,
                                wait_stream=torch.cuda.current_stream(self.device).cuda_stream)
            self.enc.launch()
            mine = self.enc.finish()
        else:
            mine = self.enc.encode(band.numpy(), fid)
        self.steps += 1
        res = gather_bytes(_pack(mine), dst=0, group=self.group)
        if res is None:
            return None
        out: list[Packet] = []
        for r, blob in enumerate(res):
            out.extend(rebase_packet(p, self.bands[r][0]) for p in _unpack(blob))
        return out

    def close(self) -> None:
        self.enc.close()
