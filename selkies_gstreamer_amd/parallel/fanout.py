"""Packet fan-in over torch.distributed (RCCL on MI355X, gloo on CPU).

Topology for a node that encodes on N GPUs but terminates the websocket
connections in one process ("encode farm" / single-server fan-out): every rank
encodes its own sessions on its own GPU and the per-step packets are gathered
to rank 0 in ONE collective per step — sizes first (one int64 all_gather),
then one padded byte all_gather — instead of one message per stripe. On xGMI
the payload of a 1080p60 step is ~165 KiB per session, so the gather is
latency- not bandwidth-bound and batching the whole step is what matters.

Used by ``bench.py --gather`` and the ``parallel`` tests (gloo, world_size 2).
"""
from __future__ import annotations

import struct
from typing import Sequence

import torch
import torch.distributed as dist


def _device(group=None) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def pack_packets(packets: Sequence[tuple[int, bytes]]) -> bytes:
    """[(session_id, packet_bytes)] -> one blob (u32 count, then u32 session, u32 len, bytes...)."""
    parts = [struct.pack("<I", len(packets))]
    for sid, data in packets:
        parts.append(struct.pack("<II", sid, len(data)))
        parts.append(data)
    return b"".join(parts)


def unpack_packets(blob: bytes) -> list[tuple[int, bytes]]:
    (n,) = struct.unpack_from("<I", blob, 0)
    off, out = 4, []
    for _ in range(n):
        sid, ln = struct.unpack_from("<II", blob, off)
        off += 8
        out.append((sid, blob[off:off + ln]))
        off += ln
    return out


def gather_bytes(blob: bytes, dst: int = 0, group=None) -> list[bytes] | None:
    """Gathers one variable-size byte blob per rank; returns the list on `dst`, None elsewhere.

    Implemented with all_gather (sizes + padded payload) because RCCL's gather
    is built from the same ring and all_gather is the best-tuned path.
    """
    dev = _device(group)
    world = dist.get_world_size(group)
    n = torch.tensor([len(blob)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    mx = max(1, max(sizes))
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    if blob:
        buf[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    if dist.get_rank(group) != dst:
        return None
    return [bytes(b[:sz].cpu().numpy().tobytes()) for b, sz in zip(bufs, sizes)]


def gather_packets(packets: Sequence[tuple[int, bytes]], dst: int = 0, group=None):
    """Gathers [(session_id, packet)] from every rank to `dst` in one step."""
    res = gather_bytes(pack_packets(packets), dst, group)
    if res is None:
        return None
    out = []
    for r, blob in enumerate(res):
        out.extend((r, sid, data) for sid, data in unpack_packets(blob))
    return out


def broadcast_object(obj, src: int = 0, group=None):
    """Control-plane broadcast (settings / keyframe requests) from the websocket rank."""
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=group)
    return lst[0]
