"""Live load rebalancing of running sessions across the GPUs of one node.

The launcher places sessions once, at start (placement.SessionPlacer). Desktops do
not keep the load they started with: a session that begins playing video or a game
costs several times what an idle desktop does, and a GPU can fail or stall. The
reference has no answer beyond restarting the container on another device
(supervisord), which costs every viewer a reconnect and a key frame.

Here a node-level :class:`Rebalancer` (run by the launcher, parallel/launcher.py
``--rebalance``) polls every session server's ``GET /api/placement`` (per display:
GPU, capture size and fps, mean capture-to-packets latency, frame count) and moves
displays with ``POST /api/move?display=..&gpu=..``. The server hands the move to its
capture thread (csrc/runtime/capture.cpp ``CaptureSession::move_to``), which between
two frames creates the encoder on the new GPU and carries the inter-frame state over
GPU-to-GPU (xGMI peer copy), so the stream continues with P frames: the viewers'
decoders and websocket connections never notice. Only a display whose state cannot
be read any more (its GPU hung) is restarted elsewhere, with a key frame
(:meth:`Supervisor.relocate`).

Policy (:func:`plan_moves`), evaluated every poll:

1. *failed GPUs* — a GPU on which no display produced a frame since the last poll
   (stalled) is evacuated: each of its displays goes to the least-weighted healthy GPU;
2. *overload* — a GPU is overloaded when a display on it misses its frame deadline
   (mean latency > ``overload`` x frame period) or its weight exceeds the capacity;
   the display whose move best levels the weights goes to the least-weighted GPU,
   only if the weight gap exceeds the display's own weight (a move can never be
   undone by the same rule: no ping-pong), at most ``max_moves`` per poll and with a
   per-display cool-down.

Weights are placement.session_weight (pixels x fps relative to 1080p60).
"""
from __future__ import annotations

import asyncio
import logging
import time
from dataclasses import dataclass
from typing import Awaitable, Callable, Iterable, Optional

from .placement import session_weight

log = logging.getLogger("rebalance")


@dataclass
class DisplayLoad:
    session: str        # launcher session (or host) name
    port: int           # that session server's port
    display: str
    gpu: int
    weight: float
    encode_ms: float    # mean capture-to-packets latency
    frames: int
    fps: float

    @property
    def key(self) -> tuple:
        return (self.port, self.display)

    def late(self, overload: float) -> bool:
        return self.fps > 0 and self.encode_ms > overload * 1000.0 / self.fps


def parse_placement(session: str, port: int, doc: dict) -> list[DisplayLoad]:
    """DisplayLoads of one server's ``/api/placement`` answer."""
    out = []
    for did, d in (doc.get("displays") or {}).items():
        if d.get("gpu") is None:
            continue
        fps = float(d.get("fps") or 60.0)
        w, h = int(d.get("width") or 1920), int(d.get("height") or 1080)
        out.append(DisplayLoad(session, port, did, int(d["gpu"]), session_weight(w, h, fps),
                               float(d.get("encode_ms_mean") or 0.0), int(d.get("frames") or 0), fps))
    return out


def plan_moves(loads: list[DisplayLoad], gpus: Iterable[int], capacity: float = 48.0,
               failed: Iterable[int] = (), overload: float = 0.75, max_moves: int = 1,
               cooling: Iterable[tuple] = ()) -> list[tuple[DisplayLoad, int]]:
    """Moves (display, target GPU) for this poll; see the module docstring."""
    failed = set(failed)
    healthy = [g for g in gpus if g not in failed]
    if not healthy:
        return []
    weight = {g: 0.0 for g in healthy}
    for d in loads:
        if d.gpu in weight:
            weight[d.gpu] += d.weight
    moves: list[tuple[DisplayLoad, int]] = []

    def lightest(exclude: int, w: float) -> Optional[int]:
        cands = [g for g in healthy if g != exclude and weight[g] + w <= capacity]
        return min(cands, key=lambda g: (weight[g], g)) if cands else None

    # 1. evacuate failed GPUs (every display, heaviest first)
    for d in sorted((d for d in loads if d.gpu in failed), key=lambda d: -d.weight):
        t = lightest(-1, d.weight)
        if t is None:
            log.error("no GPU can take display %s of %s (%.2f)", d.display, d.session, d.weight)
            continue
        moves.append((d, t))
        weight[t] += d.weight
    # 2. overload: most loaded overloaded GPU first
    cool = set(cooling)
    for _ in range(max_moves):
        over = [g for g in healthy
                if weight[g] > capacity or any(d.gpu == g and d.late(overload) for d in loads)]
        moved = {m[0].key for m in moves}
        best = None
        for g in sorted(over, key=lambda g: -weight[g]):
            for d in sorted((d for d in loads if d.gpu == g and d.key not in cool and d.key not in moved),
                            key=lambda d: -d.weight):
                t = lightest(g, d.weight)
                if t is None or weight[g] - weight[t] <= d.weight:
                    continue
                gap = abs((weight[g] - d.weight) - (weight[t] + d.weight))
                if best is None or gap < best[0]:
                    best = (gap, d, t)
            if best is not None:
                break
        if best is None:
            break
        _, d, t = best
        moves.append((d, t))
        weight[d.gpu] -= d.weight
        weight[t] += d.weight
    return moves


Fetch = Callable[[int], Awaitable[Optional[dict]]]
Move = Callable[[int, str, int], Awaitable[Optional[str]]]

# Header carrying the node's control token (launcher -> every session server through
# SELKIES_CONTROL_TOKEN; server/data_server.py refuses /api/* without it).
CONTROL_HEADER = "X-Selkies-Control-Token"


def _control_headers(token: Optional[str]) -> dict:
    return {CONTROL_HEADER: token} if token else {}


async def http_fetch(port: int, token: Optional[str] = None) -> Optional[dict]:
    import aiohttp
    try:
        async with aiohttp.ClientSession() as s:
            async with s.get(f"http://127.0.0.1:{port}/api/placement", headers=_control_headers(token),
                             timeout=aiohttp.ClientTimeout(total=3)) as r:
                if r.status != 200:
                    log.warning("placement poll of port %d: HTTP %d", port, r.status)
                    return None
                return await r.json()
    except Exception as e:
        log.debug("placement poll of port %d failed: %r", port, e)
        return None


async def http_move(port: int, display: str, gpu: int, token: Optional[str] = None) -> Optional[str]:
    """'continued' / 'keyframe' on success, None when the server could not move."""
    import aiohttp
    try:
        async with aiohttp.ClientSession() as s:
            async with s.post(f"http://127.0.0.1:{port}/api/move", params={"display": display, "gpu": str(gpu)},
                              headers=_control_headers(token), timeout=aiohttp.ClientTimeout(total=15)) as r:
                if r.status != 200:
                    log.warning("move of display %s on port %d: HTTP %d %s", display, port, r.status,
                                (await r.text())[:200])
                    return None
                return (await r.json()).get("result")
    except Exception as e:
        log.warning("move of display %s on port %d failed: %r", display, port, e)
        return None


class Rebalancer:
    """Polls the sessions of a node and applies :func:`plan_moves`.

    ``sessions``: {session name: [ports]}; ``on_failed_move(session, gpu)`` is called
    when a display of a stalled GPU could not be moved (the GPU does not answer): the
    launcher then restarts that session on ``gpu``, once per session and poll. A failed
    overload move is only logged (the display keeps running where it is). ``token``: the
    node's control token, sent with every request of the default HTTP fetch / move."""

    def __init__(self, sessions: dict, gpus: Iterable[int], capacity: float = 48.0, overload: float = 0.75,
                 cooldown_s: float = 30.0, fetch: Optional[Fetch] = None, move: Optional[Move] = None,
                 on_failed_move: Optional[Callable[[str, int], Awaitable[None]]] = None, clock=time.monotonic,
                 token: Optional[str] = None):
        self.sessions = sessions
        self.gpus = list(gpus)
        self.capacity, self.overload, self.cooldown_s = capacity, overload, cooldown_s
        self.fetch = fetch or (lambda port: http_fetch(port, token))
        self.move = move or (lambda port, display, gpu: http_move(port, display, gpu, token))
        self.on_failed_move = on_failed_move
        self.clock = clock
        self._frames: dict = {}       # display key -> frames at the previous poll
        self._moved_at: dict = {}     # display key -> time of its last move
        self.history: list = []       # (display key, from, to, result)

    async def snapshot(self) -> list[DisplayLoad]:
        out = []
        for name, ports in self.sessions.items():
            for port in ports:
                doc = await self.fetch(port)
                if doc:
                    out.extend(parse_placement(name, port, doc))
        return out

    def stalled_gpus(self, loads: list[DisplayLoad]) -> set:
        """GPUs whose every display made no frame since the previous poll. A count
        that went down is a new capture of that display (a resize, a restart or a
        relocation recreates it from 0): a fresh baseline and a live GPU, not a stall."""
        alive, seen = set(), set()
        for d in loads:
            prev = self._frames.get(d.key)
            self._frames[d.key] = d.frames
            if prev is None or d.gpu not in self.gpus:
                continue
            seen.add(d.gpu)
            if d.frames != prev:
                alive.add(d.gpu)
        return seen - alive

    async def step(self) -> list:
        loads = await self.snapshot()
        now = self.clock()
        cooling = [k for k, t in self._moved_at.items() if now - t < self.cooldown_s]
        failed = self.stalled_gpus(loads)
        if failed:
            log.error("GPU(s) %s stalled: evacuating their displays", sorted(failed))
        done = []
        relocate: dict = {}   # session -> target GPU of its first display that could not move
        for d, gpu in plan_moves(loads, self.gpus, self.capacity, failed, self.overload, cooling=cooling):
            res = await self.move(d.port, d.display, gpu)
            self._moved_at[d.key] = now
            self.history.append((d.key, d.gpu, gpu, res))
            log.info("display %s of %s: GPU %d -> %d: %s", d.display, d.session, d.gpu, gpu, res or "failed")
            if res is None and d.gpu in failed:
                relocate.setdefault(d.session, gpu)
            done.append((d, gpu, res))
        # one restart per session and poll: a multi-display session host whose displays
        # were planned onto different GPUs restarts once, on the first target
        if self.on_failed_move is not None:
            for session, gpu in relocate.items():
                await self.on_failed_move(session, gpu)
        return done

    async def run(self, interval: float = 5.0, stop: Optional[asyncio.Event] = None) -> None:
        stop = stop or asyncio.Event()
        while not stop.is_set():
            try:
                await self.step()
            except Exception as e:   # a poll that fails is retried at the next tick
                log.warning("rebalance poll failed: %r", e)
            try:
                await asyncio.wait_for(stop.wait(), interval)
            except asyncio.TimeoutError:
                pass
