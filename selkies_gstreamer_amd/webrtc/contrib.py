"""Media helpers: tracks, relay (one producer -> many consumers), recorder,
player and blackhole.

Parity target: the vendored aiortc contrib of the reference
(``src/selkies/webrtc/contrib/media.py``: ``MediaPlayer``, ``MediaRecorder``,
``MediaRelay`` 596, ``MediaBlackhole``), which is built on PyAV containers. Here
the media units are what this framework produces natively: H.264 access units
(Annex-B bytes from the HIP encoder) and PCM/encoded audio payloads, so the
containers are the two formats those map to without a demuxer library:
raw Annex-B ``.h264`` elementary streams and ``.wav`` (PCM s16le).

A frame is a ``MediaFrame(kind, data, pts, time_base)``; ``recv()`` is async and
raises ``MediaStreamError`` when the track has ended.
"""
from __future__ import annotations

import asyncio
import fractions
import struct
import time
import wave
from dataclasses import dataclass
from typing import Optional

import numpy as np


class MediaStreamError(Exception):
    pass


@dataclass
class MediaFrame:
    kind: str                    # "video" (Annex-B access unit) | "audio" (int16 PCM or codec payload)
    data: object                 # bytes or np.ndarray
    pts: int
    time_base: fractions.Fraction
    keyframe: bool = False


class MediaStreamTrack:
    """Base track: subclasses implement ``recv``; ``stop`` ends it for every reader."""

    kind = "unknown"

    def __init__(self):
        self.readyState = "live"

    async def recv(self) -> MediaFrame:   # pragma: no cover - abstract
        raise NotImplementedError

    def stop(self) -> None:
        self.readyState = "ended"


class QueueTrack(MediaStreamTrack):
    """A track fed by ``put`` (e.g. the capture callback); ``None`` ends it."""

    def __init__(self, kind: str, maxsize: int = 0):
        super().__init__()
        self.kind = kind
        self._q: asyncio.Queue = asyncio.Queue(maxsize)

    def put(self, frame: Optional[MediaFrame]) -> None:
        if self._q.maxsize and self._q.full():
            self._q.get_nowait()   # live media: drop the oldest rather than block the producer
        self._q.put_nowait(frame)

    async def recv(self) -> MediaFrame:
        if self.readyState != "live" and self._q.empty():
            raise MediaStreamError
        f = await self._q.get()
        if f is None:
            self.stop()
            raise MediaStreamError
        return f


# -- relay ---------------------------------------------------------------------------------------------

class _RelayTrack(MediaStreamTrack):
    def __init__(self, relay: "MediaRelay", source: MediaStreamTrack, buffered: bool):
        super().__init__()
        self.kind = source.kind
        self._relay = relay
        self._source = source
        self._q: asyncio.Queue = asyncio.Queue(0 if buffered else 1)

    def _push(self, frame: Optional[MediaFrame]) -> None:
        if self._q.maxsize and self._q.full():
            self._q.get_nowait()   # unbuffered consumers always see the newest frame
        self._q.put_nowait(frame)

    async def recv(self) -> MediaFrame:
        if self.readyState != "live":
            raise MediaStreamError
        self._relay._start(self._source)
        f = await self._q.get()
        if f is None:
            self.readyState = "ended"
            raise MediaStreamError
        return f

    def stop(self) -> None:
        super().stop()
        self._relay._unsubscribe(self._source, self)


class MediaRelay:
    """One reader task per source track fans every frame out to all subscribers
    (the reference uses it to share one encoded stream between peers)."""

    def __init__(self):
        self._subs: dict[MediaStreamTrack, set] = {}
        self._tasks: dict[MediaStreamTrack, asyncio.Task] = {}

    def subscribe(self, track: MediaStreamTrack, buffered: bool = True) -> MediaStreamTrack:
        proxy = _RelayTrack(self, track, buffered)
        self._subs.setdefault(track, set()).add(proxy)
        return proxy

    def _start(self, source: MediaStreamTrack) -> None:
        if source not in self._tasks:
            self._tasks[source] = asyncio.ensure_future(self._run(source))

    def _unsubscribe(self, source: MediaStreamTrack, proxy: _RelayTrack) -> None:
        subs = self._subs.get(source)
        if subs is not None:
            subs.discard(proxy)
            if not subs and source in self._tasks:
                self._tasks.pop(source).cancel()

    async def _run(self, source: MediaStreamTrack) -> None:
        while True:
            try:
                frame = await source.recv()
            except MediaStreamError:
                frame = None
            for p in list(self._subs.get(source, ())):
                p._push(frame)
            if frame is None:
                self._tasks.pop(source, None)
                return


# -- sinks ---------------------------------------------------------------------------------------------

class MediaBlackhole:
    """Consumes tracks and discards their frames (counts them)."""

    def __init__(self):
        self._tracks: list = []
        self._tasks: list = []
        self.frames = 0

    def addTrack(self, track: MediaStreamTrack) -> None:
        self._tracks.append(track)

    async def start(self) -> None:
        async def drain(t):
            try:
                while True:
                    await t.recv()
                    self.frames += 1
            except MediaStreamError:
                pass
        self._tasks = [asyncio.ensure_future(drain(t)) for t in self._tracks]

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)


class MediaRecorder:
    """Writes a video track as an Annex-B ``.h264`` elementary stream, or an audio
    track of int16 PCM as ``.wav``; the file type is chosen from the suffix."""

    def __init__(self, path: str, sample_rate: int = 48000, channels: int = 1):
        self.path = path
        self.sample_rate, self.channels = sample_rate, channels
        self._tracks: list = []
        self._tasks: list = []
        self.frames = 0

    def addTrack(self, track: MediaStreamTrack) -> None:
        self._tracks.append(track)

    async def start(self) -> None:
        self._tasks = [asyncio.ensure_future(self._record(t)) for t in self._tracks]

    async def _record(self, track: MediaStreamTrack) -> None:
        if self.path.endswith(".wav"):
            w = wave.open(self.path, "wb")
            w.setnchannels(self.channels)
            w.setsampwidth(2)
            w.setframerate(self.sample_rate)
            try:
                while True:
                    f = await track.recv()
                    w.writeframes(np.asarray(f.data, np.int16).tobytes())
                    self.frames += 1
            except (MediaStreamError, asyncio.CancelledError):
                pass
            finally:
                w.close()
        else:
            with open(self.path, "wb") as fh:
                try:
                    while True:
                        f = await track.recv()
                        fh.write(bytes(f.data))
                        self.frames += 1
                except (MediaStreamError, asyncio.CancelledError):
                    pass

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)


# -- player --------------------------------------------------------------------------------------------

def split_annexb(data: bytes) -> list[bytes]:
    """NAL units (without start codes) of an Annex-B byte stream."""
    out = []
    i, n = 0, len(data)
    starts = []
    while i + 3 <= n:
        if data[i] == 0 and data[i + 1] == 0 and data[i + 2] == 1:
            starts.append(i + 3)
            i += 3
        else:
            i += 1
    for k, s in enumerate(starts):
        e = starts[k + 1] - 3 if k + 1 < len(starts) else n
        while e > s and data[e - 1] == 0:   # 4-byte start code / trailing zeros
            e -= 1
        out.append(data[s:e])
    return out


def _first_mb_is_zero(nal: bytes) -> bool:
    # first_mb_in_slice is the first ue(v) of the slice header: ue == 0 <=> leading bit 1
    return len(nal) > 1 and bool(nal[1] & 0x80)


def access_units(data: bytes) -> list[tuple[bytes, bool]]:
    """Groups NAL units into access units (7.4.1.2.3: SPS/PPS/AUD or a slice with
    first_mb_in_slice == 0 after a slice starts a new one). Returns (Annex-B AU, is_idr)."""
    aus: list[tuple[list, bool]] = []
    cur: list = []
    idr = False
    seen_slice = False
    for nal in split_annexb(data):
        t = nal[0] & 0x1F
        new = seen_slice and (t in (6, 7, 8, 9) or (t in (1, 5) and _first_mb_is_zero(nal)))
        if new:
            aus.append((cur, idr))
            cur, idr, seen_slice = [], False, False
        cur.append(nal)
        if t in (1, 5):
            seen_slice = True
            idr = idr or t == 5
    if cur:
        aus.append((cur, idr))
    return [(b"".join(b"\x00\x00\x00\x01" + n for n in nals), k) for nals, k in aus]


class MediaPlayer:
    """Plays an Annex-B ``.h264`` file (one access unit per frame at ``fps``) or a
    ``.wav`` file (``frame_ms`` PCM chunks) as a track; ``loop`` restarts at the end."""

    def __init__(self, path: str, fps: float = 30.0, frame_ms: int = 20, loop: bool = False,
                 realtime: bool = True):
        self.path = path
        self.loop = loop
        self.realtime = realtime
        if path.endswith(".wav"):
            with wave.open(path, "rb") as w:
                self.sample_rate = w.getframerate()
                pcm = np.frombuffer(w.readframes(w.getnframes()), np.int16)
            n = self.sample_rate * frame_ms // 1000
            self._frames = [MediaFrame("audio", pcm[i:i + n], i, fractions.Fraction(1, self.sample_rate))
                            for i in range(0, len(pcm), n)]
            self._period = frame_ms / 1000.0
            kind = "audio"
        else:
            with open(path, "rb") as fh:
                aus = access_units(fh.read())
            self._frames = [MediaFrame("video", au, int(i * 90000 / fps), fractions.Fraction(1, 90000), k)
                            for i, (au, k) in enumerate(aus)]
            self._period = 1.0 / fps
            kind = "video"
        self.track = _PlayerTrack(self, kind)


class _PlayerTrack(MediaStreamTrack):
    def __init__(self, player: MediaPlayer, kind: str):
        super().__init__()
        self.kind = kind
        self._p = player
        self._i = 0
        self._t0: Optional[float] = None

    async def recv(self) -> MediaFrame:
        if self.readyState != "live":
            raise MediaStreamError
        frames = self._p._frames
        if self._i >= len(frames):
            if not self._p.loop or not frames:
                self.stop()
                raise MediaStreamError
            self._i = 0
            self._t0 = None
        if self._p.realtime:
            now = time.monotonic()
            if self._t0 is None:
                self._t0 = now - self._i * self._p._period
            wait = self._t0 + self._i * self._p._period - now
            if wait > 0:
                await asyncio.sleep(wait)
        f = frames[self._i]
        self._i += 1
        return f


def wav_header_ok(path: str) -> bool:
    with open(path, "rb") as fh:
        h = fh.read(12)
    return h[:4] == b"RIFF" and h[8:12] == b"WAVE" and struct.unpack("<I", h[4:8])[0] > 0
