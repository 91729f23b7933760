"""webrtc/contrib.py: relay fan-out, recorder -> player round trip of HIP/CPU
encoder access units, blackhole (reference: webrtc/contrib/media.py)."""
import asyncio
import fractions

import numpy as np

from selkies_gstreamer_amd.models.h264.decoder import H264Decoder
from selkies_gstreamer_amd.ops.native import H264Encoder
from selkies_gstreamer_amd.webrtc.contrib import (MediaBlackhole, MediaFrame, MediaPlayer, MediaRecorder,
                                                  MediaRelay, MediaStreamError, QueueTrack, access_units)
from tests.h264_util import synthetic_frames

TB = fractions.Fraction(1, 90000)


def _aus(n=6, W=96, H=64):
    enc = H264Encoder(W, H, fullframe=True, qp=26, backend="cpu")
    out = []
    for t, f in enumerate(synthetic_frames(W, H, n, seed=2)):
        pk = enc.encode(f, t)
        if pk:
            out.append((pk[0].data[10:], pk[0].key))
    return out


def test_relay_fans_out_and_ends():
    async def run():
        src = QueueTrack("video")
        relay = MediaRelay()
        subs = [relay.subscribe(src) for _ in range(3)]
        for i in range(5):
            src.put(MediaFrame("video", bytes([i]), i, TB))
        src.put(None)
        got = [[] for _ in subs]

        async def read(k, t):
            try:
                while True:
                    got[k].append((await t.recv()).pts)
            except MediaStreamError:
                pass
        await asyncio.gather(*(read(k, t) for k, t in enumerate(subs)))
        return got
    got = asyncio.run(run())
    assert got == [[0, 1, 2, 3, 4]] * 3


def test_unbuffered_subscriber_sees_newest():
    async def run():
        src = QueueTrack("video")
        relay = MediaRelay()
        fast = relay.subscribe(src, buffered=False)
        pending = asyncio.ensure_future(fast.recv())   # starts the relay
        await asyncio.sleep(0)
        for i in range(4):
            src.put(MediaFrame("video", b"x", i, TB))
        await asyncio.sleep(0.01)
        seen = [(await pending).pts]
        try:
            seen.append((await asyncio.wait_for(fast.recv(), 0.2)).pts)
        except asyncio.TimeoutError:
            pass
        return seen
    seen = asyncio.run(run())
    assert seen[-1] == 3 and len(seen) <= 2   # the slow reader skipped to the newest frame


def test_recorder_player_roundtrip(tmp_path):
    aus = _aus()
    path = str(tmp_path / "out.h264")

    async def record():
        src = QueueTrack("video")
        rec = MediaRecorder(path)
        rec.addTrack(src)
        await rec.start()
        for i, (au, key) in enumerate(aus):
            src.put(MediaFrame("video", au, i * 3000, TB, key))
        src.put(None)
        await asyncio.sleep(0.05)
        await rec.stop()
        return rec.frames
    assert asyncio.run(record()) == len(aus)
    # the elementary stream splits back into the same access units
    with open(path, "rb") as fh:
        split = access_units(fh.read())
    assert [k for _, k in split] == [k for _, k in aus]

    async def play():
        p = MediaPlayer(path, fps=1000, realtime=False)
        out = []
        try:
            while True:
                out.append(await p.track.recv())
        except MediaStreamError:
            pass
        return out
    frames = asyncio.run(play())
    dec = H264Decoder()
    for f in frames:
        dec.decode(f.data)
    assert len(frames) == len(aus) and frames[0].keyframe


def test_wav_recorder_and_player(tmp_path):
    path = str(tmp_path / "a.wav")
    tone = (8000 * np.sin(np.arange(4800) * 0.05)).astype(np.int16)

    async def run():
        src = QueueTrack("audio")
        rec = MediaRecorder(path, sample_rate=48000)
        rec.addTrack(src)
        await rec.start()
        for i in range(0, len(tone), 960):
            src.put(MediaFrame("audio", tone[i:i + 960], i, fractions.Fraction(1, 48000)))
        src.put(None)
        await asyncio.sleep(0.05)
        await rec.stop()
        p = MediaPlayer(path, frame_ms=20, realtime=False)
        chunks = []
        try:
            while True:
                chunks.append((await p.track.recv()).data)
        except MediaStreamError:
            pass
        return np.concatenate(chunks)
    assert np.array_equal(asyncio.run(run()), tone)


def test_blackhole_counts():
    async def run():
        src = QueueTrack("audio")
        bh = MediaBlackhole()
        bh.addTrack(src)
        await bh.start()
        for i in range(7):
            src.put(MediaFrame("audio", b"", i, TB))
        src.put(None)
        await asyncio.sleep(0.05)
        await bh.stop()
        return bh.frames
    assert asyncio.run(run()) == 7
