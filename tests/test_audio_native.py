"""Native pcmflux engine (csrc/runtime/audio_capture.cpp): the C++ capture thread,
frame pacing, silence gate, per-packet callback and stop, driven by the synthetic
tone source with raw PCM output (libpulse/libopus are absent on these machines;
with them the same loop reads PulseAudio and calls opus_encode)."""
import ctypes
import threading
import time

import numpy as np
import pytest


def _settings(dev=b"synthetic:1000", gate=False, ch=2, ms=20):
    import pcmflux
    s = pcmflux.AudioCaptureSettings()
    s.device_name = dev
    s.sample_rate, s.channels, s.opus_bitrate, s.frame_duration_ms = 48000, ch, 320000, ms
    s.use_vbr, s.use_silence_gate = True, gate
    return s


def _collect(seconds, **kw):
    import pcmflux
    chunks, threads = [], set()
    lock = threading.Lock()

    def on_chunk(res, user):
        r = res.contents
        data = bytes(ctypes.cast(r.data, ctypes.POINTER(ctypes.c_ubyte * r.size)).contents)
        with lock:
            chunks.append(data)
            threads.add(threading.get_ident())

    cap = pcmflux.AudioCapture()
    cap.start_capture(_settings(**{k: v for k, v in kw.items() if k in ("dev", "gate", "ch", "ms")}),
                      pcmflux.AudioChunkCallback(on_chunk), codec="pcm",
                      synthetic_silence_frames=kw.get("silence", 0))
    time.sleep(seconds)
    cap.stop_capture()
    st = cap.stats()
    return chunks, threads, st


def test_native_loop_paced_tone():
    chunks, threads, st = _collect(0.5)
    # 20 ms frames in real time: ~25 in 0.5 s (scheduler slack allowed)
    assert 12 <= len(chunks) <= 28, len(chunks)   # loaded CI hosts delay the first wake-ups
    assert threading.get_ident() not in threads           # delivered from the native thread
    assert all(len(c) == 960 * 2 * 2 for c in chunks)
    pcm = np.frombuffer(b"".join(chunks), dtype="<i2").reshape(-1, 2)
    assert np.array_equal(pcm[:, 0], pcm[:, 1])
    # a continuous 1 kHz tone across packet boundaries
    t = np.arange(len(pcm)) / 48000.0
    ref = np.rint(8000 * np.sin(2 * np.pi * 1000 * t)).astype(np.int16)
    assert np.abs(pcm[:, 0].astype(int) - ref).max() <= 1
    assert st["packets"] == len(chunks) and st["bytes"] == sum(map(len, chunks))


def test_native_silence_gate():
    chunks, _, st = _collect(0.4, gate=True, silence=8, ch=1)
    assert st["gated"] == 8                     # the leading silent frames never reach the callback
    assert st["frames"] == st["gated"] + st["packets"]
    assert all(np.frombuffer(c, dtype="<i2").any() for c in chunks)
    assert all(len(c) == 960 * 2 for c in chunks)


def test_native_stop_is_prompt_and_restartable():
    import pcmflux
    cap = pcmflux.AudioCapture()
    cb = pcmflux.AudioChunkCallback(lambda r, u: None)
    for _ in range(2):
        cap.start_capture(_settings(ms=10), cb, codec="pcm")
        with pytest.raises(RuntimeError):
            cap.start_capture(_settings(), cb, codec="pcm")   # one capture per object
        t0 = time.monotonic()
        cap.stop_capture()
        assert time.monotonic() - t0 < 0.5


def test_opus_requires_libopus():
    import pcmflux
    from selkies_gstreamer_amd.ops import native
    bits = native.lib().sk_audio_available()
    if bits & 2:
        pytest.skip("libopus present: Opus path is live")
    with pytest.raises(RuntimeError, match="libopus"):
        pcmflux.AudioCapture().start_capture(_settings(), pcmflux.AudioChunkCallback(lambda r, u: None))
