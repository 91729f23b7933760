"""Audio in/out helpers: pcmflux pipeline wrapper and the microphone sink.

Microphone path (reference selkies.py:1642-1840): the browser sends ``0x02`` +
s16le mono 24 kHz PCM; the server makes sure a PulseAudio virtual source
``SelkiesVirtualMic`` (master ``input.monitor``) exists and plays the PCM into
sink ``input`` through a simple playback stream, keeping at most 2 s buffered
and dropping the older half on overflow. The reference uses pulsectl + pasimple;
here ``pactl`` creates the virtual source and libpulse-simple (ctypes) plays.
Everything degrades to a logged no-op when PulseAudio is absent.
"""
from __future__ import annotations

import asyncio
import ctypes
import ctypes.util
import logging
import shutil
import threading
from typing import Optional

from . import protocol

log = logging.getLogger("audio")

VIRTUAL_SOURCE = "SelkiesVirtualMic"
MIC_WRITE_CHUNK = 4800   # 100 ms of s16 mono 24 kHz per pa_simple_write
MASTER_MONITOR = "input.monitor"


class _Spec(ctypes.Structure):
    _fields_ = [("format", ctypes.c_int), ("rate", ctypes.c_uint32), ("channels", ctypes.c_uint8)]


class MicSink:
    def __init__(self):
        self.stream = None
        self.pa = None
        self.ready = False
        self.failed = False
        self.buffer = bytearray()
        self._warned = False
        self._cv = threading.Condition()
        self._thread = None
        self._job = None          # the running writer's stop/done/orphan flags
        self.written = 0
        self.dropped = 0

    def _load(self) -> bool:
        path = ctypes.util.find_library("pulse-simple")
        if not path:
            return False
        try:
            self.pa = ctypes.CDLL(path)
        except OSError:
            return False
        self.pa.pa_simple_new.restype = ctypes.c_void_p
        self.pa.pa_simple_new.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                          ctypes.c_char_p, ctypes.POINTER(_Spec), ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_int)]
        self.pa.pa_simple_write.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.c_int)]
        self.pa.pa_simple_free.argtypes = [ctypes.c_void_p]
        return True

    async def setup(self) -> bool:
        if self.ready or self.failed:
            return self.ready
        pactl = shutil.which("pactl")
        if not pactl or not self._load():
            self.failed = True
            log.warning("microphone forwarding unavailable (needs pactl and libpulse-simple)")
            return False
        p = await asyncio.create_subprocess_exec(pactl, "list", "short", "sources", stdout=asyncio.subprocess.PIPE,
                                                 stderr=asyncio.subprocess.DEVNULL)
        out, _ = await p.communicate()
        if VIRTUAL_SOURCE not in out.decode(errors="replace"):
            p = await asyncio.create_subprocess_exec(pactl, "load-module", "module-virtual-source",
                                                     f"source_name={VIRTUAL_SOURCE}", f"master={MASTER_MONITOR}",
                                                     stdout=asyncio.subprocess.DEVNULL,
                                                     stderr=asyncio.subprocess.DEVNULL)
            if await p.wait() != 0:
                self.failed = True
                log.error("could not load module-virtual-source")
                return False
        err = ctypes.c_int(0)
        spec = _Spec(3, protocol.MIC_SAMPLE_RATE, 1)  # s16le mono 24 kHz
        self.stream = self.pa.pa_simple_new(None, b"SelkiesClientMic", 1, b"input", b"MicStream",
                                            ctypes.byref(spec), None, None, ctypes.byref(err))
        if not self.stream:
            self.failed = True
            log.error("pa_simple_new playback failed (%d)", err.value)
            return False
        self.ready = True
        return True

    def push(self, pcm: bytes) -> int:
        """Queues one chunk for playback and returns at once (called on the event
        loop). A writer thread drains the ring into pa_simple_write, which blocks for
        as long as PulseAudio's buffer is full; the ring keeps at most
        MIC_BUFFER_MAX bytes (2 s) and drops the oldest audio beyond that."""
        if not self.ready or not pcm:
            return 0
        with self._cv:
            self.buffer += pcm
            if len(self.buffer) > protocol.MIC_BUFFER_MAX:
                drop = len(self.buffer) - protocol.MIC_BUFFER_MAX
                drop += drop & 1   # whole s16 samples
                del self.buffer[:drop]
                self.dropped += drop
                if not self._warned:
                    log.warning("microphone buffer overflow; dropping old audio")
                    self._warned = True
            self._cv.notify()
        if self._thread is None:
            self._job = {"stop": False, "done": False, "orphan": False}
            self._thread = threading.Thread(target=self._writer, args=(self.stream, self._job),
                                            name="mic-writer", daemon=True)
            self._thread.start()
        return len(pcm)

    def _write(self, stream, chunk: bytes) -> bool:
        err = ctypes.c_int(0)
        if self.pa.pa_simple_write(stream, chunk, len(chunk), ctypes.byref(err)) < 0:
            log.error("microphone write failed (%d)", err.value)
            return False
        return True

    def _writer(self, stream, job: dict):
        """Drains the ring into ``stream``. ``job`` is this writer's own state: a
        close() that cannot wait out a blocking pa_simple_write marks it orphaned,
        and the writer then frees its stream itself once the write returns."""
        try:
            while True:
                with self._cv:
                    while not self.buffer and not job["stop"]:
                        self._cv.wait()
                    if job["stop"]:
                        return
                    chunk = bytes(self.buffer[:MIC_WRITE_CHUNK])
                    del self.buffer[:len(chunk)]
                if not self._write(stream, chunk):
                    with self._cv:
                        self.ready = False
                        self.buffer.clear()
                    return
                self.written += len(chunk)
        finally:
            with self._cv:
                job["done"] = True
                orphan = job["orphan"]
            if orphan:
                self.pa.pa_simple_free(stream)

    def close(self):
        t, job = self._thread, self._job
        with self._cv:
            if job is not None:
                job["stop"] = True
            self._cv.notify_all()
        if t is not None:
            t.join(timeout=2)
        stream = self.stream
        with self._cv:
            if job is not None and not job["done"]:
                # still inside pa_simple_write: never free a stream under it
                job["orphan"] = True
                stream = None
        if stream and self.pa:
            self.pa.pa_simple_free(stream)
        self._thread = self._job = None
        self.stream = None
        self.ready = False
        self.buffer.clear()


class AudioPipeline:
    """pcmflux capture -> asyncio queue -> broadcast (0x01 0x00 + opus)."""

    def __init__(self, broadcast, device_name: str, channels: int = 2, debug: bool = False):
        self.broadcast = broadcast
        self.device_name = device_name
        self.channels = channels
        self.debug = debug
        self.capture = None
        self.queue: Optional[asyncio.Queue] = None
        self.task: Optional[asyncio.Task] = None
        self.loop = None
        self._cb = None

    @property
    def running(self) -> bool:
        return self.capture is not None

    async def start(self, bitrate: int) -> bool:
        if self.running:
            return True
        try:
            import pcmflux
        except ImportError:
            return False
        if not pcmflux.available():
            log.warning("audio capture unavailable (libpulse-simple/libopus missing)")
            return False
        self.loop = asyncio.get_running_loop()
        self.queue = asyncio.Queue(maxsize=500)
        s = pcmflux.AudioCaptureSettings()
        s.device_name = self.device_name.encode() if self.device_name else None
        s.sample_rate, s.channels, s.opus_bitrate, s.frame_duration_ms = 48000, self.channels, int(bitrate), 20
        s.use_vbr, s.use_silence_gate, s.debug_logging = True, False, self.debug
        q, loop = self.queue, self.loop

        def on_chunk(res_ptr, user):
            r = res_ptr.contents
            if r.size > 0:
                data = bytes(ctypes.cast(r.data, ctypes.POINTER(ctypes.c_ubyte * r.size)).contents)
                loop.call_soon_threadsafe(_put, q, data)

        self._cb = pcmflux.AudioChunkCallback(on_chunk)
        cap = pcmflux.AudioCapture()
        try:
            await self.loop.run_in_executor(None, cap.start_capture, s, self._cb)
        except RuntimeError as e:
            log.error("audio start failed: %s", e)
            return False
        self.capture = cap
        self.task = asyncio.create_task(self._sender())
        return True

    async def _sender(self):
        while True:
            data = await self.queue.get()
            await self.broadcast(protocol.AUDIO_PREFIX + data)

    async def stop(self):
        if self.task:
            self.task.cancel()
            self.task = None
        if self.capture:
            cap, self.capture = self.capture, None
            await asyncio.get_running_loop().run_in_executor(None, cap.stop_capture)
        self.queue = None


def _put(q: asyncio.Queue, item):
    try:
        q.put_nowait(item)
    except asyncio.QueueFull:
        pass
