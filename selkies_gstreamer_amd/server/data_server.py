"""Data websocket server: sessions, displays, capture lifecycle, fan-out, backpressure.

Behavior parity with the reference ``DataStreamingServer`` (selkies.py:803-2964,
SURVEY C04/C05/C07/C08/C09/C10/C11): same wire protocol (see :mod:`.protocol`),
same display registry (``primary`` + one secondary), same settings sanitization,
same reconnect debounce and ``KILL`` on takeover, same stats cadence.

MI355X-first differences:

* video comes from the native capture session (pixelflux-compatible API over
  libselkies_native): HIP colour conversion, damage, motion search and CAVLC on
  the GPU; each display may be pinned to its own HIP device (``gpu_id`` + display
  index, see :mod:`selkies_gstreamer_amd.parallel.placement`);
* transport is aiohttp: one ordered outbound queue + writer task per client, so
  a slow viewer never blocks the event loop or other viewers, and static client
  files / ``/health`` / ``/metrics`` are served from the same port;
* frame backpressure really gates sending (for every display) and asks the
  encoder for a keyframe when it lifts, because skipped P-stripes are not
  decodable (the reference only gates secondary displays).
"""
from __future__ import annotations

import asyncio
import base64
import binascii
import ctypes
import hmac
import json
import logging
import os
import html
import time
import urllib.parse
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Callable, Optional

from aiohttp import WSMsgType, web

from . import protocol
from .audio import AudioPipeline, MicSink
from .display import WindowManagerSwap, XrandrDisplay, compute_layout, display_env, set_cursor_size, set_dpi
from .settings import Settings
from .stats import BandwidthMeter, StatsPublisher

log = logging.getLogger("data_websocket")

VIDEO_QUEUE_SIZE = 120
RECONNECT_DEBOUNCE_S = 0.5
CURSOR_SIZE = 32
VIDEO_KEYS = ("encoder", "framerate", "h264_crf", "h264_fullcolor", "h264_streaming_mode", "jpeg_quality",
              "paint_over_jpeg_quality", "use_cpu", "h264_paintover_crf", "h264_paintover_burst_frames",
              "use_paint_over_quality", "h264_bitrate")


class _VideoFrame:
    """All stripe messages of one encoded frame, queued as one unit."""
    __slots__ = ("msgs", "key")

    def __init__(self, msgs: list, key: bool):
        self.msgs = msgs
        self.key = key


class Client:
    """One websocket connection with its own ordered outbound queue.

    Video is bounded per viewer: at most ``MAX_VIDEO_FRAMES`` encoded frames may
    wait in the queue. A slower viewer loses whole frames (never a partial one),
    and once its queue has drained it asks for a keyframe through ``on_resync``
    and skips delta frames until one arrives, so its decoders resynchronise. The
    reference skips websockets above the write high-water mark in
    ``websockets.broadcast`` (selkies.py:2818); control and text messages here are
    never dropped.
    """

    MAX_VIDEO_FRAMES = 8   # ~133 ms at 60 fps

    def __init__(self, ws: web.WebSocketResponse, remote: str, meter: BandwidthMeter,
                 on_resync: Optional[Callable[["Client"], None]] = None):
        self.ws = ws
        self.remote = remote
        self.meter = meter
        self.out: asyncio.Queue = asyncio.Queue()
        self.writer = asyncio.create_task(self._write())
        self.display_id: Optional[str] = None
        self.closed = False
        self.on_resync = on_resync
        self.video_queued = 0        # video frames waiting in self.out
        self.video_state = "live"    # live | dropping (queue full) | awaiting_key (resync requested)
        self.frames_dropped = 0

    async def _write(self):
        try:
            while True:
                msg = await self.out.get()
                if msg is None:
                    break
                if isinstance(msg, _VideoFrame):
                    for m in msg.msgs:
                        await self.ws.send_bytes(m)
                        self.meter.add(len(m))
                    self.video_queued -= 1
                    if self.video_state == "dropping" and self.video_queued == 0:
                        self.video_state = "awaiting_key"
                        if self.on_resync is not None:
                            self.on_resync(self)
                    continue
                if isinstance(msg, (bytes, bytearray)):
                    await self.ws.send_bytes(msg)
                else:
                    await self.ws.send_str(msg)
                self.meter.add(len(msg))
        except (ConnectionError, RuntimeError, asyncio.CancelledError):
            pass
        finally:
            self.closed = True

    def send(self, msg) -> bool:
        if self.closed or self.ws.closed:
            return False
        self.out.put_nowait(msg)
        return True

    def send_video(self, msgs: list, key: bool, independent: bool = False) -> bool:
        """Queues one frame's stripe messages; False if this viewer dropped it.

        ``independent``: every message decodes on its own (JPEG stripes), so a
        dropped frame needs no keyframe to recover from.
        """
        if self.closed or self.ws.closed:
            return False
        if self.video_state == "awaiting_key":
            if not (key or independent):
                self.frames_dropped += 1
                return False
            self.video_state = "live"
        if self.video_state == "dropping" or self.video_queued >= self.MAX_VIDEO_FRAMES:
            if self.video_state == "live":
                log.warning("viewer %s is %d frames behind: dropping video until it drains",
                            self.remote, self.video_queued)
                self.video_state = "live" if independent else "dropping"
            self.frames_dropped += 1
            return False
        self.video_queued += 1
        self.out.put_nowait(_VideoFrame(msgs, key))
        return True

    async def send_now(self, msg) -> bool:
        return self.send(msg)

    async def close(self, code: int = 1000, reason: str = ""):
        self.out.put_nowait(None)
        try:
            await asyncio.wait_for(self.writer, 2.0)
        except (asyncio.TimeoutError, asyncio.CancelledError):
            self.writer.cancel()
        if not self.ws.closed:
            await self.ws.close(code=code, message=reason.encode())


@dataclass
class DisplayState:
    client: Client
    width: int = 0
    height: int = 0
    position: str = "right"
    video_active: bool = True
    flow: protocol.DisplayFlow = field(default_factory=protocol.DisplayFlow)
    params: dict = field(default_factory=dict)
    bp_task: Optional[asyncio.Task] = None
    scaling_dpi: Optional[Any] = None
    audio_bitrate: Optional[Any] = None


class Capture:
    """One display's capture session + queue + sender task."""

    def __init__(self, display_id: str, module, queue: asyncio.Queue, sender: asyncio.Task):
        self.display_id, self.module, self.queue, self.sender = display_id, module, queue, sender
        self.callback = None
        self.size, self.fps = (0, 0), 60.0


def files_listing_html(path: str, rel: str) -> str:
    """HTML listing of one directory of the download area: sub-directories first,
    then files with their sizes; names are escaped and links percent-encoded."""
    rows = []
    if rel.strip("/"):
        rows.append('<li><a href="../">../</a></li>')
    try:
        entries = sorted((e for e in os.scandir(path) if not e.name.startswith(".")),
                         key=lambda e: (not e.is_dir(), e.name.lower()))
    except OSError:
        entries = []
    for e in entries:
        d = e.is_dir()
        size = "" if d else f" <small>{e.stat().st_size:,} B</small>"
        rows.append(f'<li><a href="{urllib.parse.quote(e.name)}{"/" if d else ""}">'
                    f'{html.escape(e.name)}{"/" if d else ""}</a>{size}</li>')
    title = html.escape("/" + rel.strip("/"))
    return ("<!DOCTYPE html><html><head><meta charset=\"utf-8\"><title>Files " + title + "</title>"
            "<style>body{font:13px system-ui,sans-serif;margin:12px}li{margin:3px 0}</style></head>"
            "<body><h3>Files " + title + "</h3><ul>" + "".join(rows) + "</ul></body></html>")


def _basic_auth_ok(request, user: str, password: str) -> bool:
    h = request.headers.get("Authorization", "")
    if not h.startswith("Basic "):
        return False
    try:
        got = base64.b64decode(h[6:].strip(), validate=True)
    except (ValueError, binascii.Error):
        return False
    return hmac.compare_digest(got, f"{user}:{password}".encode())


class DataStreamingServer:
    def __init__(self, settings: Settings, *, upload_dir: Optional[str] = None, download_dir: Optional[str] = None,
                 input_factory=None,
                 capture_factory: Optional[Callable[[], Any]] = None, display_manager=None,
                 capture_source: str = "auto", gpu_id: int = 0, num_gpus: int = 1, clock=time.monotonic,
                 web_root: Optional[str] = None, metrics=None, frame_trace: Optional[bool] = None,
                 x_display: Optional[str] = None, basic_auth: Optional[tuple] = None,
                 control_token: Optional[str] = None):
        self.settings = settings
        # node control API (/api/placement, /api/move; parallel/rebalance.py): answered only
        # to direct loopback callers that present the launcher's token. Without a token the
        # API is off: behind a reverse proxy every client arrives from 127.0.0.1, so the
        # peer address alone proves nothing (deploy/nginx.conf also denies /api/).
        self.control_token = (control_token if control_token is not None
                              else os.environ.get("SELKIES_CONTROL_TOKEN")) or None
        # (user, password) guarding every route, the websocket upgrade included: the
        # reference puts its whole nginx server block, /ws too, behind basic auth
        # (addons/example/selkies-gstreamer-entrypoint.sh:89) and its signalling server
        # refuses an empty password (legacy/signalling_web.py:157-159). /health stays
        # open for container liveness probes.
        if basic_auth is not None and not basic_auth[1]:
            raise ValueError("basic auth is enabled but the password is empty "
                             "(set SELKIES_BASIC_AUTH_PASSWORD)")
        self.basic_auth = basic_auth
        # this session's X display, passed explicitly to capture, xrandr, DPI and
        # the WM swap: a session host runs several servers in one process, so the
        # process-wide DISPLAY cannot name each session's desktop (parallel/multi.py)
        self.x_display = x_display if x_display is not None else os.environ.get("DISPLAY")
        self.clock = clock
        self.frame_trace = (os.environ.get("SELKIES_FRAME_TRACE") == "1") if frame_trace is None else frame_trace
        self.mode = "websockets"
        self.clients: set[Client] = set()
        self.displays: "OrderedDict[str, DisplayState]" = OrderedDict()
        self.layouts: dict = {}
        self.captures: dict[str, Capture] = {}
        self._resync: set[str] = set()     # displays whose queue overflowed: wait for a keyframe
        self._key_requested: dict = {}     # display -> time of the last REQUEST_KEYFRAME served
        self.meter = BandwidthMeter(clock)
        self.recent: "OrderedDict[str, float]" = OrderedDict()
        self.reconfigure_lock = asyncio.Lock()
        self._reconfiguring = False
        self._reconfigure_pending = False
        self.settings_received = asyncio.Event()
        self.capture_cursor = False
        self.last_cursor: Optional[dict] = None
        self.download_dir = download_dir   # served read-only under /files/ (dashboard files panel)
        self.upload_dir = upload_dir
        if upload_dir:
            try:
                os.makedirs(upload_dir, exist_ok=True)
            except OSError as e:
                log.error("upload dir %s unusable: %s", upload_dir, e)
                self.upload_dir = None
        self.input_factory = input_factory
        self.input = None
        if capture_factory is None:
            import pixelflux
            capture_factory = pixelflux.ScreenCapture
        self.capture_factory = capture_factory
        self.display_manager = display_manager or XrandrDisplay(self.x_display)
        self.wm_swap = (WindowManagerSwap(display=self.x_display)
                        if getattr(self.display_manager, "available", False) else None)
        self.capture_source = capture_source
        self.gpu_id, self.num_gpus = gpu_id, max(1, num_gpus)
        self._gpu_of: dict = {}   # display -> GPU after a move (/api/move)
        self.web_root = web_root
        self.metrics = metrics
        self.audio = AudioPipeline(self._broadcast_audio, settings.audio_device_name,
                                   debug=settings.debug[0])
        self.audio_bitrate = int(settings.initial("audio_bitrate"))
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.runner: Optional[web.AppRunner] = None
        self.encoder = settings.encoder
        self.framerate = settings.initial("framerate")

    # ================================================================ app / routes
    AUTH_EXEMPT = ("/health",)
    KEY_REQUEST_MIN_S = 0.2

    @web.middleware
    async def _auth_middleware(self, request: web.Request, handler):
        # /api/* carries its own (stronger) token check instead of the viewers' password
        if (self.basic_auth is not None and request.path not in self.AUTH_EXEMPT
                and not request.path.startswith("/api/")
                and not _basic_auth_ok(request, *self.basic_auth)):
            raise web.HTTPUnauthorized(headers={"WWW-Authenticate": 'Basic realm="selkies"'})
        return await handler(request)

    def make_app(self) -> web.Application:
        app = web.Application(client_max_size=64 * 1024 * 1024, middlewares=[self._auth_middleware])
        app.router.add_get("/health", self._health)
        if self.metrics is not None:
            app.router.add_get("/metrics", self.metrics.handler)
        app.router.add_get("/api/placement", self._api_placement)
        app.router.add_post("/api/move", self._api_move)
        app.router.add_get("/files", self._files_redirect)
        app.router.add_get("/files/{name:.*}", self._files)
        app.router.add_get("/{tail:.*}", self._root)
        return app

    async def _files_redirect(self, request):
        raise web.HTTPFound("/files/")

    async def _files(self, request: web.Request):
        """Read-only listing / download of the file directory (the dashboard's files
        panel frames ./files/; reference: Sidebar.jsx:3523 iframe on the same path).
        Dot files are hidden; nothing outside the directory is reachable."""
        root = self.download_dir
        if not root or not os.path.isdir(root):
            raise web.HTTPNotFound()
        rel = request.match_info.get("name", "")
        base = os.path.realpath(root)
        path = os.path.realpath(os.path.join(base, rel))
        if not (path == base or path.startswith(base + os.sep)):
            raise web.HTTPNotFound()
        if any(part.startswith(".") for part in os.path.relpath(path, base).split(os.sep) if part not in ("", ".")):
            raise web.HTTPNotFound()
        if os.path.isdir(path):
            if rel and not rel.endswith("/"):
                raise web.HTTPFound(request.path + "/")
            return web.Response(text=files_listing_html(path, rel), content_type="text/html")
        if os.path.isfile(path):
            name = os.path.basename(path)
            return web.FileResponse(path, headers={
                "Content-Disposition": f"attachment; filename*=UTF-8''{urllib.parse.quote(name)}"})
        raise web.HTTPNotFound()

    async def _health(self, request):
        return web.Response(text="OK\n")

    # ---- node control (parallel/rebalance.py): direct loopback callers with the token
    CONTROL_HEADER = "X-Selkies-Control-Token"
    PROXY_HEADERS = ("X-Forwarded-For", "X-Real-IP", "Forwarded")

    def _control_ok(self, request: web.Request) -> bool:
        if not self.control_token:
            return False
        if (request.remote or "") not in ("127.0.0.1", "::1", "::ffff:127.0.0.1"):
            return False
        if any(h in request.headers for h in self.PROXY_HEADERS):   # relayed by a proxy
            return False
        return hmac.compare_digest(request.headers.get(self.CONTROL_HEADER, "").encode(),
                                   self.control_token.encode())

    def placement(self) -> dict:
        """Per display: the GPU its encoder runs on and its encode load (mean and last
        capture-to-packets ms, frames, target fps)."""
        out = {}
        for did, cap in self.captures.items():
            mod = cap.module
            st = {}
            try:
                st = mod.stats()
            except Exception:
                pass
            dev = getattr(mod, "device", None)
            out[did] = {"gpu": dev if isinstance(dev, int) and dev >= 0 else self._gpu_of.get(did),
                        "encode_ms_mean": st.get("encode_ms_mean"), "encode_ms_last": st.get("encode_ms_last"),
                        "frames": st.get("frames"), "fps": cap.fps, "move_stall_ms": st.get("move_stall_ms"),
                        "width": cap.size[0], "height": cap.size[1]}
        return out

    async def _api_placement(self, request):
        if not self._control_ok(request):
            raise web.HTTPForbidden()
        return web.json_response({"gpu_id": self.gpu_id, "displays": self.placement()})

    async def move_display(self, did: str, gpu: int) -> str:
        """Moves display `did`'s running encoder to GPU `gpu` (P-frame continuation when
        the state can be carried, pixelflux ScreenCapture.move_to); later capture restarts
        of the display (resolution changes) stay on that GPU."""
        cap = self.captures.get(did)
        if cap is None:
            raise KeyError(did)
        fn = getattr(cap.module, "move_to", None)
        if fn is None:
            raise RuntimeError("capture module cannot move")
        res = await asyncio.get_running_loop().run_in_executor(None, fn, int(gpu))
        self._gpu_of[did] = int(gpu)   # "keyframe": the new stream opens with an IDR itself
        log.info("display %s moved to GPU %d (%s)", did, gpu, res)
        return res

    async def _api_move(self, request):
        if not self._control_ok(request):
            raise web.HTTPForbidden()
        did = request.query.get("display", "primary")
        try:
            gpu = int(request.query["gpu"])
        except (KeyError, ValueError):
            raise web.HTTPBadRequest(text="gpu=<index> required")
        try:
            res = await self.move_display(did, gpu)
        except KeyError:
            raise web.HTTPNotFound(text=f"no running capture for display {did}")
        except RuntimeError as e:
            return web.json_response({"display": did, "gpu": gpu, "error": str(e)}, status=409)
        return web.json_response({"display": did, "gpu": gpu, "result": res})

    async def _root(self, request: web.Request):
        if request.headers.get("Upgrade", "").lower() == "websocket":
            return await self.ws_handler(request)
        if self.web_root:
            rel = request.match_info.get("tail", "") or "index.html"
            path = os.path.realpath(os.path.join(self.web_root, rel))
            root = os.path.realpath(self.web_root)
            if path.startswith(root + os.sep) or path == root:
                if os.path.isdir(path):
                    path = os.path.join(path, "index.html")
                if os.path.isfile(path):
                    return web.FileResponse(path)
        raise web.HTTPNotFound()

    async def start(self, host: str = "0.0.0.0", port: Optional[int] = None):
        self.loop = asyncio.get_running_loop()
        self.runner = web.AppRunner(self.make_app())
        await self.runner.setup()
        site = web.TCPSite(self.runner, host, port if port is not None else self.settings.port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        if self.input_factory is not None:
            self.input = await self.input_factory(self)
        log.info("data websocket server on %s:%d", host, self.port)
        return self.port

    async def stop(self):
        for c in list(self.clients):
            await c.close(1001, "server shutdown")
        async with self.reconfigure_lock:
            await self.shutdown_pipelines()
        if self.input is not None:
            await self.input.close()
        if self.runner:
            await self.runner.cleanup()

    # ================================================================ broadcast helpers
    def broadcast(self, clients, msg):
        for c in list(clients):
            c.send(msg)

    def _resync_viewer(self, client: "Client"):
        """A viewer that dropped frames has drained its queue: keyframe on its display."""
        did = client.display_id if client.display_id in self.captures else "primary"
        cap = self.captures.get(did)
        if cap is not None and hasattr(cap.module, "request_keyframe"):
            cap.module.request_keyframe()

    def primary_viewers(self) -> set:
        secondary = {d.client for did, d in self.displays.items() if did != "primary"}
        return self.clients - secondary

    async def _broadcast_audio(self, data: bytes):
        self.broadcast(self.primary_viewers(), data)

    def send_cursor(self, msg: dict):
        """Thread-safe: cursor watcher thread -> all clients."""
        self.last_cursor = msg
        if self.loop is not None:
            self.loop.call_soon_threadsafe(self.broadcast, self.clients, "cursor," + json.dumps(msg))

    async def send_clipboard(self, data: bytes, mime: str = "text/plain"):
        if mime != "text/plain" and not (self.input and self.input.enable_binary_clipboard):
            return
        for m in protocol.clipboard_messages(data, mime):
            self.broadcast(self.clients, m)
            await asyncio.sleep(0)

    # ================================================================ websocket handler
    async def ws_handler(self, request: web.Request):
        ip = request.remote or "?"
        now = self.clock()
        last = self.recent.get(ip)
        ws = web.WebSocketResponse(max_msg_size=64 * 1024 * 1024, heartbeat=None, compress=False)
        await ws.prepare(request)
        if last is not None and (now - last) < RECONNECT_DEBOUNCE_S:
            log.warning("client %s reconnecting too quickly; rejected", ip)
            await ws.close(code=4029, message=b"Rate limited: reconnecting too quickly")
            return ws
        self.recent[ip] = now
        if len(self.recent) > 1000:
            self.recent.popitem(last=False)
        client = Client(ws, ip, self.meter, on_resync=self._resync_viewer)
        self.clients.add(client)
        self.settings_received = asyncio.Event() if not self.displays else self.settings_received
        initial_done = False
        uploads = _UploadState(self.upload_dir)
        mic = MicSink()
        stats = StatsPublisher(client.send_now, self.meter, self._primary_rtt, gpu_id=self.gpu_id)
        client.send(f"MODE {self.mode}")
        if self.last_cursor:
            client.send("cursor," + json.dumps(self.last_cursor))
        client.send(json.dumps(self.settings.client_payload()))
        stats.start()
        try:
            async for msg in ws:
                if msg.type == WSMsgType.BINARY:
                    await self._on_binary(msg.data, uploads, mic)
                elif msg.type == WSMsgType.TEXT:
                    initial_done = await self._on_text(client, msg.data, uploads, initial_done)
                    if client.closed or ws.closed:
                        break
                elif msg.type in (WSMsgType.ERROR, WSMsgType.CLOSE):
                    break
        except asyncio.CancelledError:
            raise
        except Exception as e:  # keep the server alive whatever one client does
            log.error("error in data websocket handler for %s: %s", ip, e, exc_info=True)
        finally:
            await stats.cancel()
            uploads.abort()
            mic.close()
            await self._disconnect(client)
        return ws

    async def _disconnect(self, client: Client):
        self.clients.discard(client)
        gone = [did for did, d in self.displays.items() if d.client is client]
        for did in gone:
            await self._stop_bp(did)
            del self.displays[did]
        if gone:
            await self.reconfigure_displays()
        await client.close()
        if not self.clients:
            self.capture_cursor = False
            async with self.reconfigure_lock:
                await self.shutdown_pipelines()

    async def shutdown_pipelines(self):
        for did in list(self.captures):
            await self._stop_capture(did)
        await self.audio.stop()

    # ---------------------------------------------------------------- binary
    async def _on_binary(self, data: bytes, uploads: "_UploadState", mic: MicSink):
        if not data:
            return
        kind, payload = data[0], data[1:]
        if kind == 0x01:
            uploads.write(payload)
        elif kind == 0x02:
            if not self.settings.microphone_enabled[0]:
                return
            if await mic.setup():
                mic.push(payload)

    # ---------------------------------------------------------------- text
    async def _on_text(self, client: Client, m: str, uploads: "_UploadState", initial_done: bool) -> bool:
        s = self.settings
        if m.startswith("FILE_UPLOAD_START:"):
            if "upload" not in s.file_transfers:
                log.warning("upload refused: uploads disabled")
            else:
                uploads.start(m)
        elif m.startswith("FILE_UPLOAD_END:"):
            uploads.finish()
        elif m.startswith("FILE_UPLOAD_ERROR:"):
            log.error("client upload error: %s", m)
            uploads.abort()
        elif m.startswith("SETTINGS,"):
            initial_done = await self._on_settings(client, m[len("SETTINGS,"):], initial_done)
        elif m.startswith("CLIENT_FRAME_ACK"):
            did = client.display_id
            if did and did in self.displays:
                try:
                    self.displays[did].flow.on_ack(protocol.parse_frame_ack(m), self.clock())
                except ValueError:
                    log.warning("malformed ACK: %s", m)
        elif m == "REQUEST_KEYFRAME":
            # a viewer's decoder lost its reference (web/lib/video.js drops deltas when it
            # falls behind): the display's next frame is a key frame; one request per
            # KEY_REQUEST_MIN_S per display, however many viewers ask
            did = client.display_id
            cap = self.captures.get(did) if did else None
            now = self.clock()
            if cap is not None and hasattr(cap.module, "request_keyframe") and \
                    now - self._key_requested.get(did, -1e9) >= self.KEY_REQUEST_MIN_S:
                self._key_requested[did] = now
                cap.module.request_keyframe()
        elif m == "START_VIDEO":
            await self._start_video(client)
        elif m == "STOP_VIDEO":
            did = client.display_id
            if did and did in self.displays:
                self.displays[did].video_active = False
                await self._stop_capture(did)
                client.send("VIDEO_STOPPED")
        elif m == "START_AUDIO":
            async with self.reconfigure_lock:
                if s.audio_enabled[0]:
                    await self.audio.start(self.audio_bitrate)
                self.broadcast(self.clients, "AUDIO_STARTED")
        elif m == "STOP_AUDIO":
            async with self.reconfigure_lock:
                await self.audio.stop()
                self.broadcast(self.clients, "AUDIO_STOPPED")
        elif m.startswith("r,"):
            await self._on_resize(m)
        elif m.startswith("SET_NATIVE_CURSOR_RENDERING,"):
            want = m.split(",", 1)[1].strip().lower() in ("1", "true")
            if want != self.capture_cursor:
                self.capture_cursor = want
                if self.captures:
                    await self.reconfigure_displays()
        elif m.startswith("s,"):
            try:
                dpi = int(m.split(",")[1])
            except (ValueError, IndexError):
                log.error("malformed DPI message %s", m)
            else:
                await set_dpi(dpi, display=self.x_display)
                await set_cursor_size(max(1, round(dpi / 96.0 * CURSOR_SIZE)), display=self.x_display)
        elif m.startswith("cmd,"):
            if not s.command_enabled[0]:
                log.warning("cmd refused: commands disabled")
            else:
                cmd = m[len("cmd,"):]
                if cmd:
                    try:
                        p = await asyncio.create_subprocess_shell(cmd, stdout=asyncio.subprocess.DEVNULL,
                                                                  stderr=asyncio.subprocess.DEVNULL,
                                                                  cwd=os.path.expanduser("~"),
                                                                  env=display_env(self.x_display))
                        log.info("launched '%s' (pid %d)", cmd, p.pid)
                    except OSError as e:
                        log.error("cmd failed: %s", e)
        elif self.input is not None:
            await self.input.on_message(m, client.display_id or "primary")
        return initial_done

    # ---------------------------------------------------------------- SETTINGS
    async def _on_settings(self, client: Client, payload: str, initial_done: bool) -> bool:
        try:
            parsed = protocol.parse_settings_payload(payload)
        except (ValueError, TypeError) as e:
            log.error("bad SETTINGS payload: %s", e)
            return initial_done
        did = parsed.get("displayId") or "primary"
        if did != "primary" and not self.settings.second_screen[0]:
            client.send("KILL Second screens are disabled on this server.")
            await client.close(1008, "Second screens disabled")
            return initial_done
        client.display_id = did
        existing = self.displays.get(did)
        if existing is not None and existing.client is not client and not existing.client.closed:
            reason = f"a new {did} client connected connection killed"
            existing.client.send(f"KILL {reason}")
            await existing.client.close(1000, "Superseded by new client")
        if did != "primary":
            for other, st in list(self.displays.items()):
                if other != "primary" and other != did and st.client is not client:
                    await self._stop_capture(other)
                    st.video_active = False
                    st.client.send("VIDEO_STOPPED")
        if did not in self.displays:
            self.displays[did] = DisplayState(client=client, params=self._initial_params())
        else:
            st = self.displays[did]
            st.client = client
            st.video_active = True
            st.flow.reset(self.clock())
        await self.apply_client_settings(did, parsed, not initial_done)
        if not initial_done:
            initial_done = True
            if did == "primary" and self.settings.audio_enabled[0] and not self.audio.running:
                async with self.reconfigure_lock:
                    await self.audio.start(self.audio_bitrate)
        return initial_done

    def _initial_params(self) -> dict:
        s = self.settings
        return {"encoder": s.encoder, "framerate": s.initial("framerate"), "h264_crf": s.initial("h264_crf"),
                "h264_fullcolor": s.initial("h264_fullcolor"),
                "h264_streaming_mode": s.initial("h264_streaming_mode"),
                "jpeg_quality": s.initial("jpeg_quality"),
                "paint_over_jpeg_quality": s.initial("paint_over_jpeg_quality"), "use_cpu": s.initial("use_cpu"),
                "h264_paintover_crf": s.initial("h264_paintover_crf"),
                "h264_paintover_burst_frames": s.initial("h264_paintover_burst_frames"),
                "use_paint_over_quality": s.initial("use_paint_over_quality"),
                "h264_bitrate": s.initial("h264_bitrate")}

    async def apply_client_settings(self, did: str, parsed: dict, initial: bool):
        st = self.displays.get(did)
        if st is None:
            return
        s = self.settings
        restart_audio = False
        async with self.reconfigure_lock:
            old = dict(st.params)
            old_w, old_h, old_pos = st.width, st.height, st.position
            new_pos = parsed.get("displayPosition") or "right"
            tw = th = None
            if s.is_manual_resolution_mode[0] and s.is_manual_resolution_mode[1]:
                tw, th = int(s.manual_width), int(s.manual_height)
            elif s.sanitize("is_manual_resolution_mode", parsed.get("is_manual_resolution_mode")):
                tw = s.sanitize("manual_width", parsed.get("manual_width"))
                th = s.sanitize("manual_height", parsed.get("manual_height"))
            elif initial:
                tw, th = parsed.get("initialClientWidth"), parsed.get("initialClientHeight")
            if not isinstance(tw, int) or tw <= 0:
                tw = old_w if old_w > 0 else 1024
            if not isinstance(th, int) or th <= 0:
                th = old_h if old_h > 0 else 768
            tw, th = protocol.even_dims(tw, th)
            dims_changed = (tw, th) != (old_w, old_h) or new_pos != old_pos
            st.width, st.height, st.position = tw, th, new_pos
            for k in VIDEO_KEYS:
                st.params[k] = s.sanitize(k, parsed.get(k))
            bitrate = s.sanitize("audio_bitrate", parsed.get("audio_bitrate"))
            if bitrate is not None and int(bitrate) != self.audio_bitrate:
                self.audio_bitrate = int(bitrate)
                restart_audio = self.audio.running
            if self.input is not None:
                await self.input.update_binary_clipboard_setting(
                    bool(s.sanitize("enable_binary_clipboard", parsed.get("enable_binary_clipboard"))))
            dpi = s.sanitize("scaling_dpi", parsed.get("scaling_dpi"))
            if dpi is not None and dpi != st.scaling_dpi:
                if st.scaling_dpi is not None or initial:
                    await set_dpi(int(dpi), display=self.x_display)
                st.scaling_dpi = dpi
            changed = {k for k in VIDEO_KEYS if st.params.get(k) != old.get(k)}
            video_changed = bool(changed)
            if changed == {"h264_bitrate"} and did in self.captures and not initial:
                # K10 rate change: applied to the running encoder from its next frame
                self._set_rate(did, int(st.params.get("h264_bitrate") or 0))
                video_changed = False
        if restart_audio:
            await self.audio.stop()
            await self.audio.start(self.audio_bitrate)
        if initial or dims_changed:
            await self.reconfigure_displays()
        elif video_changed:
            if did in self.layouts:
                l = self.layouts[did]
                await self._stop_capture(did)
                await self._start_capture(did, l["w"], l["h"], l["x"], l["y"])
            else:
                await self.reconfigure_displays()
        if initial:
            self.settings_received.set()

    # ---------------------------------------------------------------- resize / video
    async def _on_resize(self, m: str):
        parts = m.split(",")
        if len(parts) != 3:
            log.warning("malformed resize: %s", m)
            return
        _, res, did = parts
        st = self.displays.get(did)
        if st is None:
            return
        if self.settings.is_manual_resolution_mode[0] and self.settings.is_manual_resolution_mode[1]:
            log.warning("resize ignored: manual resolution mode")
            return
        try:
            w, h = protocol.even_dims(*protocol.parse_resolution(res))
        except ValueError:
            log.error("invalid resolution %s", res)
            return
        if w <= 0 or h <= 0 or (w, h) == (st.width, st.height):
            return
        st.width, st.height = w, h
        await self.reconfigure_displays()

    async def _start_video(self, client: Client):
        did = client.display_id
        if did and did in self.displays:
            st = self.displays[did]
            st.video_active = True
            if did in self.layouts:
                l = self.layouts[did]
                await self._start_capture(did, l["w"], l["h"], l["x"], l["y"])
            else:
                await self.reconfigure_displays()
            client.send("VIDEO_STARTED")
        else:
            await self.reconfigure_displays()

    async def reconfigure_displays(self):
        """Lays out all displays and (re)starts their captures.

        Requests arriving while a reconfiguration runs are coalesced into one
        more pass (the reference drops them, which can leave a just-connected
        secondary display without a stream).
        """
        if self._reconfiguring:
            self._reconfigure_pending = True
            return
        self._reconfiguring = True
        try:
            async with self.reconfigure_lock:
                while True:
                    self._reconfigure_pending = False
                    await self._reconfigure_once()
                    if not self._reconfigure_pending:
                        break
        finally:
            self._reconfiguring = False

    async def _reconfigure_once(self):
        for did in list(self.captures):
            await self._stop_capture(did)
        if not self.displays:
            await self.display_manager.clear()
            return
        layouts, tw, th = compute_layout({k: {"width": v.width, "height": v.height, "position": v.position}
                                          for k, v in self.displays.items()})
        if not tw or not th:
            log.error("display layout is empty; not starting capture")
            return
        self.layouts = layouts
        if self.wm_swap is not None:
            await self.wm_swap.update(len(self.displays))
        if getattr(self.display_manager, "available", False):
            ok = await self.display_manager.apply(layouts, tw, th)
            if not ok:
                log.warning("xrandr layout failed; capturing the current screen")
        for did, l in layouts.items():
            st = self.displays.get(did)
            if st and st.video_active:
                await self._start_capture(did, l["w"], l["h"], l["x"], l["y"])
        p = self.displays.get("primary")
        if p and p.width and p.height:
            self.broadcast(self.clients, protocol.stream_resolution_message(p.width, p.height))
        self.broadcast(self.clients, protocol.display_config_message(list(self.displays)))

    # ---------------------------------------------------------------- capture
    def capture_settings(self, did: str, w: int, h: int, x: int, y: int):
        import pixelflux
        st = self.displays[did]
        p = st.params
        enc = p.get("encoder") or self.settings.encoder
        cs = pixelflux.default_settings(w, h)
        cs.capture_x, cs.capture_y = x, y
        cs.target_fps = float(p.get("framerate") or 60)
        cs.capture_cursor = int(self.capture_cursor)
        if self.x_display:
            cs.display = self.x_display.encode()
        cs.debug_logging = int(self.settings.debug[0])
        if enc == "jpeg":
            cs.output_mode = 0
            cs.jpeg_quality = int(p["jpeg_quality"])
            cs.paint_over_jpeg_quality = int(p["paint_over_jpeg_quality"])
            cs.stripe_height = 64
        else:
            # H.264 (striped or full frame), HEVC (x265enc) or AV1 (svtav1enc): the same
            # front end, rate control and packet framing (type 0x04 + 10-byte stripe header);
            # the client picks its WebCodecs codec from the negotiated encoder
            cs.output_mode = {"x265enc": 2, "svtav1enc": 3}.get(enc, 1)
            cs.h264_crf = int(p["h264_crf"])
            kbps = int(p.get("h264_bitrate") or 0)   # K10: CRF, or CBR at kbps
            cs.h264_rc_mode, cs.h264_bitrate_kbps = (2, kbps) if kbps > 0 else (1, 0)
            cs.h264_paintover_crf = int(p["h264_paintover_crf"])
            cs.h264_paintover_burst_frames = int(p["h264_paintover_burst_frames"])
            cs.h264_fullcolor = int(bool(p["h264_fullcolor"]))
            cs.h264_streaming_mode = int(bool(p["h264_streaming_mode"]))
            cs.h264_fullframe = int(enc in ("x264enc", "x265enc", "svtav1enc"))
            cs.h264_aq_strength = max(0, min(64, int(self.settings.h264_aq_strength)))
            cs.h264_subpel = 0 if self.settings.h264_subpel[0] else -1
            cs.h264_intra4x4 = int(bool(self.settings.h264_intra4x4[0]))
        cs.use_paint_over_quality = int(bool(p["use_paint_over_quality"]))
        cs.paint_over_trigger_frames, cs.damage_block_threshold, cs.damage_block_duration = 15, 10, 20
        cs.use_cpu = int(bool(p["use_cpu"]))
        index = list(self.displays).index(did)
        cs.device = self._gpu_of.get(did, (self.gpu_id + index) % self.num_gpus)
        cs.source = {"auto": -1, "x11": 0, "synthetic": 2, "motion": 1, "noise": 3}.get(self.capture_source, -1)
        wm = self.settings.watermark_path
        if wm and os.path.exists(wm):
            cs.watermark_path = wm.encode()
            cs.watermark_location_enum = int(self.settings.watermark_location)
        return cs, enc

    async def _start_capture(self, did: str, w: int, h: int, x: int, y: int):
        if did in self.captures:
            return
        try:
            cs, enc = self.capture_settings(did, w, h, x, y)
        except KeyError:
            return
        loop = asyncio.get_running_loop()
        queue: asyncio.Queue = asyncio.Queue(maxsize=VIDEO_QUEUE_SIZE)
        jpeg = enc == "jpeg"
        self._resync.discard(did)

        def on_frame(res_ptr, n, user):
            # one call per encoded frame (native capture thread): copy every stripe out
            msgs = []
            key = False
            fid = 0
            grab = 0
            for i in range(n):
                r = res_ptr[i]
                if r.size <= 0:
                    continue
                data = ctypes.string_at(r.data, r.size)
                key = key or (not jpeg and r.size > 1 and data[1] == 1)
                fid = r.frame_id & 0xFFFF
                grab = r.grab_ns
                msgs.append(protocol.JPEG_PREFIX + data if jpeg else data)
            if msgs:
                loop.call_soon_threadsafe(self._put_frame, did, queue, (msgs, key, fid, grab), jpeg)

        def on_stripe(res_ptr, user):   # capture modules without a per-frame callback
            r = res_ptr.contents
            if r.size <= 0:
                return
            data = ctypes.string_at(r.data, r.size)
            key = not jpeg and r.size > 1 and data[1] == 1
            item = ([protocol.JPEG_PREFIX + data if jpeg else data], key, r.frame_id & 0xFFFF, r.grab_ns)
            loop.call_soon_threadsafe(self._put_frame, did, queue, item, jpeg)

        import pixelflux
        module = self.capture_factory()
        if hasattr(module, "start_frame_capture"):
            cb = pixelflux.FrameCallback(on_frame)
            start = module.start_frame_capture
        else:
            cb = pixelflux.StripeCallback(on_stripe)
            start = module.start_capture
        sender = asyncio.create_task(self._video_sender(did, queue))
        try:
            await loop.run_in_executor(None, start, cs, cb)
        except Exception as e:
            sender.cancel()
            log.error("capture start failed for %s: %s", did, e)
            return
        cap = Capture(did, module, queue, sender)
        cap.size, cap.fps = (int(cs.capture_width), int(cs.capture_height)), float(cs.target_fps)
        cap.callback = cb
        self.captures[did] = cap
        st = self.displays.get(did)
        if st is not None:
            st.flow.reset(self.clock())
            await self._start_bp(did)
        if self.metrics is not None:
            self.metrics.capture_started(did, module)

    def _set_rate(self, did: str, kbps: int) -> None:
        """K10: CRF (kbps 0) or CBR at kbps on the display's running encoder."""
        cap = self.captures.get(did)
        fn = getattr(getattr(cap, "module", None), "set_rate", None)
        if fn is not None:
            fn("cbr" if kbps > 0 else "crf", kbps)

    async def _stop_capture(self, did: str):
        await self._stop_bp(did)
        cap = self.captures.pop(did, None)
        if cap is None:
            return
        try:
            await asyncio.get_running_loop().run_in_executor(None, cap.module.stop_capture)
        except Exception as e:
            log.error("stop_capture failed for %s: %s", did, e)
        cap.sender.cancel()
        try:
            await cap.sender
        except (asyncio.CancelledError, Exception):
            pass
        if self.metrics is not None:
            self.metrics.capture_stopped(did)

    def _put_frame(self, did: str, queue: asyncio.Queue, item, jpeg: bool) -> None:
        """Native thread -> event loop hand-off of one encoded frame (runs on the loop).

        A full queue drops the frame for every viewer. JPEG stripes stand alone,
        but an H.264 frame is a reference for the next ones: after a drop no
        P frame is queued until the keyframe requested here arrives, so decoders
        never see a broken reference chain."""
        if did in self._resync:
            if not item[1]:
                return
            self._resync.discard(did)
        try:
            queue.put_nowait(item)
        except asyncio.QueueFull:
            if jpeg:
                return
            self._resync.add(did)
            cap = self.captures.get(did)
            if cap is not None and hasattr(cap.module, "request_keyframe"):
                cap.module.request_keyframe()
            if self.metrics is not None and hasattr(self.metrics, "frame_dropped"):
                self.metrics.frame_dropped(did)

    async def _video_sender(self, did: str, queue: asyncio.Queue):
        was_enabled = True
        jpeg = None
        while True:
            msgs, key, fid, grab_ns = await queue.get()
            st = self.displays.get(did)
            if st is None:
                continue
            if not st.flow.enabled:
                was_enabled = False
                continue
            if not was_enabled:
                # frames were skipped while backpressured: resynchronise decoders
                was_enabled = True
                cap = self.captures.get(did)
                if cap is not None and hasattr(cap.module, "request_keyframe"):
                    cap.module.request_keyframe()
            st.flow.on_sent(fid, self.clock())
            viewers = self.primary_viewers() if did == "primary" else {st.client}
            jpeg = msgs[0][:2] == protocol.JPEG_PREFIX
            if self.frame_trace:
                # latency tracing (SELKIES_FRAME_TRACE=1): the frame's grab time (CLOCK_MONOTONIC ns)
                # ahead of its stripes, so a client on the same host measures capture -> receive
                trace = f"FRAME_TS {fid} {grab_ns}"
                for c in list(viewers):
                    c.send(trace)
            for c in list(viewers):
                c.send_video(msgs, key, independent=jpeg)

    # ---------------------------------------------------------------- backpressure
    async def _start_bp(self, did: str):
        await self._stop_bp(did)
        st = self.displays.get(did)
        if st is not None:
            st.bp_task = asyncio.create_task(self._bp_loop(did))

    async def _stop_bp(self, did: str):
        st = self.displays.get(did)
        if st is None or st.bp_task is None:
            return
        t, st.bp_task = st.bp_task, None
        t.cancel()
        try:
            await t
        except (asyncio.CancelledError, Exception):
            pass
        st.flow.reset(self.clock())
        msg = f"PIPELINE_RESETTING {did}"
        if did == "primary":
            self.broadcast(self.clients, msg)
        else:
            st.client.send(msg)

    async def _bp_loop(self, did: str):
        await self.settings_received.wait()
        while True:
            await asyncio.sleep(protocol.CHECK_INTERVAL_S)
            st = self.displays.get(did)
            if st is None:
                return
            before = st.flow.enabled
            after = st.flow.evaluate(self.clock(), did in self.captures, float(st.params.get("framerate") or 60))
            if before != after:
                log.warning("backpressure %s for '%s' (sent %d, acked %d, rtt %.1f ms)",
                            "lifted" if after else "engaged", did, st.flow.last_sent, st.flow.acknowledged,
                            st.flow.smoothed_rtt_ms)

    def _primary_rtt(self) -> float:
        p = self.displays.get("primary")
        return p.flow.smoothed_rtt_ms if p else 0.0

    def set_client_fps(self, fps: int, did: str = "primary"):
        st = self.displays.get(did)
        if st is not None:
            st.flow.client_fps = float(fps)


class _UploadState:
    """Per-connection upload (``FILE_UPLOAD_START`` / 0x01 chunks / END / ERROR)."""

    def __init__(self, root: Optional[str]):
        self.root = root
        self.path: Optional[str] = None
        self.fh = None
        self.expected = 0
        self.written = 0

    def start(self, msg: str):
        if not self.root:
            log.error("upload refused: no upload directory")
            return
        try:
            rel, size = protocol.parse_upload_start(msg)
        except ValueError:
            log.error("malformed %s", msg[:200])
            return
        target = protocol.sanitize_upload_path(self.root, rel)
        if target is None:
            log.error("upload path rejected: %r", rel)
            return
        self.finish()
        try:
            os.makedirs(os.path.dirname(target), exist_ok=True)
            self.fh = open(target, "wb")
        except OSError as e:
            log.error("cannot open %s: %s", target, e)
            return
        self.path, self.expected, self.written = target, size, 0

    def write(self, data: bytes):
        if self.fh is None:
            return
        try:
            self.fh.write(data)
            self.written += len(data)
        except OSError as e:
            log.error("upload write failed: %s", e)
            self.abort()

    def finish(self):
        if self.fh is not None:
            self.fh.close()
            log.info("upload finished: %s (%d bytes)", self.path, self.written)
        self.fh, self.path = None, None

    def abort(self):
        if self.fh is not None:
            self.fh.close()
            try:
                os.remove(self.path)
            except OSError:
                pass
        self.fh, self.path = None, None
