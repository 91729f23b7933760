"""Application shell and ``selkies`` entry point (reference selkies.py:113-214, 3133-3307).

Wires settings -> data websocket server -> input handler (XTest, gamepads,
clipboard, cursor) -> capture sessions on the MI355X, then serves until
SIGINT/SIGTERM. Options beyond the 56 reference settings (parsed separately so
unknown flags from container scripts are still ignored):

``--host`` bind address, ``--capture-source auto|x11|synthetic|motion|noise``,
``--gpu-id`` first HIP device, ``--num-gpus`` devices to spread displays over,
``--web-root`` static client directory, ``--upload-dir`` (default
``$FILE_MANAGER_PATH`` or ``~/Desktop``), ``--uinput-mouse-socket``,
``--js-socket-path`` (gamepad socket directory), ``--metrics-csv``, ``--display``
(X display of this session; default ``$DISPLAY``).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import threading
from pathlib import Path
from typing import Optional, Sequence

from .settings import Settings, configure_logging

log = logging.getLogger("main")

WEB_ROOT = Path(__file__).resolve().parents[1] / "web"


def app_options(argv: Sequence[str]):
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--host", default=os.environ.get("SELKIES_HOST", "0.0.0.0"))
    p.add_argument("--capture-source", default=os.environ.get("SELKIES_CAPTURE_SOURCE", "auto"),
                   choices=["auto", "x11", "synthetic", "motion", "noise"])
    p.add_argument("--gpu-id", type=int, default=int(os.environ.get("SELKIES_GPU_ID", "0")))
    p.add_argument("--num-gpus", type=int, default=int(os.environ.get("SELKIES_NUM_GPUS", "1")))
    p.add_argument("--web-root", default=os.environ.get("SELKIES_WEB_ROOT", str(WEB_ROOT)))
    p.add_argument("--upload-dir", default=os.path.expanduser(os.environ.get("FILE_MANAGER_PATH", "~/Desktop")))
    p.add_argument("--uinput-mouse-socket", default=os.environ.get("SELKIES_UINPUT_MOUSE_SOCKET", ""))
    p.add_argument("--js-socket-path", default=os.environ.get("SELKIES_JS_SOCKET_PATH", "/tmp"))
    p.add_argument("--metrics-csv", default=os.environ.get("SELKIES_METRICS_CSV", ""))
    p.add_argument("--display", default=os.environ.get("DISPLAY", ""),
                   help="X display this session captures and injects into (default $DISPLAY)")
    opts, _ = p.parse_known_args(list(argv))
    return opts


def make_input_factory(settings: Settings, opts):
    async def factory(server):
        from .gamepad import GamepadHub
        from .input import Clipboard, CursorWatcher, InputHandler, Injector, UinputMouse, X11Injector
        display = opts.display or None
        inj: Injector = X11Injector(display) if display else Injector()
        if opts.uinput_mouse_socket:
            inj = UinputMouse(opts.uinput_mouse_socket, inj)
        hub = None
        if settings.gamepad_enabled[0]:
            hub = GamepadHub(opts.js_socket_path)
            await hub.start()
        clip_mode = "true" if settings.clipboard_enabled[0] else "false"

        def offset(did):
            l = server.layouts.get(did)
            return (l["x"], l["y"]) if l else (0, 0)

        handler = InputHandler(
            inj, gamepads=hub, clipboard=Clipboard(display), enable_clipboard=clip_mode,
            enable_binary_clipboard=settings.enable_binary_clipboard[0], send_clipboard=server.send_clipboard,
            layout_offset=offset, on_client_fps=lambda fps: (server.set_client_fps(fps),
                                                             server.metrics and server.metrics.set_fps(fps)),
            on_client_latency=lambda ms: server.metrics and server.metrics.set_latency(ms),
            on_client_stats=lambda k, d: server.metrics and server.metrics.set_webrtc_stats(k, d))
        handler.start_clipboard_monitor()
        if display and not settings.use_browser_cursors[0]:
            watcher = CursorWatcher(server.send_cursor, display)
            if watcher.available:
                threading.Thread(target=watcher.run, name="cursor-watch", daemon=True).start()
                orig_close = handler.close

                async def close():
                    watcher.stop()
                    await orig_close()
                handler.close = close
        return handler
    return factory



def basic_auth_from_env(env=None):
    """(user, password) when SELKIES_ENABLE_BASIC_AUTH is true (the legacy signalling
    server's variables, legacy/signalling.py), else None."""
    env = os.environ if env is None else env
    if env.get("SELKIES_ENABLE_BASIC_AUTH", "false").lower() not in ("true", "1", "yes"):
        return None
    return env.get("SELKIES_BASIC_AUTH_USER", env.get("USER", "")), env.get("SELKIES_BASIC_AUTH_PASSWORD", "")

async def serve(argv: Sequence[str], stop: Optional[asyncio.Event] = None, ready=None):
    from .data_server import DataStreamingServer
    from .metrics import Metrics
    settings = Settings(argv)
    opts = app_options(argv)
    configure_logging(settings)
    metrics = Metrics(csv_path=opts.metrics_csv or None)
    if opts.num_gpus == 1 and opts.capture_source != "cpu":
        try:   # capture/encode threads and pinned frames next to the GPU (parallel/numa.py)
            from ..parallel.numa import bind_to_gpu
            from ..ops.native import hip_device_count
            if hip_device_count() > opts.gpu_id:
                node = bind_to_gpu(opts.gpu_id)
                if node is not None:
                    logging.getLogger("selkies").info("bound to NUMA node %d of GPU %d", node, opts.gpu_id)
        except (OSError, RuntimeError):
            pass
    server = DataStreamingServer(settings, upload_dir=opts.upload_dir if "upload" in settings.file_transfers else None,
                                 download_dir=opts.upload_dir if "download" in settings.file_transfers else None,
                                 input_factory=make_input_factory(settings, opts), capture_source=opts.capture_source,
                                 gpu_id=opts.gpu_id, num_gpus=opts.num_gpus, web_root=opts.web_root, metrics=metrics,
                                 x_display=opts.display, basic_auth=basic_auth_from_env())
    metrics.server = server
    port = await server.start(opts.host, settings.port)
    if ready is not None:
        ready(server, port)
    stop = stop or asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError, ValueError):
            pass
    await stop.wait()
    await server.stop()


def main(argv: Optional[Sequence[str]] = None) -> int:
    import sys
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    argv = sys.argv[1:] if argv is None else argv
    if "-h" in argv or "--help" in argv:
        from .settings import build_specs
        print("usage: selkies [options]\n\nsettings (CLI > SELKIES_* env > legacy env > default):")
        for s in build_specs():
            print(f"  {s.flag:<40} {s.help}")
        print("\nserver options: --host --capture-source --gpu-id --num-gpus --web-root --upload-dir "
              "--uinput-mouse-socket --js-socket-path --metrics-csv --display")
        return 0
    asyncio.run(serve(argv))
    return 0
