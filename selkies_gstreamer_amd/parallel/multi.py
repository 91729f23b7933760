"""Session host: several desktop sessions served from ONE process (one HIP context).

The launcher's default is one server process per session (parallel/launcher.py),
the reference's deployment shape (one ``selkies`` per desktop). On one MI355X
that shape stops scaling before the GPU does: every process owns a HIP context
and GPU_MAX_HW_QUEUES hardware queues, and past ~12 processes the queues
outnumber what the hardware scheduler keeps resident, so frames wait for queue
swaps (profiles/r2_e2e_sessions.md). A session host runs K complete servers
(own port, settings, capture session, encoder, websocket clients) as coroutines
of one event loop: their encoders share the process's HIP context and queues
(each encoder keeps its own streams and hipGraphs), their capture threads stay
native, and the event loop only moves finished packets.

    python -m selkies_gstreamer_amd.parallel.multi --ports 8082,8083,8084 \
        [--displays :20,:21,:22] -- [selkies flags shared by every session]

Sessions that inject input into real X servers need distinct displays (given
per session here); gamepad sockets are per process, so hosts of several
sessions run with gamepads disabled or one session per host.
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import signal
import sys
from typing import Optional, Sequence

log = logging.getLogger("session-host")


def session_argvs(ports: Sequence[int], shared: Sequence[str],
                  displays: Optional[Sequence[str]] = None) -> list[list[str]]:
    """Per-session server argv: the shared flags with that session's port and X display.

    The display is an explicit ``--display`` flag of each server, never the
    process-wide DISPLAY: every session of the host captures, injects input and
    runs xrandr/DPI tools against its own desktop."""
    out = []
    for i, p in enumerate(ports):
        argv = [a for a in shared]
        for flag in ("--port", "--display"):
            while flag in argv:
                j = argv.index(flag)
                del argv[j:j + 2]
        extra = ["--display", displays[i]] if displays else []
        out.append(["--port", str(p), *extra, *argv])
    return out


async def host(ports: Sequence[int], shared: Sequence[str], displays: Optional[Sequence[str]] = None,
               stop: Optional[asyncio.Event] = None, ready=None) -> None:
    from ..server.app import serve
    stop = stop or asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError, ValueError):
            pass
    stops = [asyncio.Event() for _ in ports]
    tasks = []
    for i, argv in enumerate(session_argvs(ports, shared, displays)):
        tasks.append(asyncio.create_task(serve(argv, stops[i], ready)))
    waiter = asyncio.create_task(stop.wait())
    pending = set(tasks)
    # one session that fails (a port taken, a display gone) is logged and the others
    # keep serving; the host ends on its stop signal or when no session is left
    while pending and not stop.is_set():
        done, _ = await asyncio.wait([waiter, *pending], return_when=asyncio.FIRST_COMPLETED)
        for t in done:
            if t is waiter:
                continue
            pending.discard(t)
    for ev in stops:
        ev.set()
    results = await asyncio.gather(*tasks, return_exceptions=True)
    waiter.cancel()
    for port, r in zip(ports, results):
        if isinstance(r, BaseException) and not isinstance(r, asyncio.CancelledError):
            log.error("session on port %d failed: %r", port, r)


def main(argv: Optional[Sequence[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    shared: list[str] = []
    if "--" in argv:
        i = argv.index("--")
        argv, shared = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description="several selkies sessions in one process")
    ap.add_argument("--ports", required=True, help="comma-separated websocket ports, one per session")
    ap.add_argument("--displays", default="", help="comma-separated X displays, one per session")
    a = ap.parse_args(argv)
    ports = [int(p) for p in a.ports.split(",") if p]
    displays = [d for d in a.displays.split(",") if d] or None
    if displays and len(displays) != len(ports):
        raise SystemExit("--displays needs one display per port")
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    asyncio.run(host(ports, shared, displays))
    return 0


if __name__ == "__main__":
    sys.exit(main())
