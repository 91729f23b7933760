"""Node launcher: many desktop sessions on one multi-GPU MI355X node.

Starts one ``selkies`` server process per session (its own X display, port and
GPU chosen by :class:`SessionPlacer`), watches them (process exit and the
``/health`` endpoint) and restarts failed sessions with exponential back-off —
the failure-detection / recovery role the reference delegates to supervisord
(addons/example/supervisord.conf).

    python -m selkies_gstreamer_amd.parallel.launcher --sessions 16 --gpus 8 \
        --base-port 8082 --display-base 20 [-- extra selkies flags]
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import secrets
import signal
import sys
import time
from dataclasses import dataclass, field
from typing import Optional

from .placement import SessionPlacer, session_weight

log = logging.getLogger("launcher")


@dataclass
class SessionSpec:
    name: str
    display: str
    port: int
    gpu: int
    extra: list = field(default_factory=list)
    hw_queues: Optional[int] = None
    ports: list = field(default_factory=list)      # > 1 entry: a session host (parallel/multi.py)
    displays: list = field(default_factory=list)

    def all_ports(self) -> list[int]:
        return self.ports or [self.port]

    def command(self, python: str = sys.executable) -> list[str]:
        if len(self.ports) > 1:
            return [python, "-m", "selkies_gstreamer_amd.parallel.multi", "--ports", ",".join(map(str, self.ports)),
                    "--displays", ",".join(self.displays), "--", "--gpu-id", str(self.gpu), *self.extra]
        return [python, "-m", "selkies_gstreamer_amd", "--port", str(self.port), "--gpu-id", str(self.gpu),
                *self.extra]

    def env(self, base: Optional[dict] = None, control_token: Optional[str] = None) -> dict:
        e = dict(os.environ if base is None else base)
        e["DISPLAY"] = self.display
        if control_token:   # the node control API (/api/*) of the server answers this token only
            e["SELKIES_CONTROL_TOKEN"] = control_token
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if self.hw_queues:
            e.setdefault("GPU_MAX_HW_QUEUES", str(self.hw_queues))
        return e


def hw_queues_for(sessions_on_gpu: int) -> Optional[int]:
    """HIP hardware queues per server process when several share a GPU.

    Every process maps GPU_MAX_HW_QUEUES (default 4) compute queues; with a dozen
    session processes on one MI355X the queues outnumber what the scheduler keeps
    resident and frames stall while queues are swapped. Measured with
    tools/bench_e2e.py at 1080p60 (profiles/r2_e2e_sessions.md): 12 sessions drop to
    52 fps with 4 queues per process, 15 sustain 60 fps with 1 or 2. A session
    needs one queue for its frames and one for uploads/copies."""
    return 2 if sessions_on_gpu > 4 else None


def plan_sessions(n: int, gpus: int, base_port: int, display_base: int, width: int = 1920, height: int = 1080,
                  fps: float = 60.0, extra: Optional[list] = None, capacity: float = 48.0) -> list[SessionSpec]:
    placer = SessionPlacer(gpus, capacity)
    out = []
    for i in range(n):
        gpu = placer.acquire(f"s{i}", session_weight(width, height, fps))
        if gpu is None:
            raise RuntimeError(f"node is full after {i} sessions (capacity {capacity} x 1080p60 per GPU)")
        out.append(SessionSpec(f"s{i}", f":{display_base + i}", base_port + i, gpu, list(extra or [])))
    per_gpu = {g: sum(1 for s in out if s.gpu == g) for g in {s.gpu for s in out}}
    for s in out:
        s.hw_queues = hw_queues_for(per_gpu[s.gpu])
    return out


def group_hosts(specs: list[SessionSpec], per_process: int) -> list[SessionSpec]:
    """Packs the sessions of each GPU into session hosts of up to `per_process`
    sessions (one process, one HIP context: parallel/multi.py); hardware queues are
    then sized for the number of processes per GPU, not sessions."""
    if per_process <= 1:
        return specs
    out: list[SessionSpec] = []
    for gpu in sorted({s.gpu for s in specs}):
        mine = [s for s in specs if s.gpu == gpu]
        for i in range(0, len(mine), per_process):
            grp = mine[i:i + per_process]
            out.append(SessionSpec(f"h{gpu}.{i // per_process}", grp[0].display, grp[0].port, gpu, list(grp[0].extra),
                                   ports=[s.port for s in grp], displays=[s.display for s in grp]))
    per_gpu = {g: sum(1 for s in out if s.gpu == g) for g in {s.gpu for s in out}}
    for s in out:
        s.hw_queues = hw_queues_for(per_gpu[s.gpu])
    return out


class Supervisor:
    def __init__(self, specs: list[SessionSpec], health_interval: float = 5.0, max_backoff: float = 60.0,
                 check_health: bool = True):
        self.specs = specs
        self.procs: dict = {}
        self.restarts: dict = {s.name: 0 for s in specs}
        self.health_interval, self.max_backoff = health_interval, max_backoff
        self.check_health = check_health
        self.stopping = False
        # shared secret of the node's control API: every server gets it in its environment,
        # the Rebalancer sends it; nothing reaching a server through a proxy knows it
        self.control_token = secrets.token_hex(16)

    async def _spawn(self, spec: SessionSpec):
        p = await asyncio.create_subprocess_exec(*spec.command(), env=spec.env(control_token=self.control_token))
        self.procs[spec.name] = p
        log.info("session %s: pid %d, display %s, port %d, gpu %d", spec.name, p.pid, spec.display, spec.port,
                 spec.gpu)
        return p

    async def _healthy(self, spec: SessionSpec) -> bool:
        import aiohttp
        try:
            async with aiohttp.ClientSession() as s:
                for port in spec.all_ports():   # a host is healthy when every session answers
                    async with s.get(f"http://127.0.0.1:{port}/health",
                                     timeout=aiohttp.ClientTimeout(total=3)) as r:
                        if r.status != 200:
                            return False
                return True
        except Exception:
            return False

    async def _watch(self, spec: SessionSpec):
        backoff = 1.0
        while not self.stopping:
            p = await self._spawn(spec)
            started = time.monotonic()
            unhealthy = 0
            while p.returncode is None and not self.stopping:
                try:
                    await asyncio.wait_for(p.wait(), self.health_interval)
                except asyncio.TimeoutError:
                    if self.check_health and time.monotonic() - started > 3 * self.health_interval:
                        unhealthy = 0 if await self._healthy(spec) else unhealthy + 1
                        if unhealthy >= 3:
                            log.error("session %s failed health checks; restarting", spec.name)
                            p.terminate()
                            await p.wait()
            if self.stopping:
                break
            self.restarts[spec.name] += 1
            if time.monotonic() - started > 60:
                backoff = 1.0
            log.warning("session %s exited (%s); restart #%d in %.0fs", spec.name, p.returncode,
                        self.restarts[spec.name], backoff)
            await asyncio.sleep(backoff)
            backoff = min(self.max_backoff, backoff * 2)

    async def relocate(self, name: str, gpu: int) -> None:
        """Restarts session `name` on GPU `gpu` (its own GPU stopped answering, so its
        encoder state cannot be carried: the viewers get a key frame after reconnecting)."""
        spec = next((s for s in self.specs if s.name == name), None)
        if spec is None or spec.gpu == gpu:
            return
        log.warning("session %s: relocating from GPU %d to GPU %d", name, spec.gpu, gpu)
        spec.gpu = gpu
        per_gpu = sum(1 for s in self.specs if s.gpu == gpu)   # processes on the new GPU, this one included
        spec.hw_queues = hw_queues_for(per_gpu)
        p = self.procs.get(name)
        if p is not None and p.returncode is None:
            p.terminate()   # _watch respawns it with the new spec

    async def run(self, rebalance: Optional[float] = None, gpus: Optional[list] = None, capacity: float = 48.0):
        """Supervises every session; with `rebalance` (poll interval, s) a Rebalancer
        moves displays between `gpus` while they run (parallel/rebalance.py)."""
        tasks = [self._watch(s) for s in self.specs]
        if rebalance:
            from .rebalance import Rebalancer
            self.rebalancer = Rebalancer({s.name: s.all_ports() for s in self.specs},
                                         gpus if gpus is not None else sorted({s.gpu for s in self.specs}),
                                         capacity=capacity, on_failed_move=self.relocate,
                                         token=self.control_token)
            self._rb_stop = asyncio.Event()
            tasks.append(self.rebalancer.run(rebalance, self._rb_stop))
        await asyncio.gather(*tasks)

    async def stop(self):
        self.stopping = True
        if getattr(self, "_rb_stop", None) is not None:
            self._rb_stop.set()
        for p in self.procs.values():
            if p.returncode is None:
                p.send_signal(signal.SIGTERM)
        for p in self.procs.values():
            try:
                await asyncio.wait_for(p.wait(), 10)
            except asyncio.TimeoutError:
                p.kill()


def main(argv=None):
    ap = argparse.ArgumentParser(description="Run many selkies sessions across the GPUs of one node")
    ap.add_argument("--sessions", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--base-port", type=int, default=8082)
    ap.add_argument("--display-base", type=int, default=20)
    ap.add_argument("--capacity", type=float, default=48.0, help="1080p60 sessions per GPU")
    ap.add_argument("--sessions-per-process", type=int, default=1,
                    help="> 1: run that many sessions per process (session hosts sharing one HIP context)")
    ap.add_argument("--rebalance", type=float, default=0.0, metavar="SECONDS",
                    help="> 0: move running displays between GPUs on overload or a stalled GPU, polling "
                         "every SECONDS (P-frame continuation, parallel/rebalance.py)")
    ap.add_argument("--dry-run", action="store_true", help="print the plan and exit")
    args, extra = ap.parse_known_args(argv)
    if extra and extra[0] == "--":
        extra = extra[1:]
    logging.basicConfig(level=logging.INFO)
    specs = plan_sessions(args.sessions, args.gpus, args.base_port, args.display_base, extra=extra,
                          capacity=args.capacity)
    specs = group_hosts(specs, args.sessions_per_process)
    if args.dry_run:
        for s in specs:
            print(f"{s.name} DISPLAY={s.display} {' '.join(s.command())}")
        return 0
    sup = Supervisor(specs)

    async def run():
        loop = asyncio.get_running_loop()
        stop = asyncio.Event()
        for sig in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(sig, stop.set)
        task = asyncio.create_task(sup.run(args.rebalance or None, list(range(args.gpus)), args.capacity))
        await stop.wait()
        await sup.stop()
        task.cancel()
    asyncio.run(run())
    return 0


if __name__ == "__main__":
    sys.exit(main())
