#!/usr/bin/env python3
"""End-to-end session benchmark: real selkies servers, headless websocket clients.

Measures what the driver's encoder bench cannot: the serving path the reference
runs (capture -> queue_data_for_display -> _video_chunk_sender -> websocket ->
client, src/selkies/selkies.py:2781-2891; client ACKs every 50 ms,
addons/gst-web-core/selkies-core.js:2550-2560), end to end on one host.

* N server processes (one per session, the deployment model of parallel/launcher.py),
  each `python -m selkies_gstreamer_amd` with the synthetic moving-desktop capture
  source on the same GPU, SELKIES_FRAME_TRACE=1 (the server sends `FRAME_TS <fid>
  <grab_ns>` — the frame's CLOCK_MONOTONIC grab time — ahead of its stripes).
* N headless aiohttp clients (sharded over --client-procs processes) speak the reference protocol (MODE,
  server_settings, SETTINGS, 0x04 stripes, CLIENT_FRAME_ACK every 50 ms) and
  timestamp the first stripe of every frame on receipt.
* Reported per N: received fps per session (min / median), capture -> client receive
  latency p50 / p99 (the server + transport share of glass-to-glass; the browser's
  decode and paint are not in it), and whether every session sustained the target
  fps. `--sweep 8,16,24` finds the largest N that does ("concurrent 60 fps sessions").

usage: python tools/bench_e2e.py --sweep 4,8,16 --seconds 6 [--width 1920 --height 1080]
"""
from __future__ import annotations

import argparse
import asyncio
import concurrent.futures
import json
import multiprocessing
import os
import signal
import socket
import subprocess
import sys
import time

import aiohttp
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from selkies_gstreamer_amd.parallel.launcher import hw_queues_for  # noqa: E402


_TAKEN: set = set()


def free_port() -> int:
    """A port below the kernel's ephemeral range. Ports the OS hands out for port 0
    (every session's data websocket, client sockets) come from that range, so a port
    picked there and released can be taken again before its server binds it (a 48-session
    run lost a server that way: 'address already in use')."""
    lo = 32768
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        pass
    base = max(1024, lo - 12000)
    rng = np.random.default_rng()
    for _ in range(1000):
        p = int(rng.integers(base, lo))
        if p in _TAKEN:
            continue
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
        except OSError:
            continue
        finally:
            s.close()
        _TAKEN.add(p)
        return p
    raise RuntimeError("no free port below the ephemeral range")


def start_servers(n: int, args) -> list:
    """N sessions as processes of --sessions-per-proc sessions each (1 = one server
    process per session, the reference shape; K > 1 = parallel/multi.py session hosts
    sharing one HIP context). Returns one (process, port, log) per session."""
    out = []
    k = max(1, int(getattr(args, "sessions_per_proc", 1) or 1))
    nproc = (n + k - 1) // k
    for j in range(nproc):
        ports = [free_port() for _ in range(min(k, n - j * k))]
        env = dict(os.environ, SELKIES_FRAME_TRACE="1", PYTHONUNBUFFERED="1")
        q = args.hw_queues if args.hw_queues is not None else hw_queues_for(nproc)
        if q:
            env["GPU_MAX_HW_QUEUES"] = str(q)  # what parallel/launcher.py gives co-located processes
        shared = ["--host", "127.0.0.1", "--capture-source", args.source, "--audio-enabled", "false",
                  "--gpu-id", str(args.gpu), "--gamepad-enabled", "false"]
        if args.use_cpu:
            shared += ["--use-cpu", "true"]
        if k == 1:
            cmd = [sys.executable, "-m", "selkies_gstreamer_amd", "--port", str(ports[0]), *shared]
        else:
            cmd = [sys.executable, "-m", "selkies_gstreamer_amd.parallel.multi", "--ports",
                   ",".join(map(str, ports)), "--", *shared]
        log = open(os.path.join(args.log_dir, f"server_{n}_{j}.log"), "w")
        p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
        out.extend((p, port, log) for port in ports)
    return out


def stop_servers(procs):
    seen = {}
    for p, _, log in procs:
        seen[p.pid] = (p, log)
    for p, log in seen.values():
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    for p, log in seen.values():
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
        log.close()


async def wait_ready(port: int, timeout: float = 90.0):
    end = time.monotonic() + timeout
    async with aiohttp.ClientSession() as s:
        while time.monotonic() < end:
            try:
                async with s.get(f"http://127.0.0.1:{port}/health", timeout=aiohttp.ClientTimeout(total=2)) as r:
                    if r.status == 200:
                        return
            except Exception:
                pass
            await asyncio.sleep(0.25)
    raise TimeoutError(f"server on port {port} did not come up")


class DecodeThread:
    """The client's decoder for full-frame AV1 sessions (--decode): dav1d on its own
    thread (ctypes releases the GIL, as a browser decodes off its main thread), fed each
    frame's temporal unit on receipt. Records grab -> decoded picture per frame."""

    def __init__(self, threads: int):
        import queue
        import threading
        from selkies_gstreamer_amd.models.av1.dav1d import Decoder
        self.dec = Decoder(n_threads=threads)
        self.q: "queue.Queue" = queue.Queue()
        self.lat_ms: list = []
        self.dec_ms: list = []
        self.errors = 0
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def push(self, tu: bytes, grab_ns, count: bool):
        self.q.put((tu, grab_ns, count))

    def _run(self):
        while True:
            item = self.q.get()
            if item is None:
                break
            tu, g, count = item
            t0 = time.monotonic_ns()
            try:
                pic = self.dec.decode(tu, planes=False)
            except Exception:
                self.errors += 1
                continue
            t1 = time.monotonic_ns()
            if count and pic is not None:
                self.dec_ms.append((t1 - t0) / 1e6)
                if g is not None:
                    self.lat_ms.append((t1 - g) / 1e6)

    def close(self):
        self.q.put(None)
        self.t.join(timeout=30)
        self.dec.close()


async def client(port: int, args, t_start: float, t_end: float, out: dict):
    grabs: dict = {}
    decoder = DecodeThread(getattr(args, "decode_threads", 4)) if getattr(args, "decode", False) else None
    seen: set = set()
    lat_ms: list = []        # grab -> first stripe of the frame received
    lat_last_ms: list = []   # grab -> last stripe of the frame received (whole frame on the client)
    cur = {"fid": None, "grab": None, "last": 0, "count": False}
    frames = 0
    last_fid = None
    bytes_rx = 0
    async with aiohttp.ClientSession() as sess:
        async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket", max_msg_size=0) as ws:
            settings = {"initialClientWidth": args.width, "initialClientHeight": args.height,
                        "framerate": args.fps, "encoder": args.encoder, "h264_crf": args.crf}
            if getattr(args, "kbps", 0):
                settings["h264_bitrate"] = int(args.kbps)
            sent_settings = False

            async def acks():
                while True:
                    await asyncio.sleep(0.05)
                    if last_fid is not None:
                        await ws.send_str(f"CLIENT_FRAME_ACK {last_fid}")
            ack_task = asyncio.create_task(acks())
            try:
                while time.monotonic() < t_end:
                    try:
                        msg = await asyncio.wait_for(ws.receive(), max(0.05, t_end - time.monotonic()))
                    except asyncio.TimeoutError:
                        break
                    now_ns = time.monotonic_ns()
                    if msg.type == aiohttp.WSMsgType.TEXT:
                        m = msg.data
                        if not sent_settings and "server_settings" in m:
                            await ws.send_str("SETTINGS," + json.dumps(settings))
                            sent_settings = True
                        elif m.startswith("FRAME_TS "):
                            _, fid, g = m.split()
                            grabs[int(fid)] = int(g)
                    elif msg.type == aiohttp.WSMsgType.BINARY:
                        d = msg.data
                        if len(d) >= 10 and d[0] == 0x04:
                            fid = (d[2] << 8) | d[3]
                            last_fid = fid
                            bytes_rx += len(d)
                            if fid != cur["fid"]:
                                # the previous frame's stripes are complete: its last one arrived at cur["last"]
                                if cur["count"] and cur["grab"] is not None:
                                    lat_last_ms.append((cur["last"] - cur["grab"]) / 1e6)
                                cur.update(fid=fid, grab=None, count=False)
                            cur["last"] = now_ns
                            if fid not in seen:
                                seen.add(fid)
                                if len(seen) > 4096:
                                    seen.clear()
                                counted = time.monotonic() >= t_start
                                g = grabs.pop(fid, None)
                                if counted:
                                    frames += 1
                                    cur["grab"], cur["count"] = g, True
                                    if g is not None:
                                        lat_ms.append((now_ns - g) / 1e6)
                                if decoder is not None:   # full-frame: one packet = one temporal unit
                                    decoder.push(bytes(d[10:]), g, counted)
                    else:
                        break
            finally:
                ack_task.cancel()
    dec = {}
    if decoder is not None:
        decoder.close()
        dec = dict(lat_dec=decoder.lat_ms, dec_ms=decoder.dec_ms, dec_errors=decoder.errors)
    out[port] = dict(frames=frames, lat=lat_ms, lat_last=lat_last_ms, bytes=bytes_rx, **dec)


def client_worker(ports, args, t_start, t_end) -> dict:
    """One client process drives a shard of the sessions (a single Python
    process cannot receive ~15k stripe messages/s for 15 sessions by itself)."""
    async def go():
        out: dict = {}
        await asyncio.gather(*(client(p, args, t_start, t_end, out) for p in ports))
        return out
    return asyncio.run(go())


class CpuSampler:
    """Where the CPU goes during the measured window (--sample-cpu): per server process
    the CPU seconds per second, its busiest thread (the Python main thread holding the
    GIL shows up here near 1.0) and the native threads; the client processes; and the
    GPU busy % from rocm-smi. Used to attribute the session-count ceiling."""

    def __init__(self, server_pids, period=0.5):
        import threading
        self.pids = sorted(set(server_pids))
        self.period = period
        self.samples = []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def start(self):
        self._t.start()

    def stop(self) -> dict:
        self._stop.set()
        self._t.join(5)
        return self.summary()

    def _snap(self):
        import psutil
        out = {"t": time.monotonic(), "servers": {}, "clients": 0.0}
        for pid in self.pids:
            try:
                p = psutil.Process(pid)
                th = {t.id: t.user_time + t.system_time for t in p.threads()}
                ct = p.cpu_times()
                out["servers"][pid] = (ct.user + ct.system, th)
            except (psutil.NoSuchProcess, psutil.AccessDenied):
                pass
        me = psutil.Process()
        for ch in me.children(recursive=True):
            if ch.pid in self.pids:
                continue
            try:
                ct = ch.cpu_times()
                out["clients"] += ct.user + ct.system
            except (psutil.NoSuchProcess, psutil.AccessDenied):
                pass
        return out

    def _gpu_busy(self):
        try:
            r = subprocess.run(["rocm-smi", "--showuse", "--json"], capture_output=True, text=True, timeout=5)
            d = json.loads(r.stdout)
            vals = [float(v.get("GPU use (%)", "nan")) for v in d.values() if isinstance(v, dict)]
            return max(vals) if vals else None
        except Exception:   # noqa: BLE001 - optional
            return None

    def _run(self):
        prev = self._snap()
        while not self._stop.wait(self.period):
            cur = self._snap()
            dt = cur["t"] - prev["t"]
            row = {"servers": [], "clients_cpu": (cur["clients"] - prev["clients"]) / dt, "gpu_busy": self._gpu_busy()}
            for pid, (tot, th) in cur["servers"].items():
                if pid not in prev["servers"]:
                    continue
                ptot, pth = prev["servers"][pid]
                per = sorted(((th[k] - pth.get(k, th[k])) / dt for k in th), reverse=True)
                main = (th.get(pid, 0.0) - pth.get(pid, th.get(pid, 0.0))) / dt
                row["servers"].append({"cpu": (tot - ptot) / dt, "main_thread": main, "busiest_thread": per[0] if per else 0.0,
                                       "threads_over_half": sum(1 for x in per if x > 0.5)})
            self.samples.append(row)
            prev = cur

    def summary(self) -> dict:
        if not self.samples:
            return {}
        import statistics as stt
        srv = [s for row in self.samples for s in row["servers"]]
        gb = [row["gpu_busy"] for row in self.samples if row["gpu_busy"] is not None]
        per_sample_total = [sum(s["cpu"] for s in row["servers"]) for row in self.samples]
        return {"samples": len(self.samples),
                "server_procs": len(self.pids),
                "servers_cpu_total": round(stt.median(per_sample_total), 2),
                "server_proc_cpu_max": round(max(s["cpu"] for s in srv), 2),
                "main_thread_cpu_median": round(stt.median(s["main_thread"] for s in srv), 2),
                "main_thread_cpu_max": round(max(s["main_thread"] for s in srv), 2),
                "busiest_thread_cpu_max": round(max(s["busiest_thread"] for s in srv), 2),
                "clients_cpu": round(stt.median(row["clients_cpu"] for row in self.samples), 2),
                "gpu_busy_median": round(stt.median(gb), 1) if gb else None,
                "cpus_available": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count(),
                "cpu_quota": _cgroup_cpus()}


def _cgroup_cpus():
    """CPUs this container may use (cgroup v2 cpu.max quota / period), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


async def run_n(n: int, args) -> dict:
    procs = start_servers(n, args)
    sampler = None
    try:
        await asyncio.gather(*(wait_ready(port) for _, port, _ in procs))
        t0 = time.monotonic()
        t_start = t0 + args.warmup
        t_end = t_start + args.seconds
        if getattr(args, "sample_cpu", False):
            sampler = CpuSampler([p.pid for p, _, _ in procs])
            loop0 = asyncio.get_running_loop()
            loop0.call_later(max(0.0, t_start - time.monotonic()), sampler.start)
        ports = [port for _, port, _ in procs]
        shards = [ports[i::args.client_procs] for i in range(min(args.client_procs, n))]
        ctx = multiprocessing.get_context("spawn")
        loop = asyncio.get_running_loop()
        with concurrent.futures.ProcessPoolExecutor(len(shards), mp_context=ctx) as ex:
            parts = await asyncio.gather(*(loop.run_in_executor(ex, client_worker, sh, args, t_start, t_end)
                                           for sh in shards))
        out: dict = {}
        for part in parts:
            out.update(part)
    finally:
        cpu = sampler.stop() if sampler is not None and sampler._t.is_alive() else None
        stop_servers(procs)
        _TAKEN.difference_update(port for _, port, _ in procs)
    fps = np.array([out[p]["frames"] / args.seconds for _, p, _ in procs]) if out else np.zeros(1)
    lat = np.concatenate([np.asarray(out[p]["lat"], dtype=np.float64) for _, p, _ in procs]) if out else np.zeros(0)
    lat_last = (np.concatenate([np.asarray(out[p]["lat_last"], dtype=np.float64) for _, p, _ in procs])
                if out else np.zeros(0))
    ok = bool(len(fps) == n and fps.min() >= args.fps * args.sustain)
    dec = {}
    if getattr(args, "decode", False) and out:
        ld = np.concatenate([np.asarray(out[p].get("lat_dec", []), dtype=np.float64) for _, p, _ in procs])
        dm = np.concatenate([np.asarray(out[p].get("dec_ms", []), dtype=np.float64) for _, p, _ in procs])
        pct = lambda a, q: round(float(np.percentile(a, q)), 2) if len(a) else None   # noqa: E731
        dec = {"decoded_latency_p50_ms": pct(ld, 50), "decoded_latency_p99_ms": pct(ld, 99),
               "decoded_samples": int(len(ld)), "dav1d_decode_p50_ms": pct(dm, 50), "dav1d_decode_p99_ms": pct(dm, 99),
               "decode_errors": int(sum(out[p].get("dec_errors", 0) for _, p, _ in procs))}
    return {"sessions": n, "fps_min": round(float(fps.min()), 2), "fps_median": round(float(np.median(fps)), 2),
            "aggregate_fps": round(float(fps.sum()), 1),
            "latency_p50_ms": round(float(np.percentile(lat, 50)), 2) if len(lat) else None,
            "latency_p99_ms": round(float(np.percentile(lat, 99)), 2) if len(lat) else None,
            "latency_samples": int(len(lat)),
            "frame_latency_p50_ms": round(float(np.percentile(lat_last, 50)), 2) if len(lat_last) else None,
            "frame_latency_p99_ms": round(float(np.percentile(lat_last, 99)), 2) if len(lat_last) else None,
            "sustained": ok, **dec, **({"cpu": cpu} if cpu else {})}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", default="1,4,8", help="comma-separated session counts")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--warmup", type=float, default=3.0)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fps", type=int, default=60)
    ap.add_argument("--crf", type=int, default=25)
    ap.add_argument("--encoder", default="x264enc-striped")
    ap.add_argument("--source", default="motion", choices=["motion", "synthetic", "noise"])
    ap.add_argument("--gpu", type=int, default=0)
    ap.add_argument("--use-cpu", action="store_true")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES per server (default: the launcher's choice for N sessions)")
    ap.add_argument("--client-procs", type=int, default=4, help="client processes the sessions are sharded over")
    ap.add_argument("--sessions-per-proc", type=int, default=1,
                    help="sessions per server process (> 1: parallel/multi.py session hosts)")
    ap.add_argument("--sustain", type=float, default=0.97, help="fraction of --fps every session must receive")
    ap.add_argument("--kbps", type=int, default=0, help="> 0: CBR at this bitrate (h264_bitrate setting)")
    ap.add_argument("--decode", action="store_true",
                    help="full-frame AV1 (--encoder svtav1enc): the clients decode every frame with dav1d and "
                         "report grab -> decoded picture latency")
    ap.add_argument("--decode-threads", type=int, default=4)
    ap.add_argument("--log-dir", default=os.path.join(ROOT, "gpurun_out", "e2e_logs"))
    ap.add_argument("--sample-cpu", action="store_true",
                    help="sample server / client CPU (per thread) and GPU busy over the measured window")
    args = ap.parse_args()
    os.makedirs(args.log_dir, exist_ok=True)
    results = []
    best = 0
    for n in [int(x) for x in args.sweep.split(",")]:
        r = asyncio.run(run_n(n, args))
        results.append(r)
        print(json.dumps(r), flush=True)
        if r["sustained"]:
            best = max(best, n)
    print(json.dumps({"metric": "concurrent sustained sessions + capture->client latency",
                      "resolution": f"{args.width}x{args.height}", "target_fps": args.fps,
                      "encoder": args.encoder, "max_sustained_sessions": best, "runs": results}), flush=True)


if __name__ == "__main__":
    main()
