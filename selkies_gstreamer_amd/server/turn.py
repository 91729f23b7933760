"""TURN / STUN configuration (reference legacy/signalling_web.py:51-90,
legacy/webrtc.py:62-286, addons/turn-rest/app.py).

* :func:`rtc_config` — RTCConfiguration JSON with time-limited HMAC-SHA1 TURN
  credentials (coturn ``--use-auth-secret``): username ``<expiry>:<user>``,
  credential ``base64(hmac_sha1(secret, username))``, 24 h lifetime, STUN list
  with the TURN host first plus Google STUN as a fallback.
* :func:`legacy_rtc_config` — long-term (static user/password) credentials.
* :func:`parse_rtc_config` — validates a JSON RTC config (file / REST payload).
* :func:`turn_rest_handler` — the TURN REST micro-service as an aiohttp handler
  (query/form/header parameters ``service``, ``username``/``x-auth-user``/
  ``x-turn-username``, ``protocol``/``x-turn-protocol``, ``tls``/``x-turn-tls``).
* :class:`RTCConfigMonitor` — periodically refreshes a config from a HMAC
  secret, a TURN REST URL or a JSON file and calls back on change.
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import hmac
import json
import logging
import os
import time
from typing import Awaitable, Callable, Optional

log = logging.getLogger("turn")

EXPIRY_HOURS = 24
GOOGLE_STUN = ("stun.l.google.com", "19302")


def hmac_credentials(secret: str, user: str, now: Optional[float] = None, hours: int = EXPIRY_HOURS):
    user = user.replace(":", "-")
    exp = int(time.time() if now is None else now) + hours * 3600
    username = f"{exp}:{user}"
    digest = hmac.new(secret.encode(), username.encode(), hashlib.sha1).digest()
    return username, base64.b64encode(digest).decode()


def _stun_urls(turn_host, turn_port, stun_host, stun_port):
    urls = [f"stun:{turn_host}:{turn_port}"]
    if stun_host is not None and stun_port is not None and (stun_host != turn_host or str(stun_port) != str(turn_port)):
        urls.insert(0, f"stun:{stun_host}:{stun_port}")
    if (stun_host, str(stun_port)) != GOOGLE_STUN:
        urls.append(f"stun:{GOOGLE_STUN[0]}:{GOOGLE_STUN[1]}")
    return urls


def rtc_config(turn_host: str, turn_port, secret: str, user: str, protocol: str = "udp", tls: bool = False,
               stun_host: Optional[str] = None, stun_port=None, now: Optional[float] = None) -> dict:
    username, credential = hmac_credentials(secret, user, now)
    protocol = "tcp" if str(protocol).lower() == "tcp" else "udp"
    return {
        "lifetimeDuration": f"{EXPIRY_HOURS * 3600}s",
        "blockStatus": "NOT_BLOCKED",
        "iceTransportPolicy": "all",
        "iceServers": [
            {"urls": _stun_urls(turn_host, turn_port, stun_host, stun_port)},
            {"urls": [f"{'turns' if tls else 'turn'}:{turn_host}:{turn_port}?transport={protocol}"],
             "username": username, "credential": credential},
        ],
    }


def legacy_rtc_config(turn_host: str, turn_port, username: str, password: str, protocol: str = "udp",
                      tls: bool = False, stun_host: Optional[str] = None, stun_port=None) -> dict:
    protocol = "tcp" if str(protocol).lower() == "tcp" else "udp"
    return {
        "lifetimeDuration": "86400s",
        "blockStatus": "NOT_BLOCKED",
        "iceTransportPolicy": "all",
        "iceServers": [
            {"urls": _stun_urls(turn_host, turn_port, stun_host, stun_port)},
            {"urls": [f"{'turns' if tls else 'turn'}:{turn_host}:{turn_port}?transport={protocol}"],
             "username": username, "credential": password},
        ],
    }


def parse_rtc_config(data) -> tuple[list[str], list[str], dict]:
    """Returns (stun_urls, turn_urls_with_credentials, config). Raises ValueError if malformed."""
    cfg = json.loads(data) if isinstance(data, (str, bytes)) else data
    servers = cfg.get("iceServers")
    if not isinstance(servers, list):
        raise ValueError("RTC config has no iceServers list")
    stun, turn = [], []
    for srv in servers:
        urls = srv.get("urls", [])
        urls = [urls] if isinstance(urls, str) else urls
        for u in urls:
            if u.startswith("stun:"):
                stun.append(u)
            elif u.startswith(("turn:", "turns:")):
                user, cred = srv.get("username", ""), srv.get("credential", "")
                scheme, rest = u.split(":", 1)
                turn.append(f"{scheme}://{user}:{cred}@{rest}")
    return stun, turn, cfg


def env_turn_defaults(env=os.environ) -> dict:
    host = (env.get("TURN_HOST") or "staticauth.openrelay.metered.ca").lower()
    port = env.get("TURN_PORT", "443")
    port = port if port.isdigit() else "3478"
    stun_host = (env.get("STUN_HOST") or host).lower()
    stun_port = env.get("STUN_PORT", port)
    if not stun_port.isdigit():
        stun_host, stun_port = GOOGLE_STUN
    return {"secret": env.get("TURN_SHARED_SECRET", "openrelayprojectsecret"), "host": host, "port": port,
            "stun_host": stun_host, "stun_port": stun_port, "protocol": env.get("TURN_PROTOCOL", "udp"),
            "tls": env.get("TURN_TLS", "false").lower() == "true"}


async def turn_rest_handler(request, defaults: Optional[dict] = None):
    """aiohttp handler implementing the TURN REST API (GET/POST /)."""
    from aiohttp import web
    d = defaults or env_turn_defaults()
    params = dict(request.query)
    if request.method == "POST":
        try:
            params.update(await request.post())
        except Exception:  # non-form body
            pass
    h = request.headers
    user = (params.get("username") or h.get("x-auth-user") or h.get("x-turn-username") or "turn-rest").lower()
    protocol = params.get("protocol") or h.get("x-turn-protocol") or d["protocol"]
    tls = str(params.get("tls") or h.get("x-turn-tls") or d["tls"]).lower() == "true"
    cfg = rtc_config(d["host"], d["port"], d["secret"], user, protocol, tls, d["stun_host"], d["stun_port"])
    return web.Response(text=json.dumps(cfg, indent=2), content_type="application/json")


class RTCConfigMonitor:
    """Refreshes an RTC config periodically (HMAC secret / TURN REST URL / JSON file)."""

    def __init__(self, on_change: Callable[[dict], Awaitable[None] | None], *, period_s: float = 60.0,
                 hmac_params: Optional[dict] = None, rest_url: Optional[str] = None,
                 rest_headers: Optional[dict] = None, json_file: Optional[str] = None):
        self.on_change, self.period = on_change, period_s
        self.hmac_params, self.rest_url, self.rest_headers = hmac_params, rest_url, rest_headers or {}
        self.json_file = json_file
        self.current: Optional[dict] = None
        self._mtime = None
        self.task: Optional[asyncio.Task] = None

    async def fetch(self) -> Optional[dict]:
        if self.json_file:
            try:
                mt = os.path.getmtime(self.json_file)
            except OSError:
                return None
            if mt == self._mtime and self.current is not None:
                return self.current
            self._mtime = mt
            with open(self.json_file) as f:
                return parse_rtc_config(f.read())[2]
        if self.rest_url:
            import aiohttp
            async with aiohttp.ClientSession() as s:
                async with s.get(self.rest_url, headers=self.rest_headers,
                                 timeout=aiohttp.ClientTimeout(total=10)) as r:
                    return parse_rtc_config(await r.text())[2]
        if self.hmac_params:
            p = self.hmac_params
            return rtc_config(p["host"], p["port"], p["secret"], p.get("user", "selkies"), p.get("protocol", "udp"),
                              p.get("tls", False), p.get("stun_host"), p.get("stun_port"))
        return None

    async def refresh(self) -> bool:
        try:
            cfg = await self.fetch()
        except Exception as e:
            log.warning("RTC config refresh failed: %s", e)
            return False
        if cfg is None or cfg == self.current:
            return False
        self.current = cfg
        res = self.on_change(cfg)
        if asyncio.iscoroutine(res):
            await res
        return True

    async def run(self):
        while True:
            await self.refresh()
            await asyncio.sleep(self.period)

    def start(self):
        self.task = asyncio.create_task(self.run())

    def stop(self):
        if self.task:
            self.task.cancel()


def main(argv=None) -> int:
    """TURN REST micro-service (reference addons/turn-rest): ``python -m
    selkies_gstreamer_amd.server.turn --port 8008``; configured by TURN_* env."""
    import argparse
    from aiohttp import web
    ap = argparse.ArgumentParser(description="TURN REST API (HMAC-SHA1 time-limited credentials)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=int(os.environ.get("PORT", "8008")))
    a = ap.parse_args(argv)
    app = web.Application()
    defaults = env_turn_defaults()

    async def handle(request):
        return await turn_rest_handler(request, defaults)
    app.router.add_route("GET", "/", handle)
    app.router.add_route("POST", "/", handle)
    web.run_app(app, host=a.host, port=a.port)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
