"""Signalling server + HTTP front of the legacy WebRTC mode (reference
legacy/signalling_web.py), on aiohttp.

Protocol (GStreamer webrtc demo signalling, unchanged so existing clients work):
  client -> ``HELLO <uid> [base64(json meta)]``          server -> ``HELLO``
  client -> ``SESSION <peer_uid>``                        server -> ``SESSION_OK <base64(peer meta)>``
            then every message is relayed verbatim to the peer (SDP / ICE JSON)
  client -> ``ROOM <room_id>``                            server -> ``ROOM_OK <peer ids>``
            room members get ``ROOM_PEER_JOINED <uid>`` / ``ROOM_PEER_LEFT <uid>``;
            ``ROOM_PEER_MSG <uid> <msg>`` is relayed inside the room
  errors: ``ERROR peer '<id>' not found`` / ``busy`` / ``invalid room id`` ...
HTTP: websocket on ``/ws`` or ``*/signalling``; ``<health>`` -> ``OK``; ``/turn``
-> RTC config (HMAC from the shared secret, or the static config); everything
else is served from the web root (path-checked). Optional basic auth and TLS
(certificate changes picked up by restarting the site). ``SELKIES_START_AFTER_
CONNECT`` / ``SELKIES_START_AFTER_DISCONNECT`` commands run on the first session /
after the last one.
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import json
import logging
import os
import ssl
import subprocess
from typing import Optional

from aiohttp import WSMsgType, web

from selkies_gstreamer_amd.server.turn import rtc_config

log = logging.getLogger("signalling")


class SignallingServer:
    def __init__(self, *, addr: str = "0.0.0.0", port: int = 8443, web_root: Optional[str] = None,
                 health_path: str = "/health", keepalive_timeout: float = 30.0, enable_basic_auth: bool = False,
                 basic_auth_user: str = "", basic_auth_password: str = "", turn_shared_secret: str = "",
                 turn_host: str = "", turn_port: str = "3478", turn_protocol: str = "udp", turn_tls: bool = False,
                 turn_auth_header_name: str = "x-auth-user", stun_host: Optional[str] = None,
                 stun_port: Optional[str] = None, rtc_config_json: Optional[str] = None,
                 https_cert: Optional[str] = None, https_key: Optional[str] = None):
        self.addr, self.port, self.web_root = addr, port, web_root
        self.health_path = health_path.rstrip("/") or "/health"
        self.keepalive = keepalive_timeout
        self.basic = (basic_auth_user, basic_auth_password) if enable_basic_auth else None
        self.turn = dict(secret=turn_shared_secret, host=turn_host, port=turn_port, protocol=turn_protocol,
                         tls=turn_tls, header=turn_auth_header_name, stun_host=stun_host, stun_port=stun_port)
        self.rtc_config_json = rtc_config_json
        self.https = (https_cert, https_key) if https_cert and https_key else None
        self.peers: dict = {}     # uid -> [ws, remote, status(None|'session'|room), meta]
        self.sessions: dict = {}  # uid <-> uid
        self.rooms: dict = {}     # room -> set(uid)
        self.runner: Optional[web.AppRunner] = None

    # ------------------------------------------------------------------ http
    def _authorized(self, request) -> bool:
        if not self.basic:
            return True
        h = request.headers.get("Authorization", "")
        if not h.lower().startswith("basic "):
            return False
        try:
            user, _, pw = base64.b64decode(h[6:]).decode().partition(":")
        except ValueError:
            return False
        return (user, pw) == self.basic

    async def _dispatch(self, request: web.Request):
        if not self._authorized(request):
            return web.Response(status=401, text="Authorization required",
                                headers={"WWW-Authenticate": 'Basic realm="restricted", charset="UTF-8"'})
        path = request.path
        if path in ("/ws", "/ws/") or path.rstrip("/").endswith("/signalling"):
            return await self.ws_handler(request)
        if path.rstrip("/") == self.health_path:
            return web.Response(text="OK\n")
        if path.rstrip("/") == "/turn":
            if self.turn["secret"]:
                user = request.headers.get(self.turn["header"], "username") or "username"
                cfg = rtc_config(self.turn["host"], self.turn["port"], self.turn["secret"], user,
                                 self.turn["protocol"], self.turn["tls"], self.turn["stun_host"],
                                 self.turn["stun_port"])
                return web.json_response(cfg)
            if self.rtc_config_json:
                return web.Response(text=self.rtc_config_json, content_type="application/json")
            return web.Response(status=404, text="404 NOT FOUND")
        if self.web_root:
            rel = path.lstrip("/") or "index.html"
            root = os.path.realpath(self.web_root)
            full = os.path.realpath(os.path.join(root, rel))
            if os.path.commonpath((root, full)) == root and os.path.isfile(full):
                return web.FileResponse(full)
        return web.Response(status=404, text="404 NOT FOUND", content_type="text/html")

    def make_app(self) -> web.Application:
        app = web.Application()
        app.router.add_route("*", "/{tail:.*}", self._dispatch)
        return app

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.https:
            return None
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(*self.https)
        return ctx

    async def start(self) -> int:
        self.runner = web.AppRunner(self.make_app())
        await self.runner.setup()
        site = web.TCPSite(self.runner, self.addr, self.port, ssl_context=self.ssl_context())
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self.port

    async def stop(self):
        for uid in list(self.peers):
            await self.remove_peer(uid)
        if self.runner:
            await self.runner.cleanup()

    # ------------------------------------------------------------------ websocket
    async def ws_handler(self, request):
        ws = web.WebSocketResponse(heartbeat=self.keepalive)
        await ws.prepare(request)
        uid = None
        try:
            uid, meta = await self._hello(ws)
            if uid is None:
                return ws
            self.peers[uid] = [ws, request.remote, None, meta]
            log.info("registered peer %r", uid)
            async for msg in ws:
                if msg.type != WSMsgType.TEXT:
                    continue
                await self._on_message(uid, msg.data)
        finally:
            if uid is not None and uid in self.peers and self.peers[uid][0] is ws:
                await self.remove_peer(uid)
        return ws

    async def _hello(self, ws):
        msg = await ws.receive()
        if msg.type != WSMsgType.TEXT:
            await ws.close(code=1002, message=b"invalid protocol")
            return None, None
        toks = msg.data.split(maxsplit=2)
        if len(toks) < 2 or toks[0] != "HELLO":
            await ws.close(code=1002, message=b"invalid protocol")
            return None, None
        uid = toks[1]
        if not uid or uid in self.peers:
            await ws.close(code=1002, message=b"invalid peer uid")
            return None, None
        meta = None
        if len(toks) > 2:
            try:
                meta = json.loads(base64.b64decode(toks[2]))
            except ValueError:
                meta = None
        await ws.send_str("HELLO")
        return uid, meta

    async def _on_message(self, uid: str, msg: str):
        ws, _, status, _ = self.peers[uid]
        if status == "session":
            other = self.sessions.get(uid)
            if other in self.peers:
                await self.peers[other][0].send_str(msg)
            return
        if status is not None:  # in a room
            if msg.startswith("ROOM_PEER_MSG"):
                parts = msg.split(maxsplit=2)
                if len(parts) < 3:
                    await ws.send_str("ERROR invalid ROOM_PEER_MSG")
                    return
                _, other, body = parts
                if other not in self.peers:
                    await ws.send_str(f"ERROR peer {other!r} not found")
                elif self.peers[other][2] != status:
                    await ws.send_str(f"ERROR peer {other!r} is not in the room")
                else:
                    await self.peers[other][0].send_str(f"ROOM_PEER_MSG {uid} {body}")
            else:
                await ws.send_str("ERROR invalid msg, already in room")
            return
        if msg.startswith("SESSION"):
            parts = msg.split(maxsplit=1)
            callee = parts[1] if len(parts) > 1 else ""
            if callee not in self.peers:
                await ws.send_str(f"ERROR peer {callee!r} not found")
                return
            if self.peers[callee][2] is not None:
                await ws.send_str(f"ERROR peer {callee!r} busy")
                return
            meta = self.peers[callee][3]
            meta64 = base64.b64encode(json.dumps(meta).encode()).decode() if meta else ""
            await ws.send_str(f"SESSION_OK {meta64}")
            if not self.sessions:
                self._run_hook("SELKIES_START_AFTER_CONNECT")
            self.peers[uid][2] = self.peers[callee][2] = "session"
            self.sessions[uid], self.sessions[callee] = callee, uid
        elif msg.startswith("ROOM"):
            parts = msg.split(maxsplit=1)
            room = parts[1] if len(parts) > 1 else ""
            if not room or room == "session" or room.split() != [room]:
                await ws.send_str(f"ERROR invalid room id {room!r}")
                return
            members = self.rooms.setdefault(room, set())
            await ws.send_str("ROOM_OK " + " ".join(sorted(members)))
            self.peers[uid][2] = room
            members.add(uid)
            for pid in members - {uid}:
                await self.peers[pid][0].send_str(f"ROOM_PEER_JOINED {uid}")
        else:
            log.info("ignoring unknown message %r from %r", msg[:80], uid)

    async def remove_peer(self, uid: str):
        other = self.sessions.pop(uid, None)
        if other is not None:
            self.sessions.pop(other, None)
            if other in self.peers:  # reset the peer too: its session is gone
                wso = self.peers.pop(other)[0]
                await wso.close()
            if not self.sessions:
                self._run_hook("SELKIES_START_AFTER_DISCONNECT")
        entry = self.peers.pop(uid, None)
        if entry is None:
            return
        ws, _, status, _ = entry
        if status and status != "session" and status in self.rooms:
            self.rooms[status].discard(uid)
            for pid in self.rooms[status]:
                if pid in self.peers:
                    await self.peers[pid][0].send_str(f"ROOM_PEER_LEFT {uid}")
            if not self.rooms[status]:
                del self.rooms[status]
        await ws.close()

    @staticmethod
    def _run_hook(var: str):
        cmd = os.environ.get(var, "")
        if cmd:
            try:
                subprocess.Popen(cmd.split(" "), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            except OSError as e:
                log.error("failed to run %s: %s", var, e)


def main(argv=None):
    p = argparse.ArgumentParser(description="Selkies signalling server")
    p.add_argument("--addr", default="0.0.0.0")
    p.add_argument("--port", type=int, default=int(os.environ.get("SELKIES_PORT", 8443)))
    p.add_argument("--web_root", default=os.environ.get("SELKIES_WEB_ROOT", ""))
    p.add_argument("--health", default="/health")
    p.add_argument("--keepalive-timeout", type=float, default=30.0)
    p.add_argument("--enable_basic_auth", default=os.environ.get("SELKIES_ENABLE_BASIC_AUTH", "false"))
    p.add_argument("--basic_auth_user", default=os.environ.get("SELKIES_BASIC_AUTH_USER", "user"))
    p.add_argument("--basic_auth_password", default=os.environ.get("SELKIES_BASIC_AUTH_PASSWORD", ""))
    p.add_argument("--turn_shared_secret", default=os.environ.get("SELKIES_TURN_SHARED_SECRET", ""))
    p.add_argument("--turn_host", default=os.environ.get("SELKIES_TURN_HOST", ""))
    p.add_argument("--turn_port", default=os.environ.get("SELKIES_TURN_PORT", "3478"))
    p.add_argument("--turn_protocol", default=os.environ.get("SELKIES_TURN_PROTOCOL", "udp"))
    p.add_argument("--turn_tls", default=os.environ.get("SELKIES_TURN_TLS", "false"))
    p.add_argument("--enable_https", default=os.environ.get("SELKIES_ENABLE_HTTPS", "false"))
    p.add_argument("--https_cert", default=os.environ.get("SELKIES_HTTPS_CERT", ""))
    p.add_argument("--https_key", default=os.environ.get("SELKIES_HTTPS_KEY", ""))
    a = p.parse_args(argv)
    https = a.enable_https.lower() == "true"
    srv = SignallingServer(addr=a.addr, port=a.port, web_root=a.web_root or None, health_path=a.health,
                           keepalive_timeout=a.keepalive_timeout,
                           enable_basic_auth=a.enable_basic_auth.lower() == "true", basic_auth_user=a.basic_auth_user,
                           basic_auth_password=a.basic_auth_password, turn_shared_secret=a.turn_shared_secret,
                           turn_host=a.turn_host, turn_port=a.turn_port, turn_protocol=a.turn_protocol,
                           turn_tls=a.turn_tls.lower() == "true", https_cert=a.https_cert if https else None,
                           https_key=a.https_key if https else None)

    async def run():
        await srv.start()
        await asyncio.Event().wait()
    asyncio.run(run())


if __name__ == "__main__":
    main()
