"""Signalling client of the legacy WebRTC mode (reference legacy/webrtc_signalling.py,
SURVEY C22): registers with ``HELLO <id>``, optionally starts a session with
``SESSION <peer>``, and turns relayed JSON into callbacks (``{"sdp": ...}`` ->
on_sdp(type, sdp), ``{"ice": ...}`` -> on_ice(mline_index, candidate)).
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
from typing import Callable, Optional

import aiohttp

log = logging.getLogger("signalling_client")


class SignallingError(Exception):
    pass


class SignallingClient:
    def __init__(self, server: str, peer_id: int | str, meta: Optional[dict] = None, *,
                 basic_auth: Optional[tuple] = None, ssl=True):
        self.server, self.id, self.meta = server, str(peer_id), meta
        self.auth = aiohttp.BasicAuth(*basic_auth) if basic_auth else None
        self.ssl = ssl
        self.session: Optional[aiohttp.ClientSession] = None
        self.ws = None
        self.on_connect: Callable[[], None] = lambda: None
        self.on_session: Callable[[Optional[dict]], None] = lambda meta: None
        self.on_sdp: Callable[[str, str], None] = lambda t, sdp: None
        self.on_ice: Callable[[int, str], None] = lambda idx, cand: None
        self.on_error: Callable[[Exception], None] = lambda e: log.error("signalling: %s", e)
        self.on_disconnect: Callable[[], None] = lambda: None

    async def connect(self, retries: int = 10, delay: float = 1.0):
        self.session = aiohttp.ClientSession(auth=self.auth)
        last = None
        for _ in range(retries):
            try:
                self.ws = await self.session.ws_connect(self.server, ssl=self.ssl)
                break
            except aiohttp.ClientError as e:
                last = e
                await asyncio.sleep(delay)
        else:
            await self.session.close()
            raise SignallingError(f"cannot connect to {self.server}: {last}")
        hello = f"HELLO {self.id}"
        if self.meta:
            hello += " " + base64.b64encode(json.dumps(self.meta).encode()).decode()
        await self.ws.send_str(hello)

    async def setup_call(self, peer: int | str):
        await self.ws.send_str(f"SESSION {peer}")

    async def send_sdp(self, sdp_type: str, sdp: str):
        await self.ws.send_str(json.dumps({"sdp": {"type": sdp_type, "sdp": sdp}}))

    async def send_ice(self, mline_index: int, candidate: str):
        await self.ws.send_str(json.dumps({"ice": {"candidate": candidate, "sdpMLineIndex": mline_index}}))

    async def start(self):
        """Receives until the socket closes, dispatching to the callbacks."""
        try:
            async for msg in self.ws:
                if msg.type != aiohttp.WSMsgType.TEXT:
                    continue
                data = msg.data
                if data == "HELLO":
                    self.on_connect()
                elif data.startswith("SESSION_OK"):
                    meta64 = data[len("SESSION_OK"):].strip()
                    meta = json.loads(base64.b64decode(meta64)) if meta64 else None
                    self.on_session(meta)
                elif data.startswith("ERROR"):
                    self.on_error(SignallingError(data))
                else:
                    try:
                        obj = json.loads(data)
                    except ValueError:
                        self.on_error(SignallingError(f"unexpected message {data[:80]!r}"))
                        continue
                    if "sdp" in obj:
                        self.on_sdp(obj["sdp"].get("type"), obj["sdp"].get("sdp"))
                    elif "ice" in obj:
                        self.on_ice(obj["ice"].get("sdpMLineIndex"), obj["ice"].get("candidate"))
        finally:
            self.on_disconnect()

    async def stop(self):
        if self.ws is not None:
            await self.ws.close()
        if self.session is not None:
            await self.session.close()
