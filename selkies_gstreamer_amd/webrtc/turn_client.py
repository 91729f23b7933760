"""TURN client (RFC 5766, UDP) for relayed ICE candidates on the server side.

Reference role: the aioice TURN support under the vendored aiortc
(src/selkies/webrtc/rtcicetransport.py:53-139 builds TURN servers from the RTC
config) and webrtcbin's ``turn-server`` / ``add-turn-server`` (legacy/gstwebrtc_app.py:
149-197). A server behind a NAT that blocks inbound UDP (the usual Kubernetes pod)
is only reachable through its own relay allocation.

The allocation shares the ICE agent's UDP socket: the agent hands every datagram
from the TURN server to :meth:`TurnAllocation.on_datagram`, which resolves pending
transactions and unwraps Data indications / ChannelData into (peer, payload).

* Allocate with the long-term credential mechanism: unauthenticated request ->
  401 (REALM, NONCE) -> authenticated retry; 438 Stale Nonce retries once more.
* CreatePermission per peer IP before anything is relayed to it, ChannelBind
  (0x4000+) per peer so data uses the 4-byte ChannelData header instead of a
  36+ byte Send indication.
* Refresh of the allocation (LIFETIME) and of permissions / channels (5 / 10 min
  lifetimes) in the background; ``close()`` releases the allocation (LIFETIME 0).
"""
from __future__ import annotations

import asyncio
import logging
import struct
from typing import Callable, Optional

from . import stun

log = logging.getLogger("webrtc.turn")

UDP = 17
PERMISSION_REFRESH_S = 240.0    # permissions live 300 s
CHANNEL_REFRESH_S = 540.0       # channel bindings live 600 s


def is_channel_data(data: bytes) -> bool:
    """RFC 7983: first byte 64..79 is TURN ChannelData."""
    return len(data) >= 4 and 64 <= data[0] <= 79


class TurnError(OSError):
    pass


class TurnAllocation:
    def __init__(self, server: tuple, username: str, password: str,
                 sendto: Callable[[bytes, tuple], None], lifetime: int = 600):
        self.server = server
        self.username, self.password = username, password
        self._sendto = sendto
        self.lifetime = lifetime
        self.realm: Optional[str] = None
        self.nonce: Optional[str] = None
        self.key: Optional[bytes] = None
        self.relayed: Optional[tuple] = None
        self.mapped: Optional[tuple] = None
        self.permissions: dict = {}     # peer ip -> last refresh (loop time)
        self.channels: dict = {}        # peer (ip, port) -> channel number
        self.bound_at: dict = {}        # peer (ip, port) -> last ChannelBind (loop time)
        self.permission_refresh_s = PERMISSION_REFRESH_S
        self.channel_refresh_s = CHANNEL_REFRESH_S
        self.peers_by_channel: dict = {}
        self._next_channel = 0x4000
        self._pending: dict = {}
        self._tasks: list = []
        self.on_data: Callable[[bytes, tuple], None] = lambda data, peer: None

    # -- transactions -----------------------------------------------------------------
    async def _transact(self, msg: stun.Message, auth: bool, retries: int = 5, interval: float = 0.2):
        if auth:
            msg.attrs[stun.USERNAME] = self.username
            msg.attrs[stun.REALM] = self.realm
            msg.attrs[stun.NONCE] = self.nonce
        data = msg.encode(self.key if auth else None)
        fut = asyncio.get_running_loop().create_future()
        self._pending[msg.tid] = fut
        try:
            for i in range(retries):
                self._sendto(data, self.server)
                try:
                    return await asyncio.wait_for(asyncio.shield(fut), interval * (2 ** min(i, 3)))
                except asyncio.TimeoutError:
                    continue
            raise asyncio.TimeoutError(f"TURN server {self.server} did not answer")
        finally:
            self._pending.pop(msg.tid, None)

    async def _authed(self, make: Callable[[], stun.Message]) -> stun.Message:
        """Sends an authenticated request; refreshes the nonce on 438 (once)."""
        for attempt in range(2):
            res = await self._transact(make(), auth=True)
            if res.cls == stun.SUCCESS:
                return res
            code = res.attrs.get(stun.ERROR_CODE, (0, ""))[0]
            if code == 438 and attempt == 0 and stun.NONCE in res.attrs:
                self.nonce = res.attrs[stun.NONCE]
                continue
            raise TurnError(f"TURN request failed: {res.attrs.get(stun.ERROR_CODE)}")
        raise TurnError("TURN stale nonce")

    # -- allocation ------------------------------------------------------------------------
    async def allocate(self) -> tuple:
        def req():
            m = stun.Message(stun.ALLOCATE, stun.REQUEST)
            m.attrs[stun.REQUESTED_TRANSPORT] = UDP
            m.attrs[stun.LIFETIME] = self.lifetime
            return m
        res = await self._transact(req(), auth=False)
        if res.cls == stun.ERROR:
            code = res.attrs.get(stun.ERROR_CODE, (0, ""))[0]
            if code != 401 or stun.REALM not in res.attrs or stun.NONCE not in res.attrs:
                raise TurnError(f"TURN allocate refused: {res.attrs.get(stun.ERROR_CODE)}")
            self.realm, self.nonce = res.attrs[stun.REALM], res.attrs[stun.NONCE]
            self.key = stun.long_term_key(self.username, self.realm, self.password)
            res = await self._authed(req)
        self.relayed = res.attrs.get(stun.XOR_RELAYED_ADDRESS)
        self.mapped = res.attrs.get(stun.XOR_MAPPED_ADDRESS)
        self.lifetime = res.attrs.get(stun.LIFETIME, self.lifetime)
        if self.relayed is None:
            raise TurnError("TURN allocate response without XOR-RELAYED-ADDRESS")
        self._tasks.append(asyncio.ensure_future(self._refresh_loop()))
        log.info("TURN allocation %s:%d via %s:%d", *self.relayed, *self.server)
        return self.relayed

    async def _refresh_loop(self) -> None:
        loop = asyncio.get_running_loop()
        last_alloc = loop.time()
        while True:
            await asyncio.sleep(min(30.0, max(0.05, self.lifetime / 4), self.permission_refresh_s / 4,
                                    self.channel_refresh_s / 4))
            now = loop.time()
            try:
                if now - last_alloc > max(1.0, self.lifetime - 60):
                    await self._authed(lambda: self._refresh_msg(self.lifetime))
                    last_alloc = now
                # a binding's age is its own: permission refreshes do not renew a
                # channel (RFC 5766 §11), and a binding that lapses after 600 s
                # takes the relayed media and ICE keepalives with it
                for peer, ch in list(self.channels.items()):
                    if now - self.bound_at.get(peer, 0) > self.channel_refresh_s:
                        await self._bind(peer, ch)
                for ip, t in list(self.permissions.items()):
                    if now - t > self.permission_refresh_s:
                        await self.create_permission(ip)
            except (OSError, asyncio.TimeoutError) as e:
                log.warning("TURN refresh failed: %s", e)

    def _refresh_msg(self, lifetime: int) -> stun.Message:
        m = stun.Message(stun.REFRESH, stun.REQUEST)
        m.attrs[stun.LIFETIME] = lifetime
        return m

    async def create_permission(self, ip: str) -> None:
        def req():
            m = stun.Message(stun.CREATE_PERMISSION, stun.REQUEST)
            m.attrs[stun.XOR_PEER_ADDRESS] = (ip, 0)
            return m
        await self._authed(req)
        self.permissions[ip] = asyncio.get_running_loop().time()

    async def _bind(self, peer: tuple, ch: int) -> None:
        def req():
            m = stun.Message(stun.CHANNEL_BIND, stun.REQUEST)
            m.attrs[stun.CHANNEL_NUMBER] = ch
            m.attrs[stun.XOR_PEER_ADDRESS] = peer
            return m
        await self._authed(req)
        now = asyncio.get_running_loop().time()
        self.bound_at[peer] = now
        self.permissions[peer[0]] = now    # a ChannelBind installs/refreshes the peer's permission too

    async def channel_bind(self, peer: tuple) -> int:
        peer = (peer[0], peer[1])
        if peer in self.channels:
            return self.channels[peer]
        ch = self._next_channel
        self._next_channel += 1
        await self._bind(peer, ch)
        self.channels[peer] = ch
        self.peers_by_channel[ch] = peer
        return ch

    # -- data ------------------------------------------------------------------------------------
    def send_to(self, peer: tuple, data: bytes) -> None:
        ch = self.channels.get((peer[0], peer[1]))
        if ch is not None:
            self._sendto(struct.pack("!HH", ch, len(data)) + data, self.server)
            return
        m = stun.Message(stun.SEND, stun.INDICATION)
        m.attrs[stun.XOR_PEER_ADDRESS] = (peer[0], peer[1])
        m.attrs[stun.DATA_ATTR] = data
        self._sendto(m.encode(None, fingerprint=False), self.server)

    def on_datagram(self, data: bytes) -> Optional[tuple]:
        """A datagram from the TURN server. Returns (payload, peer) for relayed data,
        None for transaction responses (resolved here) and garbage."""
        if is_channel_data(data):
            ch, ln = struct.unpack_from("!HH", data, 0)
            peer = self.peers_by_channel.get(ch)
            return (data[4:4 + ln], peer) if peer is not None and 4 + ln <= len(data) else None
        try:
            msg, offs = stun.decode(data)
        except stun.StunError:
            return None
        if msg.method == stun.DATA and msg.cls == stun.INDICATION:
            peer, payload = msg.attrs.get(stun.XOR_PEER_ADDRESS), msg.attrs.get(stun.DATA_ATTR)
            return (payload, peer) if peer is not None and payload is not None else None
        fut = self._pending.get(msg.tid)
        if fut is None or fut.done():
            return None
        if msg.cls == stun.SUCCESS and self.key is not None and not stun.check_integrity(data, offs, self.key):
            return None   # forged success
        fut.set_result(msg)
        return None

    async def close(self) -> None:
        for t in self._tasks:
            t.cancel()
        if self.key is not None and self.relayed is not None:
            try:
                await asyncio.wait_for(self._authed(lambda: self._refresh_msg(0)), 1.0)
            except (OSError, asyncio.TimeoutError):
                pass
        self.relayed = None


def parse_turn_url(url: str) -> Optional[tuple]:
    """``turn://user:pass@host:port[?transport=udp]`` (the form server/turn.py's
    parse_rtc_config produces) -> (host, port, user, password); None for TCP/TLS TURN,
    which this UDP client does not speak."""
    if not url.startswith(("turn://", "turn:")):
        return None
    rest = url.split("://", 1)[1] if "://" in url else url.split(":", 1)[1]
    rest, _, query = rest.partition("?")
    if "transport=tcp" in query:
        return None
    cred, _, hostport = rest.rpartition("@")
    user, _, pwd = cred.partition(":")
    host, _, port = hostport.rpartition(":")
    if not host:
        host, port = hostport, "3478"
    return host, int(port), user, pwd
