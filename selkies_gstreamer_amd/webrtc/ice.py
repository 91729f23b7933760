"""ICE agent (RFC 8445 subset) on one asyncio UDP socket.

Role in the reference: webrtcbin/libnice (legacy/gstwebrtc_app.py) or aioice
under the vendored aiortc (webrtc/rtcicetransport.py:1-410). Scope here:

* host candidates for the configured / discovered local addresses, plus a
  server-reflexive candidate from a STUN server when one is configured
  (the RTC config of server/turn.py);
* connectivity checks for every candidate pair with retransmission, short-term
  credentials (USERNAME ``remote:local``, MESSAGE-INTEGRITY with the remote
  password) and FINGERPRINT; role conflict is resolved by tie-breaker;
* aggressive nomination when controlling (USE-CANDIDATE on every check, the
  first pair that succeeds is selected); when controlled the pair the peer
  nominates is selected;
* ``lite=True`` answers checks only (RFC 8445 §2.5 — a server on a public
  address);
* consent freshness (RFC 7675): a check every 5 s on the selected pair, the
  connection is failed after 30 s without any valid packet.

RFC 7983 demultiplexing: STUN stays in the agent, every other datagram
(DTLS 20-63, RTP/RTCP 128-191) goes to ``on_packet``.
Relayed candidates: with a TURN server configured (``turn_server=(host, port,
user, password)``, from the RTC config's iceServers) the agent allocates a relay on
its own socket (turn_client.TurnAllocation) and offers a ``relay`` candidate; every
remote candidate then gets a direct pair and a relayed pair (checks, responses and
media travel as Send/Data indications, then ChannelData once the selected peer is
channel-bound). ``relay_only=True`` is the iceTransportPolicy "relay": only the
relay candidate is offered and only relayed pairs are checked.
"""
from __future__ import annotations

import asyncio
import ipaddress
import logging
import random
import secrets
import socket
import string
import time
from dataclasses import dataclass
from typing import Callable, Optional

from . import stun
from .turn_client import TurnAllocation

log = logging.getLogger("webrtc.ice")

TYPE_PREF = {"host": 126, "prflx": 110, "srflx": 100, "relay": 0}


def random_string(n: int) -> str:
    alphabet = string.ascii_letters + string.digits + "+/"
    return "".join(secrets.choice(alphabet) for _ in range(n))


def candidate_priority(typ: str, local_pref: int = 65535, component: int = 1) -> int:
    return (TYPE_PREF[typ] << 24) | (local_pref << 8) | (256 - component)


@dataclass
class Candidate:
    foundation: str
    component: int
    transport: str
    priority: int
    host: str
    port: int
    type: str
    related_address: Optional[str] = None
    related_port: Optional[int] = None

    def to_sdp(self) -> str:
        s = (f"{self.foundation} {self.component} {self.transport} {self.priority} {self.host} {self.port} "
             f"typ {self.type}")
        if self.related_address is not None:
            s += f" raddr {self.related_address} rport {self.related_port}"
        return s

    @classmethod
    def from_sdp(cls, line: str) -> "Candidate":
        if line.startswith("a="):
            line = line[2:]
        if line.startswith("candidate:"):
            line = line[len("candidate:"):]
        b = line.split()
        if len(b) < 8 or b[6] != "typ":
            raise ValueError(f"bad candidate: {line!r}")
        c = cls(b[0], int(b[1]), b[2].lower(), int(b[3]), b[4], int(b[5]), b[7])
        for i in range(8, len(b) - 1, 2):
            if b[i] == "raddr":
                c.related_address = b[i + 1]
            elif b[i] == "rport":
                c.related_port = int(b[i + 1])
        return c


def local_addresses() -> list[str]:
    """Non-loopback IPv4 addresses of this host (loopback if there is none)."""
    addrs = set()
    try:
        for info in socket.getaddrinfo(socket.gethostname(), None, socket.AF_INET):
            addrs.add(info[4][0])
    except OSError:
        pass
    try:  # the source address the kernel would use for a public destination (no packet is sent)
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.connect(("192.0.2.1", 9))
        addrs.add(s.getsockname()[0])
        s.close()
    except OSError:
        pass
    addrs = {a for a in addrs if not ipaddress.ip_address(a).is_loopback}
    return sorted(addrs) or ["127.0.0.1"]


class _Protocol(asyncio.DatagramProtocol):
    def __init__(self, agent: "IceAgent"):
        self.agent = agent

    def datagram_received(self, data, addr):
        self.agent._on_datagram(data, addr)

    def error_received(self, exc):
        log.debug("ice socket error: %s", exc)


@dataclass
class _Pair:
    remote: tuple
    priority: int
    state: str = "waiting"   # waiting, in-progress, succeeded, failed
    nominated: bool = False
    relayed: bool = False    # local side is the TURN relay candidate


class IceAgent:
    def __init__(self, controlling: bool, lite: bool = False, addresses: Optional[list[str]] = None,
                 port: int = 0, stun_server: Optional[tuple] = None, turn_server: Optional[tuple] = None,
                 relay_only: bool = False):
        self.controlling = controlling and not lite
        self.lite = lite
        self.local_ufrag = random_string(4)
        self.local_pwd = random_string(22)
        self.remote_ufrag: Optional[str] = None
        self.remote_pwd: Optional[str] = None
        self.tie_breaker = random.getrandbits(64)
        self.addresses = addresses
        self.port = port
        self.stun_server = stun_server
        self.turn_server = turn_server
        self.relay_only = relay_only
        self.turn: Optional[TurnAllocation] = None
        self.local_candidates: list[Candidate] = []
        self.remote_candidates: list[Candidate] = []
        self.pairs: dict = {}
        self.selected: Optional[tuple] = None
        self.selected_relayed = False
        self.state = "new"   # new, checking, connected, failed, closed
        self.on_packet: Callable[[bytes, tuple], None] = lambda data, addr: None
        self.on_state: Callable[[str], None] = lambda st: None
        self._transport = None
        self._pending: dict = {}
        self._connected = asyncio.Event()
        self._tasks: list = []
        self._last_rx = time.monotonic()
        self._remote_done = False

    # -- gathering --------------------------------------------------------------
    async def gather(self) -> list[Candidate]:
        loop = asyncio.get_running_loop()
        self._transport, _ = await loop.create_datagram_endpoint(lambda: _Protocol(self),
                                                                 local_addr=("0.0.0.0", self.port))
        port = self._transport.get_extra_info("sockname")[1]
        for i, addr in enumerate(self.addresses or local_addresses()):
            self.local_candidates.append(Candidate(str(1 + i), 1, "udp", candidate_priority("host", 65535 - i),
                                                   addr, port, "host"))
        if self.stun_server:
            try:
                srv = await self._resolve(self.stun_server[0], int(self.stun_server[1]))
                res = await self._request(srv, stun.Message(stun.BINDING, stun.REQUEST), None,
                                          retries=3, interval=0.2)
                mapped = res.attrs.get(stun.XOR_MAPPED_ADDRESS)
                if mapped and all(mapped[0] != c.host for c in self.local_candidates):
                    base = self.local_candidates[0]
                    self.local_candidates.append(Candidate("srflx1", 1, "udp", candidate_priority("srflx"),
                                                           mapped[0], mapped[1], "srflx", base.host, base.port))
            except (asyncio.TimeoutError, OSError) as e:
                log.info("STUN server %s unreachable: %s", self.stun_server, e)
        if self.turn_server:
            host, tport, user, pwd = self.turn_server
            try:
                self.turn = TurnAllocation(await self._resolve(host, int(tport)), user, pwd, self._transport.sendto)
                relayed = await self.turn.allocate()
                mapped = self.turn.mapped or (self.local_candidates[0].host, port)
                self.local_candidates.append(Candidate("relay1", 1, "udp", candidate_priority("relay"), relayed[0],
                                                       relayed[1], "relay", mapped[0], mapped[1]))
            except (asyncio.TimeoutError, OSError) as e:
                log.warning("TURN server %s:%s unusable: %s", host, tport, e)
                self.turn = None
        if self.relay_only:
            if self.turn is None:
                raise ConnectionError("relay-only ICE policy without a TURN allocation")
            self.local_candidates = [c for c in self.local_candidates if c.type == "relay"]
        return self.local_candidates

    @staticmethod
    async def _resolve(host: str, port: int, timeout: float = 2.0) -> tuple:
        """IPv4 address of a STUN/TURN server without blocking the loop (a hostname handed
        to sendto would resolve synchronously); OSError when it does not resolve in time."""
        try:
            return (str(ipaddress.IPv4Address(host)), port)
        except ValueError:
            pass
        loop = asyncio.get_running_loop()
        try:
            infos = await asyncio.wait_for(loop.getaddrinfo(host, port, family=socket.AF_INET,
                                                            type=socket.SOCK_DGRAM), timeout)
        except asyncio.TimeoutError:
            raise OSError(f"cannot resolve {host}") from None
        return (infos[0][4][0], port)

    # -- remote description ---------------------------------------------------------
    def set_remote_credentials(self, ufrag: str, pwd: str) -> None:
        self.remote_ufrag, self.remote_pwd = ufrag, pwd

    def add_remote_candidate(self, c: Optional[Candidate]) -> None:
        """None marks end-of-candidates."""
        if c is None:
            self._remote_done = True
            return
        if c.transport != "udp" or c.component != 1:
            return
        try:
            ip = ipaddress.ip_address(c.host)
        except ValueError:
            return  # mDNS (.local) names cannot be resolved here
        if ip.version != 4:
            return
        self.remote_candidates.append(c)
        for relayed in ((True,) if self.relay_only else ((False, True) if self.turn else (False,))):
            key = (c.host, c.port, relayed)
            if key in self.pairs:
                continue
            cands = [lc for lc in self.local_candidates if (lc.type == "relay") == relayed]
            local = cands[0].priority if cands else 0
            g, d = (local, c.priority) if self.controlling else (c.priority, local)
            prio = (1 << 32) * min(g, d) + 2 * max(g, d) + (1 if g > d else 0)
            self.pairs[key] = _Pair((c.host, c.port), prio, relayed=relayed)
            if self.state == "checking" and not self.lite:
                self._tasks.append(asyncio.ensure_future(self._check(self.pairs[key])))

    # -- connectivity -------------------------------------------------------------
    async def connect(self, timeout: float = 30.0) -> None:
        self._set_state("checking")
        if not self.lite:
            for p in sorted(self.pairs.values(), key=lambda p: -p.priority):
                self._tasks.append(asyncio.ensure_future(self._check(p)))
        try:
            await asyncio.wait_for(self._connected.wait(), timeout)
        except asyncio.TimeoutError:
            self._set_state("failed")
            raise ConnectionError("ICE connectivity checks failed") from None
        self._tasks.append(asyncio.ensure_future(self._consent_loop()))

    async def _check(self, pair: _Pair) -> None:
        if self.remote_pwd is None:
            return
        pair.state = "in-progress"
        req = stun.Message(stun.BINDING, stun.REQUEST)
        req.attrs[stun.USERNAME] = f"{self.remote_ufrag}:{self.local_ufrag}"
        req.attrs[stun.PRIORITY] = candidate_priority("prflx")
        if self.controlling:
            req.attrs[stun.ICE_CONTROLLING] = self.tie_breaker
            req.attrs[stun.USE_CANDIDATE] = True
        else:
            req.attrs[stun.ICE_CONTROLLED] = self.tie_breaker
        try:
            if pair.relayed and pair.remote[0] not in self.turn.permissions:
                await self.turn.create_permission(pair.remote[0])
            await self._request(pair.remote, req, self.remote_pwd.encode(), retries=7, interval=0.1,
                                relayed=pair.relayed)
        except (asyncio.TimeoutError, OSError):
            pair.state = "failed"
            return
        pair.state = "succeeded"
        if self.controlling:
            pair.nominated = True
            self._select(pair.remote, pair.relayed)
        elif pair.nominated:
            self._select(pair.remote, pair.relayed)

    def _send(self, data: bytes, addr, relayed: bool) -> None:
        if relayed:
            if self.turn is not None:
                self.turn.send_to(addr, data)
        elif self._transport is not None:
            self._transport.sendto(data, addr)

    async def _request(self, addr, msg: stun.Message, key: Optional[bytes], retries: int, interval: float,
                       relayed: bool = False):
        fut = asyncio.get_running_loop().create_future()
        self._pending[msg.tid] = (fut, key)
        data = msg.encode(key)
        try:
            for i in range(retries):
                self._send(data, addr, relayed)
                try:
                    return await asyncio.wait_for(asyncio.shield(fut), interval * (2 ** min(i, 3)))
                except asyncio.TimeoutError:
                    continue
            raise asyncio.TimeoutError()
        finally:
            self._pending.pop(msg.tid, None)

    def _select(self, remote: tuple, relayed: bool = False) -> None:
        if self.selected is None:
            self.selected = remote
            self.selected_relayed = relayed
            log.info("ICE selected pair -> %s:%d%s", *remote, " (relayed)" if relayed else "")
            self._set_state("connected")
            self._connected.set()
            if relayed:   # media: 4-byte ChannelData instead of Send indications
                self._tasks.append(asyncio.ensure_future(self._bind_channel(remote)))

    async def _bind_channel(self, remote: tuple) -> None:
        try:
            await self.turn.channel_bind(remote)
        except (OSError, asyncio.TimeoutError) as e:
            log.info("TURN channel bind failed (staying on Send indications): %s", e)

    def _set_state(self, st: str) -> None:
        if st != self.state:
            self.state = st
            self.on_state(st)

    async def _consent_loop(self) -> None:
        while self.state == "connected":
            await asyncio.sleep(5.0)
            if time.monotonic() - self._last_rx > 30.0:
                log.warning("ICE consent expired")
                self._set_state("failed")
                return
            if not self.lite and self.selected and self.remote_pwd:
                req = stun.Message(stun.BINDING, stun.REQUEST)
                req.attrs[stun.USERNAME] = f"{self.remote_ufrag}:{self.local_ufrag}"
                req.attrs[stun.PRIORITY] = candidate_priority("prflx")
                req.attrs[stun.ICE_CONTROLLING if self.controlling else stun.ICE_CONTROLLED] = self.tie_breaker
                self._send(req.encode(self.remote_pwd.encode()), self.selected, self.selected_relayed)

    # -- datagrams --------------------------------------------------------------------
    def _on_datagram(self, data: bytes, addr, relayed: bool = False) -> None:
        if not relayed and self.turn is not None and addr[:2] == self.turn.server:
            got = self.turn.on_datagram(data)
            if got is not None:
                self._on_datagram(got[0], got[1], relayed=True)
            return
        if not stun.is_stun(data):
            if self.selected is not None and addr[:2] == self.selected[:2] and relayed == self.selected_relayed:
                self._last_rx = time.monotonic()
                self.on_packet(data, addr)
            elif self.selected is None and addr[:2] + (relayed,) in self.pairs:
                self.on_packet(data, addr)
            return
        try:
            msg, offs = stun.decode(data)
        except stun.StunError:
            return
        if not stun.check_fingerprint(data, offs):
            return
        if msg.cls in (stun.SUCCESS, stun.ERROR):
            ent = self._pending.get(msg.tid)
            if ent is None:
                return
            fut, key = ent
            if key is not None and not stun.check_integrity(data, offs, key):
                return
            self._last_rx = time.monotonic()
            if not fut.done():
                if msg.cls == stun.SUCCESS:
                    fut.set_result(msg)
                else:
                    fut.set_exception(OSError(f"STUN error {msg.attrs.get(stun.ERROR_CODE)}"))
            return
        if msg.method == stun.BINDING and msg.cls == stun.REQUEST:
            self._on_binding_request(msg, offs, data, addr, relayed)

    def _on_binding_request(self, msg: stun.Message, offs: dict, data: bytes, addr, relayed: bool = False) -> None:
        user = msg.attrs.get(stun.USERNAME, "")
        if not user.startswith(self.local_ufrag + ":") or not stun.check_integrity(data, offs,
                                                                                   self.local_pwd.encode()):
            self._reply_error(msg, addr, 401, "Unauthorized", relayed)
            return
        if self.relay_only and not relayed:
            return   # policy "relay": nothing reaches us except through the allocation
        # role conflict (RFC 8445 §7.3.1.1)
        if self.controlling and stun.ICE_CONTROLLING in msg.attrs:
            if self.tie_breaker >= msg.attrs[stun.ICE_CONTROLLING]:
                self._reply_error(msg, addr, 487, "Role Conflict", relayed)
                return
            self.controlling = False
        elif not self.controlling and stun.ICE_CONTROLLED in msg.attrs and not self.lite:
            if self.tie_breaker < msg.attrs[stun.ICE_CONTROLLED]:
                self._reply_error(msg, addr, 487, "Role Conflict", relayed)
                return
            self.controlling = True
        self._last_rx = time.monotonic()
        res = stun.Message(stun.BINDING, stun.SUCCESS, msg.tid)
        res.attrs[stun.XOR_MAPPED_ADDRESS] = addr[:2]
        self._send(res.encode(self.local_pwd.encode()), addr, relayed)
        key = addr[:2] + (relayed,)
        pair = self.pairs.get(key)
        if pair is None:  # peer-reflexive remote candidate
            pair = self.pairs[key] = _Pair(addr[:2], 0, relayed=relayed)
            if not self.lite and self.remote_pwd:
                self._tasks.append(asyncio.ensure_future(self._check(pair)))
        if stun.USE_CANDIDATE in msg.attrs and not self.controlling:
            pair.nominated = True
            if self.lite or pair.state == "succeeded":
                self._select(addr[:2], relayed)
            elif self.remote_pwd and pair.state != "in-progress":  # triggered check
                self._tasks.append(asyncio.ensure_future(self._check(pair)))

    def _reply_error(self, msg: stun.Message, addr, code: int, reason: str, relayed: bool = False) -> None:
        res = stun.Message(msg.method, stun.ERROR, msg.tid)
        res.attrs[stun.ERROR_CODE] = (code, reason)
        self._send(res.encode(None), addr, relayed)

    # -- data -----------------------------------------------------------------------------
    def send(self, data: bytes) -> None:
        if self.selected is not None:
            self._send(data, self.selected, self.selected_relayed)

    @property
    def local_port(self) -> int:
        return self._transport.get_extra_info("sockname")[1] if self._transport else 0

    async def close(self) -> None:
        self._set_state("closed")
        for t in self._tasks:
            t.cancel()
        if self.turn is not None:
            await self.turn.close()
            self.turn = None
        if self._transport:
            self._transport.close()
            self._transport = None
