"""SCTP over DTLS (RFC 8261) with WebRTC data channels (RFC 8831/8832).

Reference equivalents: webrtcbin's usrsctp data channels used for input and
stats (legacy/gstwebrtc_app.py:1481-1496) and the vendored aiortc
``RTCSctpTransport``/``RTCDataChannel`` (webrtc/rtcsctptransport.py,
webrtc/rtcdatachannel.py). This is a compact association for one DTLS
transport:

* four-way handshake (INIT / INIT-ACK + cookie / COOKIE-ECHO / COOKIE-ACK),
  T1 retransmission, CRC32c from the native core;
* reliable delivery: TSNs, SACK with gap blocks and duplicate reports, T3
  retransmission with RTT-based RTO (RFC 4960 §6.3), fast retransmit after
  three miss indications, a receive window and an outstanding-bytes limit;
* message fragmentation / reassembly (B/E flags), ordered and unordered
  delivery, FORWARD-TSN acceptance;
* DCEP open/ack, string/binary/empty PPIDs, stream reset (RE-CONFIG) on close;
* HEARTBEAT answering, SHUTDOWN / ABORT handling.

Partial reliability requested by a peer is accepted and served reliably
(a superset of the guarantee).
"""
from __future__ import annotations

import asyncio
import logging
import os
import struct
import time
from typing import Callable, Optional

from .native import crc32c

log = logging.getLogger("webrtc.sctp")

# chunk types
DATA, INIT, INIT_ACK, SACK, HEARTBEAT, HEARTBEAT_ACK, ABORT, SHUTDOWN, SHUTDOWN_ACK, ERROR_CHUNK, \
    COOKIE_ECHO, COOKIE_ACK = 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11
SHUTDOWN_COMPLETE, RECONFIG, FORWARD_TSN = 14, 130, 192
# parameters
STATE_COOKIE = 7
FORWARD_TSN_SUPPORTED = 0xC000
SUPPORTED_EXTENSIONS = 0x8008
OUTGOING_RESET_REQUEST = 13
RECONFIG_RESPONSE = 16
# payload protocol identifiers
PPID_DCEP, PPID_STRING, PPID_BINARY, PPID_STRING_EMPTY, PPID_BINARY_EMPTY = 50, 51, 53, 56, 57
DCEP_OPEN, DCEP_ACK = 0x03, 0x02

MTU = 1200
MAX_DATA = MTU - 12 - 16 - 16   # common header, DATA chunk header, slack for bundling
RWND = 1 << 20
MAX_OUTSTANDING = 1 << 20


def _tsn_gt(a: int, b: int) -> bool:
    return a != b and ((a - b) & 0xFFFFFFFF) < 0x80000000


def _tsn_ge(a: int, b: int) -> bool:
    return a == b or _tsn_gt(a, b)


def _chunk(ctype: int, flags: int, body: bytes) -> bytes:
    n = 4 + len(body)
    return struct.pack("!BBH", ctype, flags, n) + body + b"\x00" * ((4 - n % 4) % 4)


def _param(ptype: int, body: bytes) -> bytes:
    n = 4 + len(body)
    return struct.pack("!HH", ptype, n) + body + b"\x00" * ((4 - n % 4) % 4)


def _params(data: bytes):
    pos = 0
    while pos + 4 <= len(data):
        t, n = struct.unpack_from("!HH", data, pos)
        if n < 4:
            return
        yield t, data[pos + 4:pos + n]
        pos += n + (4 - n % 4) % 4


def parse_packet(data: bytes):
    """(src_port, dst_port, vtag, [(type, flags, body)]) or None on a bad checksum."""
    if len(data) < 12:
        return None
    sp, dp, vtag, ck = struct.unpack_from("!HHII", data, 0)
    ck = struct.unpack_from("<I", data, 8)[0]
    if crc32c(data[:8] + b"\x00\x00\x00\x00" + data[12:]) != ck:
        return None
    chunks, pos = [], 12
    while pos + 4 <= len(data):
        t, f, n = struct.unpack_from("!BBH", data, pos)
        if n < 4 or pos + n > len(data):
            break
        chunks.append((t, f, data[pos + 4:pos + n]))
        pos += n + (4 - n % 4) % 4
    return sp, dp, vtag, chunks


class DataChannel:
    def __init__(self, assoc: "SctpAssociation", stream_id: int, label: str, ordered: bool = True,
                 protocol: str = ""):
        self._assoc = assoc
        self.id = stream_id
        self.label = label
        self.ordered = ordered
        self.protocol = protocol
        self.ready_state = "connecting"
        self.on_message: Callable[[object], None] = lambda m: None
        self.on_open: Callable[[], None] = lambda: None
        self.on_close: Callable[[], None] = lambda: None
        self.bytes_sent = 0
        self.messages_sent = 0

    def send(self, data) -> None:
        if self.ready_state != "open":
            raise ConnectionError(f"data channel {self.label!r} is {self.ready_state}")
        if isinstance(data, str):
            raw = data.encode()
            ppid = PPID_STRING if raw else PPID_STRING_EMPTY
        else:
            raw = bytes(data)
            ppid = PPID_BINARY if raw else PPID_BINARY_EMPTY
        self._assoc._send_user(self.id, ppid, raw or b"\x00", self.ordered)
        self.bytes_sent += len(raw)
        self.messages_sent += 1

    def close(self) -> None:
        if self.ready_state in ("closing", "closed"):
            return
        self.ready_state = "closing"
        self._assoc._reset_stream(self.id)

    def _opened(self) -> None:
        if self.ready_state == "connecting":
            self.ready_state = "open"
            self.on_open()

    def _closed(self) -> None:
        if self.ready_state != "closed":
            self.ready_state = "closed"
            self.on_close()


class SctpAssociation:
    def __init__(self, send: Callable[[bytes], None], is_client: bool, port: int = 5000, remote_port: int = 5000):
        self._send_raw = send
        self.is_client = is_client
        self.port, self.remote_port = port, remote_port
        self.state = "closed"   # closed, cookie-wait, cookie-echoed, established, shutdown
        self.local_vtag = struct.unpack("!I", os.urandom(4))[0] or 1
        self.remote_vtag = 0
        self.local_tsn = struct.unpack("!I", os.urandom(4))[0]
        self.remote_cum_tsn: Optional[int] = None
        self.peer_rwnd = RWND
        self.channels: dict[int, DataChannel] = {}
        self.on_datachannel: Callable[[DataChannel], None] = lambda ch: None
        self.on_established: Callable[[], None] = lambda: None
        self._next_stream = 0 if is_client else 1   # RFC 8832 §6: DTLS client even, server odd
        self._ssn: dict[int, int] = {}
        self._cookie = os.urandom(16)
        self._init_chunk: Optional[bytes] = None
        self._cookie_echo: Optional[bytes] = None
        self._t1: Optional[asyncio.TimerHandle] = None
        self._t1_tries = 0
        # sending
        self._queue: list = []                   # (stream, ppid, flags, ssn, payload) not yet assigned a TSN
        self._sent: dict[int, list] = {}         # tsn -> [chunk bytes, sent time, tries, misses, size]
        self._outstanding = 0
        self._t3: Optional[asyncio.TimerHandle] = None
        self._srtt: Optional[float] = None
        self._rttvar = 0.0
        self.rto = 1.0
        # receiving
        self._received: dict[int, tuple] = {}    # tsn -> (flags, stream, ssn, ppid, data) above cum
        self._dups: list = []
        self._frag: dict = {}                    # (stream, ordered) -> [ppid, parts]
        self._reconfig_seq = struct.unpack("!I", os.urandom(4))[0]
        self._established = asyncio.Event()
        self.stats = {"packets_in": 0, "packets_out": 0, "retransmits": 0, "messages_in": 0}

    # -- packets ------------------------------------------------------------------------
    def _packet(self, chunks: list, vtag: Optional[int] = None) -> None:
        body = b"".join(chunks)
        hdr = struct.pack("!HHI", self.port, self.remote_port, self.remote_vtag if vtag is None else vtag)
        data = hdr + b"\x00\x00\x00\x00" + body
        data = hdr + struct.pack("<I", crc32c(data)) + body
        self.stats["packets_out"] += 1
        self._send_raw(data)

    def _loop(self):
        return asyncio.get_event_loop()

    # -- association setup -----------------------------------------------------------------
    def start(self) -> None:
        if not self.is_client:
            return  # wait for the peer's INIT (both sides may still initiate; we answer either way)
        body = struct.pack("!IIHHI", self.local_vtag, RWND, 65535, 65535, self.local_tsn)
        body += _param(FORWARD_TSN_SUPPORTED, b"") + _param(SUPPORTED_EXTENSIONS, bytes([FORWARD_TSN, RECONFIG]))
        self._init_chunk = _chunk(INIT, 0, body)
        self.state = "cookie-wait"
        self._t1_tries = 0
        self._send_t1()

    def _send_t1(self) -> None:
        if self.state == "cookie-wait" and self._init_chunk:
            self._packet([self._init_chunk], vtag=0)
        elif self.state == "cookie-echoed" and self._cookie_echo:
            self._packet([self._cookie_echo])
        else:
            return
        self._t1_tries += 1
        if self._t1_tries < 10:
            self._t1 = self._loop().call_later(min(1.0 * 2 ** (self._t1_tries - 1), 8.0), self._send_t1)

    async def wait_established(self, timeout: float = 10.0) -> None:
        await asyncio.wait_for(self._established.wait(), timeout)

    def _set_established(self) -> None:
        if self.state != "established":
            self.state = "established"
            if self._t1:
                self._t1.cancel()
            self._established.set()
            self.on_established()
            self._flush()

    # -- input -------------------------------------------------------------------------------
    def feed(self, data: bytes) -> None:
        p = parse_packet(data)
        if p is None:
            return
        sp, dp, vtag, chunks = p
        self.stats["packets_in"] += 1
        got_data = False
        for t, f, body in chunks:
            if t == INIT:
                self._on_init(body)
            elif vtag != self.local_vtag and t not in (ABORT, SHUTDOWN_COMPLETE):
                return  # not for this association (RFC 4960 §8.5)
            elif t == INIT_ACK:
                self._on_init_ack(body)
            elif t == COOKIE_ECHO:
                if body[:16] == self._cookie:
                    self._packet([_chunk(COOKIE_ACK, 0, b"")])
                    self._set_established()
            elif t == COOKIE_ACK:
                if self.state == "cookie-echoed":
                    self._set_established()
            elif t == DATA:
                got_data = True
                self._on_data(f, body)
            elif t == SACK:
                self._on_sack(body)
            elif t == HEARTBEAT:
                self._packet([_chunk(HEARTBEAT_ACK, 0, body)])
            elif t == FORWARD_TSN:
                self._on_forward_tsn(body)
            elif t == RECONFIG:
                self._on_reconfig(body)
            elif t == SHUTDOWN:
                self._packet([_chunk(SHUTDOWN_ACK, 0, b"")])
                self._close_all()
            elif t == SHUTDOWN_ACK:
                self._packet([_chunk(SHUTDOWN_COMPLETE, 0, b"")])
                self._close_all()
            elif t == ABORT:
                log.info("SCTP association aborted by peer")
                self._close_all()
        if got_data:
            self._deliver()
            self._send_sack()

    def _on_init(self, body: bytes) -> None:
        tag, rwnd, _os, _is, tsn = struct.unpack_from("!IIHHI", body, 0)
        self.remote_vtag, self.peer_rwnd = tag, rwnd
        self.remote_cum_tsn = (tsn - 1) & 0xFFFFFFFF
        ack = struct.pack("!IIHHI", self.local_vtag, RWND, 65535, 65535, self.local_tsn)
        ack += _param(STATE_COOKIE, self._cookie) + _param(FORWARD_TSN_SUPPORTED, b"")
        ack += _param(SUPPORTED_EXTENSIONS, bytes([FORWARD_TSN, RECONFIG]))
        self._packet([_chunk(INIT_ACK, 0, ack)])

    def _on_init_ack(self, body: bytes) -> None:
        if self.state != "cookie-wait":
            return
        tag, rwnd, _os, _is, tsn = struct.unpack_from("!IIHHI", body, 0)
        self.remote_vtag, self.peer_rwnd = tag, rwnd
        self.remote_cum_tsn = (tsn - 1) & 0xFFFFFFFF
        cookie = next((v for t, v in _params(body[16:]) if t == STATE_COOKIE), None)
        if cookie is None:
            return
        if self._t1:
            self._t1.cancel()
        self._cookie_echo = _chunk(COOKIE_ECHO, 0, cookie)
        self.state = "cookie-echoed"
        self._t1_tries = 0
        self._send_t1()

    # -- receive path -----------------------------------------------------------------------
    def _on_data(self, flags: int, body: bytes) -> None:
        if len(body) < 12 or self.remote_cum_tsn is None:
            return
        tsn, stream, ssn, ppid = struct.unpack_from("!IHHI", body, 0)
        if not _tsn_gt(tsn, self.remote_cum_tsn) or tsn in self._received:
            self._dups.append(tsn)
            return
        self._received[tsn] = (flags, stream, ssn, ppid, body[12:])

    def _deliver(self) -> None:
        while True:
            nxt = (self.remote_cum_tsn + 1) & 0xFFFFFFFF
            item = self._received.pop(nxt, None)
            if item is None:
                return
            self.remote_cum_tsn = nxt
            flags, stream, _ssn, ppid, data = item
            key = (stream, not (flags & 0x04))
            if flags & 0x02:  # B
                self._frag[key] = [ppid, [data]]
            elif key in self._frag:
                self._frag[key][1].append(data)
            else:
                continue  # middle of a message whose start was abandoned (FORWARD-TSN)
            if flags & 0x01:  # E
                ppid, parts = self._frag.pop(key)
                self._on_message(stream, ppid, b"".join(parts))

    def _send_sack(self) -> None:
        cum = self.remote_cum_tsn
        gaps, start, prev = [], None, None
        for tsn in sorted(self._received, key=lambda t: (t - cum) & 0xFFFFFFFF):
            off = (tsn - cum) & 0xFFFFFFFF
            if start is None:
                start = prev = off
            elif off == prev + 1:
                prev = off
            else:
                gaps.append((start, prev))
                start = prev = off
        if start is not None:
            gaps.append((start, prev))
        gaps = gaps[:64]
        dups, self._dups = self._dups[:32], []
        body = struct.pack("!IIHH", cum, RWND, len(gaps), len(dups))
        body += b"".join(struct.pack("!HH", a, b) for a, b in gaps)
        body += b"".join(struct.pack("!I", d) for d in dups)
        self._packet([_chunk(SACK, 0, body)])

    def _on_forward_tsn(self, body: bytes) -> None:
        new_cum = struct.unpack_from("!I", body, 0)[0]
        if self.remote_cum_tsn is None or not _tsn_gt(new_cum, self.remote_cum_tsn):
            return
        for tsn in list(self._received):
            if _tsn_ge(new_cum, tsn):
                del self._received[tsn]
        self.remote_cum_tsn = new_cum
        self._frag.clear()
        self._deliver()
        self._send_sack()

    def _on_message(self, stream: int, ppid: int, data: bytes) -> None:
        self.stats["messages_in"] += 1
        if ppid == PPID_DCEP:
            self._on_dcep(stream, data)
            return
        ch = self.channels.get(stream)
        if ch is None:
            return
        if ppid in (PPID_STRING, 52):
            msg = data.decode("utf-8", "replace")
        elif ppid == PPID_STRING_EMPTY:
            msg = ""
        elif ppid == PPID_BINARY_EMPTY:
            msg = b""
        else:
            msg = data
        ch.on_message(msg)

    def _on_dcep(self, stream: int, data: bytes) -> None:
        if not data:
            return
        if data[0] == DCEP_OPEN and len(data) >= 12:
            ctype, _prio, _rel, llen, plen = struct.unpack_from("!BHIHH", data, 1)
            label = data[12:12 + llen].decode("utf-8", "replace")
            proto = data[12 + llen:12 + llen + plen].decode("utf-8", "replace")
            ch = DataChannel(self, stream, label, ordered=not (ctype & 0x80), protocol=proto)
            self.channels[stream] = ch
            self._send_user(stream, PPID_DCEP, bytes([DCEP_ACK]), True)
            ch.ready_state = "open"
            self.on_datachannel(ch)
            ch.on_open()
        elif data[0] == DCEP_ACK:
            ch = self.channels.get(stream)
            if ch:
                ch._opened()

    def _on_reconfig(self, body: bytes) -> None:
        for t, v in _params(body):
            if t == OUTGOING_RESET_REQUEST and len(v) >= 12:
                req_seq = struct.unpack_from("!I", v, 0)[0]
                streams = [struct.unpack_from("!H", v, i)[0] for i in range(12, len(v) - 1, 2)]
                self._packet([_chunk(RECONFIG, 0, _param(RECONFIG_RESPONSE, struct.pack("!II", req_seq, 1)))])
                for s in streams or list(self.channels):
                    ch = self.channels.pop(s, None)
                    self._ssn.pop(s, None)
                    if ch:
                        ch._closed()
            elif t == RECONFIG_RESPONSE:
                pass

    # -- send path ---------------------------------------------------------------------------
    def create_channel(self, label: str, ordered: bool = True, protocol: str = "") -> DataChannel:
        sid = self._next_stream
        self._next_stream += 2
        ch = DataChannel(self, sid, label, ordered, protocol)
        self.channels[sid] = ch
        lb, pb = label.encode(), protocol.encode()
        msg = struct.pack("!BBHIHH", DCEP_OPEN, 0x00 if ordered else 0x80, 0, 0, len(lb), len(pb)) + lb + pb
        self._send_user(sid, PPID_DCEP, msg, True)
        return ch

    def _send_user(self, stream: int, ppid: int, data: bytes, ordered: bool) -> None:
        if ordered:
            ssn = self._ssn.get(stream, 0)
            self._ssn[stream] = (ssn + 1) & 0xFFFF
        else:
            ssn = 0
        u = 0 if ordered else 0x04
        n = len(data)
        for off in range(0, max(n, 1), MAX_DATA):
            flags = u | (0x02 if off == 0 else 0) | (0x01 if off + MAX_DATA >= n else 0)
            self._queue.append((stream, ppid, flags, ssn, data[off:off + MAX_DATA]))
        self._flush()

    def _flush(self) -> None:
        if self.state != "established":
            return
        chunks, size = [], 12
        limit = min(self.peer_rwnd, MAX_OUTSTANDING)
        while self._queue and self._outstanding < limit:
            stream, ppid, flags, ssn, payload = self._queue.pop(0)
            tsn = self.local_tsn
            self.local_tsn = (self.local_tsn + 1) & 0xFFFFFFFF
            ch = _chunk(DATA, flags, struct.pack("!IHHI", tsn, stream, ssn, ppid) + payload)
            self._sent[tsn] = [ch, time.monotonic(), 1, 0, len(payload)]
            self._outstanding += len(payload)
            if size + len(ch) > MTU and chunks:
                self._packet(chunks)
                chunks, size = [], 12
            chunks.append(ch)
            size += len(ch)
        if chunks:
            self._packet(chunks)
        self._arm_t3()

    def _arm_t3(self) -> None:
        if self._t3:
            self._t3.cancel()
            self._t3 = None
        if self._sent:
            self._t3 = self._loop().call_later(self.rto, self._on_t3)

    def _on_t3(self) -> None:
        self._t3 = None
        if not self._sent:
            return
        self.rto = min(self.rto * 2, 60.0)
        self._retransmit(sorted(self._sent, key=lambda t: (t - self.local_tsn) & 0xFFFFFFFF))
        self._arm_t3()

    def _retransmit(self, tsns) -> None:
        chunks, size = [], 12
        for tsn in tsns:
            ent = self._sent.get(tsn)
            if ent is None:
                continue
            ent[1] = time.monotonic()
            ent[2] += 1
            ent[3] = 0
            self.stats["retransmits"] += 1
            if size + len(ent[0]) > MTU and chunks:
                self._packet(chunks)
                chunks, size = [], 12
            chunks.append(ent[0])
            size += len(ent[0])
        if chunks:
            self._packet(chunks)

    def _on_sack(self, body: bytes) -> None:
        cum, rwnd, ngap, _ndup = struct.unpack_from("!IIHH", body, 0)
        self.peer_rwnd = rwnd
        now = time.monotonic()
        acked_any = False
        for tsn in list(self._sent):
            if _tsn_ge(cum, tsn):
                ent = self._sent.pop(tsn)
                self._outstanding -= ent[4]
                acked_any = True
                if ent[2] == 1:
                    self._rtt_sample(now - ent[1])
        highest = cum
        for i in range(ngap):
            a, b = struct.unpack_from("!HH", body, 12 + 4 * i)
            for off in range(a, b + 1):
                tsn = (cum + off) & 0xFFFFFFFF
                ent = self._sent.pop(tsn, None)
                if ent:
                    self._outstanding -= ent[4]
                highest = tsn if _tsn_gt(tsn, highest) else highest
        if ngap:  # fast retransmit: three miss indications (RFC 4960 §7.2.4)
            fast = []
            for tsn, ent in self._sent.items():
                if _tsn_gt(highest, tsn):
                    ent[3] += 1
                    if ent[3] == 3:
                        fast.append(tsn)
            if fast:
                self._retransmit(fast)
        if acked_any:
            self._arm_t3()
        self._flush()

    def _rtt_sample(self, r: float) -> None:
        if self._srtt is None:
            self._srtt, self._rttvar = r, r / 2
        else:
            self._rttvar = 0.75 * self._rttvar + 0.25 * abs(self._srtt - r)
            self._srtt = 0.875 * self._srtt + 0.125 * r
        self.rto = min(max(self._srtt + 4 * self._rttvar, 0.2), 60.0)

    def _reset_stream(self, stream: int) -> None:
        self._reconfig_seq = (self._reconfig_seq + 1) & 0xFFFFFFFF
        last = (self.local_tsn - 1) & 0xFFFFFFFF
        req = struct.pack("!IIIH", self._reconfig_seq, self._reconfig_seq, last, stream)
        if self.state == "established":
            self._packet([_chunk(RECONFIG, 0, _param(OUTGOING_RESET_REQUEST, req))])
        ch = self.channels.pop(stream, None)
        self._ssn.pop(stream, None)
        if ch:
            ch._closed()

    def _close_all(self) -> None:
        self.state = "closed"
        for t in (self._t1, self._t3):
            if t:
                t.cancel()
        for ch in list(self.channels.values()):
            ch._closed()
        self.channels.clear()

    def close(self) -> None:
        if self.state == "established":
            self._packet([_chunk(ABORT, 0, b"")])
        self._close_all()
