"""Minimal in-process TURN server (RFC 5766 over UDP) for the relay tests.

Long-term credentials (401 challenge with REALM/NONCE, MESSAGE-INTEGRITY checked on
every authenticated request), one relay socket per allocation, permissions by peer
IP (data from peers without one is dropped, as a real server does), channel
bindings, Send/Data indications and ChannelData in both directions.
"""
from __future__ import annotations

import asyncio
import struct

from selkies_gstreamer_amd.webrtc import stun
from selkies_gstreamer_amd.webrtc.turn_client import is_channel_data


class _Relay(asyncio.DatagramProtocol):
    def __init__(self, server, client):
        self.server, self.client = server, client

    def datagram_received(self, data, addr):
        self.server._from_peer(self.client, data, addr)


class TurnStub(asyncio.DatagramProtocol):
    def __init__(self, users: dict, realm: str = "selkies.test"):
        self.requests: list = []
        self.users, self.realm, self.nonce = users, realm, "n0nce"
        self.allocs: dict = {}      # client addr -> {relay transport, perms, channels, peers_by_ch}
        self.transport = None
        self.relayed_packets = 0

    async def start(self, host="127.0.0.1"):
        loop = asyncio.get_running_loop()
        self.transport, _ = await loop.create_datagram_endpoint(lambda: self, local_addr=(host, 0))
        return self.transport.get_extra_info("sockname")[:2]

    def close(self):
        for a in self.allocs.values():
            a["relay"].close()
        if self.transport:
            self.transport.close()

    def _reply(self, req, cls, attrs, addr, key):
        m = stun.Message(req.method, cls, req.tid, attrs)
        self.transport.sendto(m.encode(key), addr)

    def datagram_received(self, data, addr):
        a = self.allocs.get(addr)
        if is_channel_data(data):
            if a:
                ch, ln = struct.unpack_from("!HH", data, 0)
                peer = a["peers_by_ch"].get(ch)
                if peer:
                    a["relay"].sendto(data[4:4 + ln], peer)
                    self.relayed_packets += 1
            return
        try:
            msg, offs = stun.decode(data)
        except stun.StunError:
            return
        if msg.method == stun.SEND and msg.cls == stun.INDICATION:
            peer = msg.attrs.get(stun.XOR_PEER_ADDRESS)
            if a and peer and peer[0] in a["perms"]:
                a["relay"].sendto(msg.attrs[stun.DATA_ATTR], peer)
                self.relayed_packets += 1
            return
        if msg.cls != stun.REQUEST:
            return
        user = msg.attrs.get(stun.USERNAME)
        if user not in self.users or stun.MESSAGE_INTEGRITY not in msg.attrs:
            self._reply(msg, stun.ERROR, {stun.ERROR_CODE: (401, "Unauthorized"), stun.REALM: self.realm,
                                          stun.NONCE: self.nonce}, addr, None)
            return
        key = stun.long_term_key(user, self.realm, self.users[user])
        if not stun.check_integrity(data, offs, key):
            self._reply(msg, stun.ERROR, {stun.ERROR_CODE: (401, "Unauthorized"), stun.REALM: self.realm,
                                          stun.NONCE: self.nonce}, addr, None)
            return
        asyncio.ensure_future(self._handle(msg, addr, key))

    async def _handle(self, msg, addr, key):
        self.requests.append(msg.method)
        a = self.allocs.get(addr)
        if msg.method == stun.ALLOCATE:
            if a is None:
                loop = asyncio.get_running_loop()
                relay, _ = await loop.create_datagram_endpoint(lambda: _Relay(self, addr), local_addr=("127.0.0.1", 0))
                a = self.allocs[addr] = {"relay": relay, "perms": set(), "channels": {}, "peers_by_ch": {}}
            self._reply(msg, stun.SUCCESS, {stun.XOR_RELAYED_ADDRESS: a["relay"].get_extra_info("sockname")[:2],
                                            stun.XOR_MAPPED_ADDRESS: addr[:2], stun.LIFETIME: 600}, addr, key)
        elif a is None:
            self._reply(msg, stun.ERROR, {stun.ERROR_CODE: (437, "Allocation Mismatch")}, addr, key)
        elif msg.method == stun.CREATE_PERMISSION:
            a["perms"].add(msg.attrs[stun.XOR_PEER_ADDRESS][0])
            self._reply(msg, stun.SUCCESS, {}, addr, key)
        elif msg.method == stun.CHANNEL_BIND:
            ch, peer = msg.attrs[stun.CHANNEL_NUMBER], msg.attrs[stun.XOR_PEER_ADDRESS]
            a["channels"][peer] = ch
            a["peers_by_ch"][ch] = peer
            a["perms"].add(peer[0])
            self._reply(msg, stun.SUCCESS, {}, addr, key)
        elif msg.method == stun.REFRESH:
            if msg.attrs.get(stun.LIFETIME) == 0:
                a["relay"].close()
                del self.allocs[addr]
            self._reply(msg, stun.SUCCESS, {stun.LIFETIME: msg.attrs.get(stun.LIFETIME, 600)}, addr, key)

    def _from_peer(self, client, data, peer):
        a = self.allocs.get(client)
        if a is None or peer[0] not in a["perms"]:
            return   # no permission: dropped
        self.relayed_packets += 1
        ch = a["channels"].get(peer[:2])
        if ch is not None:
            self.transport.sendto(struct.pack("!HH", ch, len(data)) + data, client)
        else:
            m = stun.Message(stun.DATA, stun.INDICATION)
            m.attrs[stun.XOR_PEER_ADDRESS] = peer[:2]
            m.attrs[stun.DATA_ATTR] = data
            self.transport.sendto(m.encode(None, fingerprint=False), client)
