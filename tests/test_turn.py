"""Relayed ICE connectivity through a TURN allocation (webrtc/turn_client.py and the
relay pairs of webrtc/ice.py) against the in-process TURN stub (tests/turn_stub.py).
Reference role: aioice TURN under src/selkies/webrtc/rtcicetransport.py:53-139."""
import asyncio

import pytest

from selkies_gstreamer_amd.webrtc import stun
from selkies_gstreamer_amd.webrtc.ice import IceAgent
from selkies_gstreamer_amd.webrtc.turn_client import TurnAllocation, TurnError, parse_turn_url
from tests.turn_stub import TurnStub


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


def test_parse_turn_url():
    assert parse_turn_url("turn://u:p@turn.example.com:3478") == ("turn.example.com", 3478, "u", "p")
    assert parse_turn_url("turn://u:p@10.0.0.1:443?transport=udp") == ("10.0.0.1", 443, "u", "p")
    assert parse_turn_url("turn://u:p@10.0.0.1:443?transport=tcp") is None
    assert parse_turn_url("stun:stun.l.google.com:19302") is None


def test_allocation_auth_and_bad_password():
    async def main():
        srv = TurnStub({"alice": "secret"})
        addr = await srv.start()
        loop = asyncio.get_running_loop()

        class P(asyncio.DatagramProtocol):
            def datagram_received(self, data, a):
                for x in allocs:
                    x.on_datagram(data)
        tr, _ = await loop.create_datagram_endpoint(P, local_addr=("127.0.0.1", 0))
        alloc = TurnAllocation(addr, "alice", "secret", tr.sendto)
        allocs = [alloc]
        relayed = await alloc.allocate()
        assert relayed[0] == "127.0.0.1" and relayed[1] > 0 and alloc.realm == "selkies.test"
        await alloc.create_permission("127.0.0.1")
        ch = await alloc.channel_bind(("127.0.0.1", 9))
        assert ch == 0x4000 and ("127.0.0.1", 9) in srv.allocs[tr.get_extra_info("sockname")[:2]]["channels"]
        await alloc.close()
        assert not srv.allocs   # LIFETIME 0 released the allocation
        bad = TurnAllocation(addr, "alice", "wrong", tr.sendto)
        allocs.append(bad)
        with pytest.raises(TurnError):
            await bad.allocate()
        tr.close()
        srv.close()
    run(main())


@pytest.mark.parametrize("relay_side", ["controlling", "controlled"])
def test_relay_only_connectivity_and_data(relay_side):
    """One agent uses policy 'relay' (only its TURN relay candidate is offered and only
    relayed pairs are checked); the other is an ordinary host-candidate agent. ICE must
    connect through the relay, and data must flow both ways through it."""
    async def main():
        srv = TurnStub({"bob": "pw"})
        taddr = await srv.start()
        relay_ctrl = relay_side == "controlling"
        a = IceAgent(controlling=relay_ctrl, addresses=["127.0.0.1"], turn_server=(taddr[0], taddr[1], "bob", "pw"),
                     relay_only=True)
        b = IceAgent(controlling=not relay_ctrl, addresses=["127.0.0.1"])
        ca, cb = await a.gather(), await b.gather()
        assert [c.type for c in ca] == ["relay"]
        assert "typ relay raddr" in ca[0].to_sdp()
        a.set_remote_credentials(b.local_ufrag, b.local_pwd)
        b.set_remote_credentials(a.local_ufrag, a.local_pwd)
        for c in cb:
            a.add_remote_candidate(c)
        for c in ca:
            b.add_remote_candidate(c)
        got_a, got_b = asyncio.Queue(), asyncio.Queue()
        a.on_packet = lambda d, addr: got_a.put_nowait(d)
        b.on_packet = lambda d, addr: got_b.put_nowait(d)
        await asyncio.gather(a.connect(10), b.connect(10))
        assert a.selected_relayed and b.selected == (ca[0].host, ca[0].port)
        # DTLS-like payloads (first byte 22) both ways, before and after the channel bind
        for i in range(3):
            a.send(bytes([22, i]) + b"x" * 100)
            b.send(bytes([23, i]) + b"y" * 50)
            assert (await asyncio.wait_for(got_b.get(), 5))[:2] == bytes([22, i])
            assert (await asyncio.wait_for(got_a.get(), 5))[:2] == bytes([23, i])
            await asyncio.sleep(0.05)
        assert a.turn.channels   # the selected peer got a channel (ChannelData framing)
        assert srv.relayed_packets >= 6
        await a.close()
        await b.close()
        srv.close()
    run(main())


def test_relay_candidate_alongside_host():
    """Default policy: host + relay candidates are offered, both pair kinds exist, and the
    direct pair (higher priority, reachable here) is the one selected."""
    async def main():
        srv = TurnStub({"bob": "pw"})
        taddr = await srv.start()
        a = IceAgent(controlling=True, addresses=["127.0.0.1"], turn_server=(taddr[0], taddr[1], "bob", "pw"))
        b = IceAgent(controlling=False, addresses=["127.0.0.1"])
        ca, cb = await a.gather(), await b.gather()
        assert sorted(c.type for c in ca) == ["host", "relay"]
        a.set_remote_credentials(b.local_ufrag, b.local_pwd)
        b.set_remote_credentials(a.local_ufrag, a.local_pwd)
        for c in cb:
            a.add_remote_candidate(c)
        for c in ca:
            b.add_remote_candidate(c)
        assert {p.relayed for p in a.pairs.values()} == {False, True}
        await asyncio.gather(a.connect(10), b.connect(10))
        assert a.selected is not None
        await a.close()
        await b.close()
        srv.close()
    run(main())


def test_channel_binding_refreshed_independently_of_permissions():
    """Permission refreshes (every ~240 s) must not reset a channel binding's age:
    the binding itself is re-sent before its 600 s lifetime runs out (RFC 5766 §11).
    Lifetimes are shortened 1000x here."""
    async def main():
        srv = TurnStub({"alice": "secret"})
        addr = await srv.start()
        loop = asyncio.get_running_loop()

        class P(asyncio.DatagramProtocol):
            def datagram_received(self, data, a):
                alloc.on_datagram(data)
        tr, _ = await loop.create_datagram_endpoint(P, local_addr=("127.0.0.1", 0))
        alloc = TurnAllocation(addr, "alice", "secret", tr.sendto)
        alloc.permission_refresh_s, alloc.channel_refresh_s = 0.24, 0.54
        await alloc.allocate()
        await alloc.create_permission("127.0.0.1")
        await alloc.channel_bind(("127.0.0.1", 9))
        await asyncio.sleep(1.5)
        binds = srv.requests.count(stun.CHANNEL_BIND)
        perms = srv.requests.count(stun.CREATE_PERMISSION)
        await alloc.close()
        tr.close()
        srv.close()
        assert binds >= 3, srv.requests         # initial bind + at least two refreshes in 1.5 s
        assert perms >= 1
    run(main())
