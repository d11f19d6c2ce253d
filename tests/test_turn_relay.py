"""Server-side TURN relay (RFC 8656 client, mxdesk/server/turn_client.py) against an
in-process TURN server (tests/mini_turn.py): long-term auth, permissions, Send/Data and
ChannelData paths, refresh-on-close; then a full WHEP session whose media, RTCP and data
channel all travel through the relay candidate."""
import asyncio

import pytest

from mxdesk.codec.h264_decoder import Decoder
from mxdesk.models.synthetic import read_barcode
from mxdesk.server import turn_client as T
from mxdesk.server.turn import hmac_credentials
from mxdesk.server.webrtc import parse_sdp, turn_relay_settings
from mxdesk.server.whep_client import whep_view

from .mini_turn import MiniTurnServer
from .test_server import free_port, make_server


def test_offer_candidate_ips_and_channel_framing():
    sdp = ("a=candidate:1 1 udp 2122260223 192.168.1.5 50000 typ host\r\n"
           "a=candidate:2 1 udp 2122260223 abcd.local 50001 typ host\r\n"
           "a=candidate:3 1 tcp 1518280447 10.0.0.1 9 typ host tcptype active\r\n"
           "a=candidate:4 1 udp 1686052607 203.0.113.7 61000 typ srflx raddr 192.168.1.5 rport 50000\r\n")
    assert T.offer_candidate_ips(sdp) == ["192.168.1.5", "203.0.113.7"]
    assert T.channel_data(0x4001, b"abcde") == b"\x40\x01\x00\x05abcde"
    assert T.channel_data(0x4001, b"abcde", pad=True) == b"\x40\x01\x00\x05abcde\0\0\0"


def test_turn_client_allocate_permission_send_data_channel():
    async def go():
        srv = MiniTurnServer({"alice": "pw"})
        port = await srv.start()
        got = []
        c = T.TurnClient("127.0.0.1", port, "alice", "pw", on_data=lambda d, p: got.append((d, p)))
        relay = await c.allocate()
        loop = asyncio.get_running_loop()
        q = asyncio.Queue()

        class P(asyncio.DatagramProtocol):
            def datagram_received(self, d, a):
                q.put_nowait((d, a))
        tr, _ = await loop.create_datagram_endpoint(P, local_addr=("127.0.0.1", 0))
        me = tr.get_extra_info("sockname")
        tr.sendto(b"early", relay)            # no permission yet: dropped by the server
        await asyncio.sleep(0.05)
        await c.create_permission([me[0]])
        tr.sendto(b"hello", relay)             # -> Data indication
        c.send(b"back", me)                    # Send indication
        back = await asyncio.wait_for(q.get(), 2)
        await c.channel_bind(me)
        tr.sendto(b"via channel", relay)       # -> ChannelData
        c.send(b"chan back", me)
        back2 = await asyncio.wait_for(q.get(), 2)
        await asyncio.sleep(0.05)
        await c.aclose()
        srv.close()
        tr.close()
        return relay, back, back2, got, dict(c.stats), srv
    relay, back, back2, got, stats, srv = asyncio.run(go())
    assert back == (b"back", relay) and back2 == (b"chan back", relay)
    assert [d for d, _ in got] == [b"hello", b"via channel"] and srv.dropped == 1
    assert stats == {"sent": 1, "received": 1, "channel_sent": 1, "channel_received": 1}
    # 401 challenge first, then the authenticated Allocate; Refresh(lifetime 0) on close
    assert srv.log[0] == (T.ALLOCATE, T.REQUEST) and (T.REFRESH, T.REQUEST) in srv.log


def test_turn_client_bad_password():
    async def go():
        srv = MiniTurnServer({"alice": "pw"})
        port = await srv.start()
        c = T.TurnClient("127.0.0.1", port, "alice", "wrong")
        try:
            with pytest.raises(T.TurnError):
                await c.allocate()
        finally:
            c.close()
            srv.close()
    asyncio.run(go())


def test_turn_relay_settings_from_config():
    from mxdesk.utils import config as C

    assert turn_relay_settings(C.load(env={}, argv=[])) is None
    cfg = C.load(env={"TURN_HOST": "turn.example", "TURN_SHARED_SECRET": "s3", "TURN_PROTOCOL": "TCP"}, argv=[])
    t = turn_relay_settings(cfg)
    assert t["host"] == "turn.example" and t["port"] == 3478 and t["protocol"] == "tcp"
    expiry, user = t["username"].split(":")
    assert user == "mxdesk-server" and t["password"] == hmac_credentials("s3", "mxdesk-server",
                                                                           now=int(expiry) - 86400)[1]
    cfg = C.load(env={"TURN_HOST": "t", "TURN_USERNAME": "u", "TURN_PASSWORD": "p", "MXDESK_TURN_RELAY": "false"},
                 argv=[])
    assert turn_relay_settings(cfg) is None


def test_whep_media_and_datachannel_through_server_relay(monkeypatch):
    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")

    async def go():
        turn = MiniTurnServer({"srv": "secret"})
        tport = await turn.start()
        cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "TURN_HOST": "127.0.0.1",
                                      "TURN_PORT": str(tport), "TURN_USERNAME": "srv", "TURN_PASSWORD": "secret"})
        from mxdesk.server.app import serve

        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            res = await whep_view(f"http://127.0.0.1:{port}/whep", 8, drop_seq_every=6, via_relay=True,
                                  dc_messages=["m,7,8,0,0"])
            peer = srv.whep.last_peer
            return res, dict(peer.relay.stats), turn, srv
        finally:
            await runner.cleanup()
            turn.close()

    res, stats, turn, srv = asyncio.run(go())
    relay = [c for c in parse_sdp(res.answer).media[0].attrs_named("candidate") if "typ relay" in c]
    assert len(relay) == 1
    frames = Decoder().decode(res.stream)
    assert len(frames) == 8 and res.rtx == res.lost > 0
    ids = [read_barcode(y)[0] for y, _, _ in frames]
    assert all(b == a + 1 for a, b in zip(ids, ids[1:]))
    assert (srv.injector.x, srv.injector.y) == (7, 8)
    # after nomination the server bound a channel: media flows as ChannelData
    assert stats["channel_sent"] > 0 and turn.relayed_in > 0 and turn.relayed_out > 0
