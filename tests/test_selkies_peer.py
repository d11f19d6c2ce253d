"""The selkies streaming peer on /ws: a headless client speaking the selkies
signalling protocol (HELLO 1 -> server's SDP offer -> answer -> ICE / DTLS-SRTP) receives
barcoded H.264 frames that the independent decoder decodes in order, and its messages on the
server-opened ``input`` data channel reach the input handler.  Reference: selkies-gstreamer
web app (reference Dockerfile:472) against the streaming app (selkies-gstreamer-entrypoint.sh:44-47)."""
import asyncio

from mxdesk.codec.h264_decoder import Decoder
from mxdesk.models.synthetic import read_barcode
from mxdesk.server.selkies_client import make_answer, selkies_view
from mxdesk.server.webrtc import build_offer, parse_answer

from .test_server import free_port, make_server


def test_offer_answer_roundtrip():
    offer = build_offer("uf", "pw", "sha-256 AA:BB", "127.0.0.1", 5000, 42, audio_ssrc=7)
    assert "a=setup:actpass" in offer and "a=ice-lite" in offer and "webrtc-datachannel" in offer
    ans = make_answer(offer, "cu", "cp", "sha-256 CC:DD")
    a, setup = parse_answer(ans, 96)
    assert setup == "active" and a.pt == 96 and a.remote_ufrag == "cu" and a.remote_fingerprint == "sha-256 CC:DD"
    assert a.audio_pt == 0 and a.dc_mid == "2" and a.remote_sctp_port == 5000


def test_selkies_client_gets_offer_media_and_input_channel(native, monkeypatch):
    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    # the PLI comes a few frames after the first IDR: a short coalescing interval (the coalescer's
    # own timing is tests/test_server.py's) so its IDR lands inside the short stream
    monkeypatch.setenv("MXDESK_IDR_MIN_INTERVAL", "0.02")
    monkeypatch.setenv("MXDESK_IDR_COVER", "0.01")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    from mxdesk.server.app import serve

    got = []
    orig = srv._on_client_message

    def spy(text):
        got.append(text)
        return orig(text)
    srv.whep.on_input = spy  # the selkies peers are built with the WHEP endpoint's input handler

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            res = await selkies_view(f"ws://127.0.0.1:{port}/ws", 8, dc_messages=["m,40,30,0,0", "kd,65", "ku,65"],
                                     pli_after=4)
            for _ in range(50):  # the input messages are delivered asynchronously
                if len(got) >= 3:
                    break
                await asyncio.sleep(0.05)
            return res, dict(srv.selkies.sessions)
        finally:
            await runner.cleanup()

    res, sessions = asyncio.run(go())
    assert len(res.aus) == 8
    frames = Decoder().decode(res.stream)
    ids = [read_barcode(y)[0] for y, _, _ in frames]
    assert len(ids) == 8 and all(b == a + 1 for a, b in zip(ids, ids[1:]))
    assert res.dc_labels == ["input"] and res.dc_sent == 3
    assert got[:3] == ["m,40,30,0,0", "kd,65", "ku,65"]
    # the PLI after frame 4 produced an IDR later in the stream
    idr = [i for i, au in enumerate(res.aus) if any((n[0] & 0x1F) == 5 for n in native.net.split_annexb(au))]
    assert idr[0] == 0 and any(i >= 4 for i in idr[1:])
    assert not sessions  # the client's disconnect closed its peer


def test_browser_to_browser_session_releases_streaming_peers():
    """two browsers that link to each other leave their streaming-peer sessions,
    and disconnecting afterwards leaves no peer behind (no orphaned WebRtcPeer)."""
    import aiohttp
    from aiohttp import web

    from mxdesk.server.selkies_peer import SelkiesServerPeer
    from mxdesk.server.signalling import SignallingRelay

    class FakePeer:
        closed = 0
        id = "fake"

        async def start_offer(self):
            return "v=0"

        def close(self):
            FakePeer.closed += 1

    relay = SignallingRelay()
    srv = SelkiesServerPeer(relay, FakePeer)
    relay.attach_server(srv)

    async def go():
        app = web.Application()
        app.router.add_get("/ws", relay.handler)
        runner = web.AppRunner(app)
        await runner.setup()
        port = free_port()
        site = web.TCPSite(runner, "127.0.0.1", port)
        await site.start()
        try:
            async with aiohttp.ClientSession() as cs:
                a = await cs.ws_connect(f"http://127.0.0.1:{port}/ws")
                b = await cs.ws_connect(f"http://127.0.0.1:{port}/ws")
                await a.send_str("HELLO A")
                await b.send_str("HELLO B")
                for ws in (a, b):
                    assert (await ws.receive_str()) == "HELLO"
                    assert "offer" in (await ws.receive_str())  # the streaming peer's offer
                assert set(srv.sessions) == {"A", "B"}
                await a.send_str("SESSION B")
                assert (await a.receive_str()) == "SESSION_OK"
                assert not srv.sessions and relay.sessions == {"A": "B", "B": "A"}
                await a.send_str('{"sdp": "x"}')  # relayed browser -> browser
                assert (await b.receive_str()) == '{"sdp": "x"}'
                await a.close()
                msg = await b.receive_str()
                assert msg == "ERROR peer A disconnected"
                await b.close()
                for _ in range(50):
                    if not relay.peers:
                        break
                    await asyncio.sleep(0.02)
        finally:
            await runner.cleanup()

    asyncio.run(go())
    assert not srv.sessions and not relay.sessions and not relay.peers
    assert FakePeer.closed == 2
