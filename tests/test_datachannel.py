"""WebRTC data channels: native SCTP (csrc/net/sctp.cpp) over DTLS, DCEP, and the WHEP
loopback with input travelling over the ``input`` channel (SURVEY.md C37 webrtcbin/usrsctp,
C52 selkies input channel).

The SCTP engine is exercised through an in-memory link with a pinned clock, so loss,
retransmission timers and partial reliability are deterministic."""
import asyncio
import random
import struct

import pytest

from mxdesk.server.webrtc import build_answer, parse_sdp
from mxdesk.server.whep_client import make_offer, whep_view

from .test_server import free_port, make_server


class Link:
    """Two endpoints joined by a lossy in-memory link; ``run`` advances the shared clock."""

    def __init__(self, a, b, loss=0.0, seed=1, drop=None):
        self.a, self.b, self.t = a, b, 0
        self.loss, self.rng = loss, random.Random(seed)
        self.drop = drop  # drop(direction, packet) -> bool, for targeted losses
        self.sent = {"ab": 0, "ba": 0}
        a.set_clock(0)
        b.set_clock(0)

    def _keep(self, d, p):
        self.sent[d] += 1
        if self.drop is not None and self.drop(d, p):
            return False
        return self.rng.random() >= self.loss

    def run(self, from_a=(), from_b=(), ms=10000):
        qa, qb = list(from_a), list(from_b)
        end = self.t + ms
        while True:
            if not qa and not qb:
                if self.t >= end:
                    return
                self.t += 20
                self.a.set_clock(self.t)
                self.b.set_clock(self.t)
                qa += self.a.tick()
                qb += self.b.tick()
                continue
            na, nb = [], []
            for p in qa:
                if self._keep("ab", p):
                    nb += self.b.feed(p)
            for p in qb:
                if self._keep("ba", p):
                    na += self.a.feed(p)
            qa, qb = na, nb


def test_crc32c_vector(native):
    # RFC 3720 B.4 / the common "123456789" check value of CRC-32C
    assert native.net.crc32c(b"123456789") == 0xE3069283
    assert native.net.crc32c(b"\x00" * 32) == 0x8A9136AA


def test_association_handshake_and_ordered_delivery(native):
    N = native.net
    a, b = N.SctpAssociation(), N.SctpAssociation()
    link = Link(a, b)
    link.run(a.connect())
    assert a.established and b.established
    msgs = [f"m{i}".encode() * (i + 1) for i in range(40)]
    out = []
    for m in msgs:
        out += a.send(3, 51, m)
    link.run(out)
    got = b.take_messages()
    assert [m[3] for m in got] == msgs
    assert all(m[0] == 3 and m[1] == 51 and not m[2] for m in got)
    assert a.buffered_amount == 0 and a.stats.messages_out == 40 and b.stats.messages_in == 40


def test_fragmentation_and_loss_recovery(native):
    N = native.net
    a, b = N.SctpAssociation(), N.SctpAssociation()
    link = Link(a, b, loss=0.15, seed=7)
    link.run(a.connect())
    assert a.established
    rng = random.Random(3)
    msgs = [rng.randbytes(rng.choice([10, 1000, 5000, 70000])) for _ in range(30)]
    out = []
    for m in msgs:
        out += a.send(1, 53, m)
    link.run(out, ms=60000)
    got = [m[3] for m in b.take_messages()]
    assert got == msgs  # reliable + ordered despite 15 % loss both ways
    st = a.stats
    assert st.retransmits > 0 and a.buffered_amount == 0
    assert b.stats.sacks_out > 0


def test_t3_timeout_retransmits_lost_tail(native):
    """The only DATA packet is lost: no SACK gap reports it, so the T3 timer must fire."""
    N = native.net
    a, b = N.SctpAssociation(), N.SctpAssociation()
    link = Link(a, b)
    link.run(a.connect())
    lost = {"n": 0}

    def drop(d, p):
        if d == "ab" and p[12] == 0 and lost["n"] == 0:  # first DATA chunk
            lost["n"] += 1
            return True
        return False
    link.drop = drop
    link.run(a.send(0, 51, b"only"), ms=5000)
    assert [m[3] for m in b.take_messages()] == [b"only"]
    assert lost["n"] == 1 and a.stats.t3_expiries >= 1


def test_unordered_delivery(native):
    N = native.net
    a, b = N.SctpAssociation(), N.SctpAssociation()
    link = Link(a, b)
    link.run(a.connect())
    dropped = {"n": 0}

    def drop(d, p):  # lose the first transmission of the first DATA packet
        if d == "ab" and p[12] == 0 and dropped["n"] == 0:
            dropped["n"] += 1
            return True
        return False
    link.drop = drop
    out = []
    for i in range(5):
        out += a.send(2, 51, b"u%d" % i, unordered=True)
    link.run(out, ms=5000)
    # u1..u4 are delivered as they arrive; u0 comes last, after its (fast) retransmission
    assert [m[3] for m in b.take_messages()] == [b"u1", b"u2", b"u3", b"u4", b"u0"]
    assert a.stats.fast_retransmits == 1


def test_partial_reliability_abandons_and_forward_tsn(native):
    N = native.net
    a, b = N.SctpAssociation(), N.SctpAssociation()
    link = Link(a, b)
    link.run(a.connect())
    assert a.peer_supports_forward_tsn
    link.drop = lambda d, p: d == "ab" and p[12] == 0 and b"LOSSY" in p
    out = a.send(4, 51, b"LOSSY", max_retransmits=0)
    link.run(out, ms=3000)
    link.drop = None
    link.run(a.send(4, 51, b"after"), ms=3000)
    # the abandoned message never arrives, the next one on the same ordered stream does
    assert [m[3] for m in b.take_messages()] == [b"after"]
    assert a.stats.abandoned == 1 and a.stats.forward_tsn_out >= 1 and b.stats.forward_tsn_in >= 1
    assert a.buffered_amount == 0


def test_bad_checksum_and_tag_are_dropped(native):
    N = native.net
    a, b = N.SctpAssociation(), N.SctpAssociation()
    link = Link(a, b)
    link.run(a.connect())
    pkt = a.send(0, 51, b"x")[0]
    bad = bytearray(pkt)
    bad[-1] ^= 1
    assert b.feed(bytes(bad)) == [] and b.stats.bad_checksum == 1
    assert b.take_messages() == []
    link.run([pkt])
    assert [m[3] for m in b.take_messages()] == [b"x"]


def test_shutdown(native):
    N = native.net
    a, b = N.SctpAssociation(), N.SctpAssociation()
    link = Link(a, b)
    link.run(a.connect())
    link.run(a.send(0, 51, b"bye") + a.shutdown())
    assert [m[3] for m in b.take_messages()] == [b"bye"]
    assert not a.established and not b.established and a.state == 0 and b.state == 0  # Closed


def test_dcep_open_message_close(native):
    N = native.net
    cli, srv = N.DataChannelEndpoint(False), N.DataChannelEndpoint(True)
    link = Link(cli, srv)
    link.run(cli.connect())
    cid, pk = cli.open("input", "selkies")
    sid, pk2 = srv.open("stats", ordered=False, max_retransmits=0)
    assert cid % 2 == 0 and sid % 2 == 1  # DTLS client even, server odd (RFC 8832 §6)
    link.run(pk, pk2)
    ev_s = srv.take_events()
    ev_c = cli.take_events()
    assert (0, cid, "input", "selkies", False, b"") in ev_s
    assert any(e[0] == 0 and e[1] == sid and e[2] == "stats" for e in ev_c)
    assert cli.is_open(cid) and srv.is_open(cid) and srv.is_open(sid)
    link.run(cli.send(cid, "m,10,20,1,0".encode()) + cli.send(cid, b"\x00\x01", True) + cli.send(cid, b""))
    msgs = [(e[4], e[5]) for e in srv.take_events() if e[0] == 1]
    assert msgs == [(False, b"m,10,20,1,0"), (True, b"\x00\x01"), (False, b"")]
    link.run(cli.close(cid))
    assert any(e[0] == 2 and e[1] == cid for e in srv.take_events())
    assert any(e[0] == 2 and e[1] == cid for e in cli.take_events())
    assert cid not in srv.channels() and sid in srv.channels()


def test_dtls_application_data_roundtrip(native):
    N = native.net
    c, s = N.DtlsEndpoint(False), N.DtlsEndpoint(True)
    q = list(c.start())
    for _ in range(20):
        back = [x for d in q for x in s.feed(d)]
        q = [x for d in back for x in c.feed(d)]
        if c.handshake_done and s.handshake_done and not q:
            break
    assert c.handshake_done and s.handshake_done
    assert c.write(b"") == []
    for d in c.write(b"sctp-packet-1") + c.write(b"\x00" * 1100):
        assert s.feed(d) == []
    assert s.take_app_data() == [b"sctp-packet-1", b"\x00" * 1100]
    for d in s.write(b"pong"):
        c.feed(d)
    assert c.take_app_data() == [b"pong"]


def test_sdp_answer_accepts_datachannel():
    offer = make_offer("uf", "pw", "sha-256 AA:BB", with_datachannel=True)
    ans = build_answer(offer, "u2", "p2", "sha-256 CC", "127.0.0.1", 5000, 42)
    sdp = parse_sdp(ans.sdp)
    app = next(m for m in sdp.media if m.kind == "application")
    assert app.port == 5000 and app.proto == "UDP/DTLS/SCTP" and app.fmts == ["webrtc-datachannel"]
    assert app.attr("sctp-port") == "5000" and app.attr("max-message-size") == "262144"
    assert ans.dc_mid == "2" and ans.remote_sctp_port == 5000
    assert "a=group:BUNDLE 0 1 2" in ans.sdp or "a=group:BUNDLE 0 2" in ans.sdp
    off = build_answer(offer, "u2", "p2", "sha-256 CC", "127.0.0.1", 5000, 42, datachannel=False)
    assert off.dc_mid is None
    assert next(m for m in parse_sdp(off.sdp).media if m.kind == "application").port == 0


def test_whep_loopback_input_over_datachannel(native, monkeypatch):
    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    from mxdesk.server.app import serve

    msgs = ["m,100,50,1,0", "kd,65", "ku,65", "kd,66", '{"type": "clipboard", "text": "héllo"}', "m2,5,-3,0,0"]

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            res = await whep_view(f"http://127.0.0.1:{port}/whep", 4, dc_messages=msgs, dc_wait_stats=True)
            peer = srv.whep.last_peer
            return res, dict(peer.stats), dict(peer.dc_channels)
        finally:
            await runner.cleanup()

    res, stats, chans = asyncio.run(go())
    inj = srv.injector
    assert len(res.aus) >= 4 and res.dc_sent == len(msgs)
    assert stats["dc_in"] == len(msgs)
    assert (inj.x, inj.y) == (105, 47) and inj.keys_down == {66} and inj.clipboard == "héllo"
    assert any('"stats"' in m for m in res.dc_received)
    assert list(chans.values()) == ["input"]


def test_whep_audio_over_datachannel(native, monkeypatch):
    """48 kHz stereo PCM chunks on a browser-opened unordered / no-retransmit channel."""
    from mxdesk.audio.pipeline import CHANNELS, RATE, parse_audio_message

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "MXDESK_AUDIO_SOURCE": "synthetic"})
    from mxdesk.server.app import serve

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            res = await whep_view(f"http://127.0.0.1:{port}/whep", 2, dc_messages=[], dc_audio_chunks=20)
            return res, dict(srv.whep.last_peer.stats)
        finally:
            await runner.cleanup()

    res, stats = asyncio.run(go())
    msgs = [parse_audio_message(m) for m in res.dc_audio]
    assert len(msgs) >= 20 and stats["dc_audio"] >= 20
    assert all(m["rate"] == RATE and m["channels"] == CHANNELS and len(m["pcm"]) == RATE // 100 * CHANNELS
               for m in msgs)
    seqs = [m["seq"] for m in msgs]
    assert len(set(seqs)) == len(seqs)  # unordered channel: no duplicates (no retransmissions)
    assert max(abs(int(x)) for m in msgs for x in m["pcm"]) > 1000  # the synthetic tone, not silence
