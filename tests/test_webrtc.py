"""WebRTC transport: STUN (RFC 5769 vectors), SRTP (RFC 3711 B.2/B.3 vectors + roundtrip),
DTLS-SRTP handshake, RFC 6184 packetizer <-> depacketizer, RTCP builders, SDP answer, and a
full WHEP loopback (ICE-lite -> DTLS -> SRTP -> H.264 depacketize -> independent decoder ->
barcode) with NACK retransmission and PLI -> IDR."""
import asyncio
import os
import random
import struct

import pytest

from mxdesk.codec.h264_decoder import Decoder
from mxdesk.models.synthetic import read_barcode
from mxdesk.server import rtp as R
from mxdesk.server import stun as S
from mxdesk.server.webrtc import build_answer, parse_sdp, pick_h264
from mxdesk.server.whep_client import make_offer, whep_view

from .test_server import free_port, make_server

# RFC 5769 §2.1 sample request (password "VOkJxbRl1RmTxUk/WvJxBt")
RFC5769_REQ = bytes.fromhex(
    "000100582112a442b7e7a701bc34d686fa87dfae802200105354554e2074657374"
    "20636c69656e7400240004" "6e0001ff80290008932ff9b151263b36000600096576746a3a6836765920202000080014"
    "9aeaa70cbfd8cb56781ef2b5b2d3f249c1b571a280280004e57a3bcf")


def test_stun_rfc5769_request_vector():
    m = S.StunMessage.decode(RFC5769_REQ)
    assert m.type == S.BINDING_REQUEST
    assert m.get(S.A_USERNAME) == b"evtj:h6vY"
    assert m.check_integrity(b"VOkJxbRl1RmTxUk/WvJxBt")
    assert not m.check_integrity(b"wrong")
    bad = bytearray(RFC5769_REQ)
    bad[30] ^= 1
    assert not S.StunMessage.decode(bytes(bad)).check_integrity(b"VOkJxbRl1RmTxUk/WvJxBt")


def test_stun_roundtrip_and_xor_address():
    tid = os.urandom(12)
    for host, port in [("192.0.2.1", 32853), ("2001:db8:1234:5678:11:2233:4455:6677", 32853)]:
        v = S.xor_address(host, port, tid)
        assert S.parse_xor_address(v, tid) == (host, port)
    m = S.StunMessage(S.BINDING_SUCCESS, tid, [(S.A_XOR_MAPPED_ADDRESS, S.xor_address("10.1.2.3", 5000, tid))])
    raw = m.encode(b"key")
    d = S.StunMessage.decode(raw)
    assert S.is_stun(raw) and d.tid == tid and d.check_integrity(b"key")
    assert S.parse_xor_address(d.get(S.A_XOR_MAPPED_ADDRESS), tid) == ("10.1.2.3", 5000)
    # RFC 5769 §2.2 response XOR-MAPPED-ADDRESS (192.0.2.1:32853)
    tid2 = bytes.fromhex("b7e7a701bc34d686fa87dfae")
    assert S.parse_xor_address(bytes.fromhex("0001a147e112a643"), tid2) == ("192.0.2.1", 32853)


def test_srtp_rfc3711_vectors(native):
    net = native.net
    ks = net.SrtpSession.aes_cm_keystream(bytes.fromhex("2B7E151628AED2A6ABF7158809CF4F3C"),
                                          bytes.fromhex("F0F1F2F3F4F5F6F7F8F9FAFBFCFD0000"), 48)
    assert ks.hex() == ("e03ead0935c95e80e166b16dd92b4eb4d23513162b02d0f72a43a2fe4a5f97ab"
                        "41e95b3bb0a2e8dd477901e4fca894c0")
    s = net.SrtpSession(bytes.fromhex("E1F97A0D3E018BE0D64FA32C06DE4139"), bytes.fromhex("0EC675AD498AFEEBB6960B3AABE6"))
    assert s.rtp_key.hex() == "c61e7a93744f39ee10734afe3ff7a087"
    assert s.rtp_salt.hex() == "30cbbc08863d8c85d49db34a9ae1"
    assert s.rtp_auth.hex()[:40] == "cebe321f6ff7716b6fd4ab49af256a156d38baa4"


def test_srtp_roundtrip_tamper_and_wrap(native):
    net = native.net
    k, salt = os.urandom(16), os.urandom(14)
    tx, rx = net.SrtpSession(k, salt), net.SrtpSession(k, salt)
    seqs = list(range(65530, 65536)) + list(range(0, 6))
    sent = []
    for i, seq in enumerate(seqs):
        pkt = struct.pack("!BBHII", 0x80, 96, seq, 1000 * i, 0x1234) + os.urandom(50)
        p = tx.protect_rtp(pkt)
        sent.append((pkt, p))
        assert len(p) == len(pkt) + 10 and p[12:62] != pkt[12:]
        assert rx.unprotect_rtp(p) == pkt
    # retransmission of a pre-wrap packet after the wrap keeps its ROC
    pkt0, p0 = sent[2]
    assert tx.protect_rtp(pkt0) == p0
    assert rx.unprotect_rtp(p0) == pkt0
    bad = bytearray(sent[-1][1])
    bad[20] ^= 0x40
    assert rx.unprotect_rtp(bytes(bad)) == b""
    rtcp = R.build_pli(1, 2)
    c = tx.protect_rtcp(rtcp)
    assert rx.unprotect_rtcp(c) == rtcp and len(c) == len(rtcp) + 14


def test_dtls_srtp_handshake(native):
    net = native.net
    srv, cli = net.DtlsEndpoint(True), net.DtlsEndpoint(False)
    assert srv.fingerprint.startswith("sha-256 ") and len(srv.fingerprint) == 8 + 32 * 3 - 1  # one identity per process
    to_srv = cli.start()
    for _ in range(20):
        to_cli = [d for x in to_srv for d in srv.feed(x)]
        to_srv = [d for x in to_cli for d in cli.feed(x)]
        if srv.handshake_done and cli.handshake_done:
            break
    assert srv.handshake_done and cli.handshake_done, (srv.error, cli.error)
    assert srv.peer_fingerprint == cli.fingerprint and cli.peer_fingerprint == srv.fingerprint
    assert srv.srtp_profile == cli.srtp_profile == "SRTP_AES128_CM_SHA1_80"
    km = srv.export_srtp_keys()
    assert len(km) == 60 and km == cli.export_srtp_keys()


def _annexb(nals):
    return b"".join(b"\x00\x00\x00\x01" + n for n in nals)


def test_packetizer_depacketizer_roundtrip(native):
    net = native.net
    sps, pps = b"\x67\x42\xc0\x2a" + os.urandom(8), b"\x68\xce\x3c\x80"
    big = b"\x65" + os.urandom(5000)
    small = b"\x41" + os.urandom(100)
    au = _annexb([sps, pps, big, small])
    assert [bytes(x) for x in net.split_annexb(au)] == [sps, pps, big, small]
    pk = net.RtpH264Packetizer(0xABCD, 102, 1150, 65534)
    pkts = pk.packetize(au, 12345)
    assert all(len(p) <= 12 + 1150 for p in pkts)
    hs = [R.rtp_header(p) for p in pkts]
    assert [h["marker"] for h in hs] == [False] * (len(pkts) - 1) + [True]
    assert hs[0]["payload"][0] & 0x1F == 24  # STAP-A with SPS+PPS
    assert any(h["payload"][0] & 0x1F == 28 for h in hs)  # FU-A
    assert [h["seq"] for h in hs][:3] == [65534, 65535, 0] and all(h["ts"] == 12345 for h in hs)
    d = R.H264Depacketizer()
    outs = [d.push(p) for p in pkts]
    assert outs[-1] == au and all(o is None for o in outs[:-1]) and d.lost == 0
    assert pk.packets == len(pkts)


def test_rtcp_builders_parse():
    nack = R.build_nack(1, 2, [100, 101, 105, 116, 117, 200])
    (p,) = R.parse_rtcp(nack)
    assert p["pt"] == 205 and p["fmt"] == 1 and sorted(p["nack"]) == [100, 101, 105, 116, 117, 200]
    parsed = R.parse_rtcp(R.build_sr(7, 9000, 10, 1000) + R.build_pli(1, 7))
    assert [(x["pt"], x["fmt"]) for x in parsed] == [(200, 0), (202, 1), (206, 1)]
    assert parsed[0]["ssrc"] == 7


def test_sdp_answer():
    offer = make_offer("abcd", "p" * 24, "sha-256 AA:BB", h264_pt=102)
    assert pick_h264(parse_sdp(offer).media[0]) == "102"
    a = build_answer(offer, "uf", "pw" * 12, "sha-256 CC:DD", "127.0.0.1", 5000, 42)
    assert a.pt == 102 and a.mid == "0" and a.remote_ufrag == "abcd" and a.remote_fingerprint == "sha-256 AA:BB"
    sdp = parse_sdp(a.sdp)
    assert "a=ice-lite" in sdp.session and "a=group:BUNDLE 0" in sdp.session
    v, au = sdp.media
    assert v.kind == "video" and v.port == 5000 and v.fmts == ["102"] and v.attr("setup") == "passive"
    assert "packetization-mode=1" in v.attr("fmtp") and v.attr("sendonly") == ""
    assert au.kind == "audio" and au.port == 0
    with pytest.raises(ValueError):
        build_answer(offer.replace("H264", "H265"), "uf", "pw", "fp", "127.0.0.1", 5000, 42)


def test_whep_loopback_decodes_with_nack_and_pli(native, monkeypatch):
    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    # the PLI comes a few frames after the first IDR: a short coalescing interval (the coalescer's
    # own timing is tests/test_server.py's) so its IDR lands inside the short stream
    monkeypatch.setenv("MXDESK_IDR_MIN_INTERVAL", "0.02")
    monkeypatch.setenv("MXDESK_IDR_COVER", "0.01")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    from mxdesk.server.app import serve

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            res = await whep_view(f"http://127.0.0.1:{port}/whep", 12, drop_seq_every=7, pli_after=5)
            peers = dict(srv.whep.peers)
            return res, peers
        finally:
            await runner.cleanup()

    res, peers = asyncio.run(go())
    assert len(res.aus) == 12 and res.lost > 0 and res.rtx == res.lost
    frames = Decoder().decode(res.stream)
    assert len(frames) == 12
    ids = [read_barcode(y)[0] for y, _, _ in frames]
    assert all(b == a + 1 for a, b in zip(ids, ids[1:]))
    # 90 kHz timestamps follow the capture clock (30 fps -> ~3000 ticks)
    dts = [(b - a) & 0xFFFFFFFF for a, b in zip(res.rtp_ts, res.rtp_ts[1:])]
    assert all(1000 < d < 9000 for d in dts)
    # the PLI after frame 5 produced a second IDR (NAL type 5) within the next frames
    idr = [i for i, au in enumerate(res.aus) if any((n[0] & 0x1F) == 5 for n in native.net.split_annexb(au))]
    assert idr[0] == 0 and any(i >= 5 for i in idr[1:])
    assert not peers  # DELETE /whep/<id> removed the session


def test_rtcp_rr_and_remb_roundtrip():
    rr = R.build_rr(11, 22, 0.25, cum_lost=7, ext_seq=1000)
    (p,) = R.parse_rtcp(rr)
    assert p["pt"] == 201 and p["reports"][0]["ssrc"] == 22 and abs(p["reports"][0]["fraction_lost"] - 0.25) < 1e-9
    assert p["reports"][0]["cum_lost"] == 7
    (q,) = R.parse_rtcp(R.build_remb(11, 22, 3_500_000))
    assert q["pt"] == 206 and q["fmt"] == 15 and abs(q["remb_bps"] - 3_500_000) < 3_500_000 / 2 ** 17


def test_congestion_controller():
    from mxdesk.server.webrtc import CongestionController

    class P:
        bitrate_kbps = 8000
        calls = []

        def set_bitrate(self, k):
            self.calls.append(k)

    p = P()
    cc = CongestionController(p, enabled=True)
    cc.on_loss(0.30)  # heavy loss: multiplicative decrease
    assert p.calls[-1] == int(8000 * 0.85)
    cc.on_remb(2_000_000)  # receiver estimate caps the target
    assert p.calls[-1] == 1900
    for _ in range(30):
        cc.on_loss(0.0)  # probing never exceeds the REMB cap / configured max
    assert p.calls[-1] == 1900
    cc.on_remb(50_000_000)
    for _ in range(40):
        cc.on_loss(0.0)
    assert p.calls[-1] == 8000
    off = CongestionController(P(), enabled=False)
    off.on_loss(0.5)
    assert off.pipeline.calls == p.calls  # disabled: no set_bitrate calls added


def test_answer_lists_every_host_candidate():
    offer = make_offer("abcd", "p" * 24, "sha-256 AA:BB")
    a = build_answer(offer, "uf", "pw" * 12, "sha-256 CC:DD", "10.0.0.5", 5000, 42, extra_hosts=["10.0.0.5", "192.168.1.9"])
    v = parse_sdp(a.sdp).media[0]
    cands = v.attrs_named("candidate")
    assert [c.split()[4] for c in cands] == ["10.0.0.5", "192.168.1.9"] and all(c.split()[5] == "5000" for c in cands)


def test_h265_packetizer_depacketizer_roundtrip(native):
    net = native.net
    rng = random.Random(1234)

    def body(n):  # seeded; a NAL never ends in 0x00 (ambiguous in Annex-B: it would read as a start code)
        b = bytearray(rng.getrandbits(8) for _ in range(n))
        b[-1] |= 1
        return bytes(b)

    vps, sps, pps = b"\x40\x01" + body(20), b"\x42\x01" + body(30), b"\x44\x01" + body(6)
    idr = b"\x26\x01" + body(4000)  # IDR_W_RADL slice
    small = b"\x02\x01" + body(50)  # TRAIL_R slice
    au = _annexb([vps, sps, pps, idr, small])
    pk = net.RtpH265Packetizer(0x1234, 104, 1150, 7)
    pkts = pk.packetize(au, 999)
    hs = [R.rtp_header(p) for p in pkts]
    assert all(len(p) <= 12 + 1150 for p in pkts)
    assert [h["marker"] for h in hs] == [False] * (len(pkts) - 1) + [True]
    types = [(h["payload"][0] >> 1) & 0x3F for h in hs]
    assert types[0] == 48  # aggregation packet with VPS/SPS/PPS
    assert 49 in types  # fragmentation units of the IDR slice
    d = R.H265Depacketizer()
    outs = [d.push(p) for p in pkts]
    assert outs[-1] == au and all(o is None for o in outs[:-1]) and d.lost == 0


def test_sdp_answer_h265():
    from mxdesk.server.whep_client import make_offer

    offer = make_offer("uf", "pw", "sha-256 AA:BB")
    ans = build_answer(offer, "u", "p", "sha-256 CC", "10.0.0.1", 5000, 42, level_idc=153, codec="hevc")
    assert ans.pt == 104
    assert "a=rtpmap:104 H265/90000" in ans.sdp and "level-id=153" in ans.sdp
    ans264 = build_answer(offer, "u", "p", "sha-256 CC", "10.0.0.1", 5000, 42)
    assert ans264.pt == 102


def test_rtp_vp8_packetizer_roundtrip(native):
    """RFC 7741: descriptor with X / I / M (15-bit PictureID), S + PID 0 on a frame's first packet
    only, marker on its last; the depacketizer reassembles the frame and drops one with a hole."""
    net = native.net
    rng = random.Random(7)
    frame = bytes(rng.getrandbits(8) for _ in range(5000))
    pk = net.RtpVp8Packetizer(0x55, 96, 1150, 65530, 0x7FFE)
    pkts = pk.packetize(frame, 1234)
    hs = [R.rtp_header(p) for p in pkts]
    assert len(pkts) == 5 and all(len(p) <= 12 + 1150 for p in pkts)
    assert [h["seq"] for h in hs] == [65530, 65531, 65532, 65533, 65534]
    assert [h["marker"] for h in hs] == [False] * 4 + [True]
    descs = [R.Vp8Depacketizer.descriptor(h["payload"]) for h in hs]
    assert [d["S"] for _, d in descs] == [True] + [False] * 4
    assert all(off == 4 and d["picture_id"] == 0x7FFE and d["PID"] == 0 and not d["N"] for off, d in descs)
    d = R.Vp8Depacketizer()
    outs = [d.push(p) for p in pkts]
    assert outs[-1] == frame and all(o is None for o in outs[:-1])
    nxt = pk.packetize(frame[:100], 4321)  # picture id wraps at 15 bits
    assert len(nxt) == 1 and R.Vp8Depacketizer.descriptor(R.rtp_header(nxt[0])["payload"])[1]["picture_id"] == 0x7FFF
    assert pk.next_picture_id == 0
    lossy = R.Vp8Depacketizer()
    third = pk.packetize(frame, 5555)
    assert [lossy.push(p) for i, p in enumerate(third) if i != 2] == [None] * 4 and lossy.lost == 1


def test_sdp_answer_vp8():
    offer = make_offer("uf", "pw", "sha-256 AA:BB")
    ans = build_answer(offer, "u", "p", "sha-256 CC", "10.0.0.1", 5000, 42, codec="vp8")
    assert ans.pt == 96 and "a=rtpmap:96 VP8/90000" in ans.sdp and "a=fmtp:96" not in ans.sdp
    with pytest.raises(ValueError, match="VP8"):
        build_answer(offer.replace("a=rtpmap:96 VP8/90000", ""), "u", "p", "sha-256 CC", "10.0.0.1", 5000, 42,
                     codec="vp8")


def test_whep_loopback_vp8(native, monkeypatch):
    """WEBRTC_ENCODER=cpuvp8enc: the answer negotiates VP8/90000, RFC 7741 packets reassemble,
    NACK retransmissions fill the gaps and the frames decode (in-tree RFC 6386 decoder) with
    contiguous barcodes."""
    from mxdesk.codec.vp8_decoder import Decoder as Vp8Decoder

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "WEBRTC_ENCODER": "cpuvp8enc"}, codec="vp8")
    from mxdesk.server.app import serve

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await whep_view(f"http://127.0.0.1:{port}/whep", 6, drop_seq_every=9)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    assert " VP8/90000" in res.answer
    assert len(res.aus) == 6 and res.rtx == res.lost and not res.aus[0][0] & 1  # starts on a key frame
    frames = Vp8Decoder().decode(res.aus)
    ids = [read_barcode(y)[0] for y, _, _ in frames]
    assert len(ids) == 6 and all(b == a + 1 for a, b in zip(ids, ids[1:]))


def test_whep_loopback_hevc(native, monkeypatch):
    """WEBRTC_ENCODER=x265enc: the answer negotiates H265/90000, RFC 7798 packets reassemble,
    NACK retransmissions fill the gaps and the stream decodes (HEVC reference decoder)."""
    from mxdesk.codec.hevc_decoder import Decoder as HevcDecoder

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "WEBRTC_ENCODER": "x265enc"}, codec="hevc")
    from mxdesk.server.app import serve

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await whep_view(f"http://127.0.0.1:{port}/whep", 6, drop_seq_every=9)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    assert " H265/90000" in res.answer
    assert len(res.aus) == 6 and res.rtx == res.lost
    frames = HevcDecoder().decode(res.stream)
    assert len(frames) == 6
    ids = [read_barcode(y)[0] for y, _, _ in frames]
    assert all(b == a + 1 for a, b in zip(ids, ids[1:]))


def test_whep_client_repairs_real_loss_with_nack(native, monkeypatch):
    """10 % of video packets silently lost: the viewer NACKs every hole (as browsers do) and
    the server retransmits from its history; the decoded sequence stays contiguous."""
    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    from mxdesk.server.app import serve

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await whep_view(f"http://127.0.0.1:{port}/whep", 15, simulate_loss=0.1)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    assert res.nacked > 0 and res.recovered == res.nacked and res.gave_up == 0
    frames = Decoder().decode(res.stream)
    ids = [read_barcode(y)[0] for y, _, _ in frames]
    assert len(ids) == 15 and all(b == a + 1 for a, b in zip(ids, ids[1:]))


def test_rtcp_sr_maps_rtp_to_wall_clock(native, monkeypatch):
    """The sender report carries the RTP clock of the moment it is sent, so the viewer maps every
    frame's RTP timestamp to the capture wall-clock time: the end-to-end latencies derived from
    it are small and positive on one host (tools/bench_density.py relies on this)."""
    from mxdesk.server.whep_client import e2e_latency_ms

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    from mxdesk.server.app import serve

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await whep_view(f"http://127.0.0.1:{port}/whep", 45)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    assert res.srs >= 1 and res.sr_map is not None
    lat = e2e_latency_ms(res)
    assert len(lat) == 45
    assert all(-2.0 < v < 500.0 for v in lat), lat  # same host: capture precedes arrival (ms resolution)


@pytest.mark.parametrize("mode", [True, "native"])
def test_whep_lite_viewer_counts_frames(native, monkeypatch, mode):
    """The density harness's lite viewer (tools/bench_density.py --client lite): frames counted
    from the plaintext RTP headers of the SRTP stream (one timestamp, marker bit, no sequence gap)
    after the same ICE / DTLS set-up; RTCP sender reports still decrypted for the latency map.
    "native": the count by the native recvmmsg loop (--client native), the socket handed over
    after DTLS."""
    from mxdesk.server.whep_client import e2e_latency_ms

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "WEBRTC_ENCODER": "x264enc"})
    from mxdesk.server.app import serve

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await whep_view(f"http://127.0.0.1:{port}/whep", 70, lite=mode)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    assert len(res.aus) == 70 and res.lost == 0 and res.packets >= 70
    assert res.stage == "media" and len(set(res.rtp_ts)) == 70
    assert res.srs >= 1 and len(e2e_latency_ms(res)) > 0  # an SR arrived within ~1.2 s of frames


def test_send_au_batches_more_than_one_sendmmsg(native):
    """An access unit of ~150 packets goes out through several sendmmsg batches (64 each,
    csrc/net/rtp_sender.cpp): every datagram arrives once, in order, and decrypts to the packetizer's
    packet; the return value counts them."""
    import socket
    net = native.net
    rx_sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx_sock.bind(("127.0.0.1", 0))
    rx_sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    rx_sock.settimeout(2.0)
    tx_sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        k, salt = os.urandom(16), os.urandom(14)
        tx, rx = net.SrtpSession(k, salt), net.SrtpSession(k, salt)
        peer = net.UdpPeer(tx_sock.fileno(), "127.0.0.1", rx_sock.getsockname()[1])
        pk = net.RtpH264Packetizer(0x1234, 96, 1150, 100)
        au = b"\x00\x00\x00\x01\x65" + os.urandom(170_000)  # one IDR NAL: FU-A fragments
        hist = net.RtpHistory(1024)
        n = net.send_au(pk, tx, hist, peer, au, 9000)
        assert n == pk.packets > 128
        got = [rx.unprotect_rtp(rx_sock.recv(2048)) for _ in range(n)]
        seqs = [struct.unpack("!H", g[2:4])[0] for g in got]
        assert seqs == list(range(100, 100 + n))
        assert all(hist.get(s) == g for s, g in zip(seqs, got))
    finally:
        rx_sock.close()
        tx_sock.close()
