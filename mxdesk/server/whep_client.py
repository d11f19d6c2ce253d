"""Headless WHEP/WebRTC viewer: plays the browser's role against ``POST /whep`` (full ICE
agent in the controlling role, DTLS client, SRTP receiver, RTCP PLI/NACK sender).  Used by the
loopback tests and as a CLI smoke-check of a running server (``python -m mxdesk.server.whep_client``).
"""
from __future__ import annotations

import asyncio
import os
import secrets
import socket
import struct
import time
from dataclasses import dataclass, field

from . import rtp as R
from . import stun as S
from .webrtc import parse_sdp


def _native():
    from .. import native

    return native()


def make_offer(ufrag: str, pwd: str, fingerprint: str, h264_pt: int = 102, with_audio: bool = True,
               h265_pt: int = 104, with_datachannel: bool = False, candidate_ip: str | None = None) -> str:
    mids = "0 1" + (" 2" if with_datachannel else "")
    lines = ["v=0", "o=- 4611731400430051336 2 IN IP4 127.0.0.1", "s=-", "t=0 0", f"a=group:BUNDLE {mids}",
             "a=msid-semantic: WMS"]
    media = []
    if with_datachannel:  # the section browsers put in the offer after createDataChannel()
        media += ["m=application 9 UDP/DTLS/SCTP webrtc-datachannel", "c=IN IP4 0.0.0.0", f"a=ice-ufrag:{ufrag}",
                  f"a=ice-pwd:{pwd}", f"a=fingerprint:{fingerprint}", "a=setup:actpass", "a=mid:2",
                  "a=sctp-port:5000", "a=max-message-size:262144"]
    if with_audio:
        media += ["m=audio 9 UDP/TLS/RTP/SAVPF 111 0", "c=IN IP4 0.0.0.0", f"a=ice-ufrag:{ufrag}",
                  f"a=ice-pwd:{pwd}", f"a=fingerprint:{fingerprint}", "a=setup:actpass", "a=mid:1", "a=recvonly",
                  "a=rtcp-mux", "a=rtpmap:111 opus/48000/2", "a=rtpmap:0 PCMU/8000"]
    cand = [f"a=candidate:1 1 udp 2122260223 {candidate_ip} 9 typ host"] if candidate_ip else []
    media = ["m=video 9 UDP/TLS/RTP/SAVPF 96 %d 108 %d" % (h264_pt, h265_pt), "c=IN IP4 0.0.0.0", *cand,
             f"a=ice-ufrag:{ufrag}",
             f"a=ice-pwd:{pwd}", "a=ice-options:trickle", f"a=fingerprint:{fingerprint}", "a=setup:actpass", "a=mid:0",
             "a=recvonly", "a=rtcp-mux", "a=rtcp-rsize", "a=rtpmap:96 VP8/90000",
             f"a=rtpmap:{h264_pt} H264/90000", f"a=rtcp-fb:{h264_pt} nack", f"a=rtcp-fb:{h264_pt} nack pli",
             f"a=fmtp:{h264_pt} level-asymmetry-allowed=1;packetization-mode=1;profile-level-id=42e01f",
             "a=rtpmap:108 H264/90000", "a=fmtp:108 packetization-mode=0;profile-level-id=42e01f",
             f"a=rtpmap:{h265_pt} H265/90000", f"a=rtcp-fb:{h265_pt} nack", f"a=rtcp-fb:{h265_pt} nack pli",
             f"a=fmtp:{h265_pt} profile-id=1;tier-flag=0;level-id=186;tx-mode=SRST"] + media
    return "\r\n".join(lines + media) + "\r\n"


@dataclass
class WhepResult:
    aus: list[bytes] = field(default_factory=list)
    rtp_ts: list[int] = field(default_factory=list)
    packets: int = 0
    lost: int = 0
    rtx: int = 0
    srs: int = 0
    answer: str = ""
    connect_ms: float = 0.0
    stream: bytes = b""
    arrival_us: list[int] = field(default_factory=list)  # CLOCK_MONOTONIC us when each AU completed
    arrival_wall: list[float] = field(default_factory=list)  # time.time() when each AU completed
    sr_map: tuple[float, int] | None = None  # last RTCP SR: (NTP seconds, RTP timestamp) of one instant
    audio_payloads: list[bytes] = field(default_factory=list)  # PCMU packets (20 ms each)
    audio_seqs: list[int] = field(default_factory=list)
    nacked: int = 0        # RTP packets NACKed after a real (not test-injected) loss
    recovered: int = 0     # of those, retransmissions that arrived
    gave_up: int = 0       # holes not repaired in time -> PLI, resync at the next IDR
    dropped_aus: int = 0   # access units discarded while waiting for that IDR
    dc_received: list[str] = field(default_factory=list)  # server -> client data-channel messages
    dc_audio: list[bytes] = field(default_factory=list)   # MXA1 chunks from the "audio" channel
    dc_sent: int = 0
    dc_labels: list[str] = field(default_factory=list)  # server-opened channels (selkies "input")
    stage: str = "post"    # diagnostics: post / ice / dtls / media -- where a failed session stopped
    ice_tx: int = 0        # ICE binding requests sent (retransmissions included)
    datagrams: int = 0     # datagrams received


def e2e_latency_ms(res: WhepResult) -> list[float]:
    """Capture -> viewer latency of every received access unit, from the sender's RTCP SR
    (RFC 3550 6.4.1: NTP time and RTP timestamp of one instant) -- valid when sender and viewer
    share a clock (same host).  Empty before the first SR."""
    if res.sr_map is None:
        return []
    ntp, rtp_sr = res.sr_map
    wall_sr = ntp - R.NTP_EPOCH_OFFSET
    out = []
    for ts, arr in zip(res.rtp_ts, res.arrival_wall):
        d = ((ts - rtp_sr + 0x80000000) & 0xFFFFFFFF) - 0x80000000  # signed 32-bit RTP distance
        out.append((arr - (wall_sr + d / 90000.0)) * 1e3)
    return out


class _Client(asyncio.DatagramProtocol):
    def __init__(self):
        self.q: asyncio.Queue = asyncio.Queue()

    def connection_made(self, transport):
        self.transport = transport

    def datagram_received(self, data, addr):
        self.q.put_nowait(data)


async def whep_view(url: str, n_frames: int, auth=None, drop_seq_every: int = 0, pli_after: int = 0,
                    timeout: float = 30.0, dc_messages: list[str] | None = None,
                    dc_wait_stats: bool = False, via_relay: bool = False, dc_audio_chunks: int = 0,
                    simulate_loss: float = 0.0, lite: bool | str = False) -> WhepResult:
    """Connect to ``url`` (http://host:port/whep), receive ``n_frames`` access units.

    ``drop_seq_every``: discard every Nth RTP packet and recover it with a generic NACK.
    ``pli_after``: send a PLI after that many frames (the server must answer with an IDR).
    ``dc_messages``: offer a data channel, open ``input`` on it (SCTP client side, even
    stream id) and send these text messages; the call returns once all are acknowledged
    (and, with ``dc_wait_stats``, a server stats message has arrived).
    ``dc_audio_chunks``: also open an unordered, no-retransmit ``audio`` channel and wait for
    that many PCM chunks on it.
    ``simulate_loss``: silently drop that fraction of received video packets (seeded), so only
    the client's automatic NACK / PLI repair brings them back.
    ``via_relay``: connect to the server's TURN relay candidate instead of its host candidate
    (the offer then carries a host candidate so the server can create the TURN permission).
    ``lite``: count frames from the plaintext RTP headers (a frame = the packets of one timestamp,
    complete when its marker packet arrives with no sequence gap) instead of decrypting and
    depacketising every packet -- ICE, DTLS, the server's SRTP and RTCP sender reports are the
    same; for density runs where a hundred Python viewers share the server's host (``aus`` then
    holds empty placeholders).  ``lite="native"``: the same count by the native receive loop
    (``_native.net.count_rtp_frames``: recvmmsg batches with the GIL released) once DTLS is up.
    """
    import aiohttp

    N = _native()
    dtls = N.net.DtlsEndpoint(False)
    ufrag, pwd = secrets.token_hex(4), secrets.token_hex(12)
    offer = make_offer(ufrag, pwd, dtls.fingerprint, with_datachannel=dc_messages is not None,
                       candidate_ip="127.0.0.1" if via_relay else None)
    res = WhepResult()
    t0 = time.monotonic()
    async with aiohttp.ClientSession(headers={"Authorization": auth.encode()} if auth else None) as s:
        async with s.post(url, data=offer, headers={"Content-Type": "application/sdp"}) as r:
            if r.status != 201:
                raise RuntimeError(f"WHEP POST failed: {r.status} {await r.text()}")
            res.answer = await r.text()
            location = r.headers["Location"]
    try:
        await media_session(res, res.answer, dtls, ufrag, N, n_frames, t0, timeout=timeout,
                            drop_seq_every=drop_seq_every, pli_after=pli_after, dc_messages=dc_messages,
                            dc_wait_stats=dc_wait_stats, via_relay=via_relay, dc_audio_chunks=dc_audio_chunks,
                            simulate_loss=simulate_loss, lite=lite)
    except Exception as e:
        e.whep_result = res  # (the diagnostics of a failed session: stage, counters)
        raise
    finally:
        try:
            async with aiohttp.ClientSession(headers={"Authorization": auth.encode()} if auth else None) as s:
                base = url.rsplit("/whep", 1)[0]
                async with s.delete(base + location):
                    pass
        except Exception:
            pass
    return res


async def media_session(res: WhepResult, remote_sdp: str, dtls, ufrag: str, N, n_frames: int, t0: float,
                        timeout: float = 30.0, drop_seq_every: int = 0, pli_after: int = 0,
                        dc_messages: list[str] | None = None, dc_wait_stats: bool = False, via_relay: bool = False,
                        dc_audio_chunks: int = 0, simulate_loss: float = 0.0,
                        server_channel: str | None = None, lite: bool | str = False) -> None:
    """The browser side of an established negotiation (remote SDP = the server's answer for
    WHEP, its offer for the selkies protocol): ICE check, DTLS client, SRTP receive with NACK /
    PLI repair, data channels.  ``server_channel``: the server opens that channel (selkies
    ``input``); ``dc_messages`` are sent on it once it is open instead of on one we open."""
    ans = parse_sdp(remote_sdp)
    vid = next(m for m in ans.media if m.kind == "video" and m.port)
    cands = [c.split() for c in vid.attrs_named("candidate")]
    want = "relay" if via_relay else "host"
    cand = next((c for c in cands if c[7] == want), None)
    if cand is None:
        raise RuntimeError(f"answer has no {want} candidate")
    host, port = cand[4], int(cand[5])
    r_ufrag, r_pwd = vid.attr("ice-ufrag"), vid.attr("ice-pwd")
    r_fp = vid.attr("fingerprint")
    loop = asyncio.get_running_loop()
    tr, cl = await loop.create_datagram_endpoint(_Client, remote_addr=(host, port))
    try:  # a 1080p IDR is hundreds of packets in one burst; the default buffer can overflow
        tr.get_extra_info("socket").setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    except OSError:
        pass
    deadline = time.monotonic() + timeout
    try:
        # ICE connectivity check (controlling, nominating)
        req = S.StunMessage(S.BINDING_REQUEST, None, [
            (S.A_USERNAME, f"{r_ufrag}:{ufrag}".encode()), (S.A_PRIORITY, struct.pack("!I", 1853824767)),
            (S.A_ICE_CONTROLLING, os.urandom(8)), (S.A_USE_CANDIDATE, b"")])
        # retransmitted like a browser's ICE agent (RFC 8445 / 5389: RTO from 250 ms, doubling):
        # a single lost check must not stall the session until the deadline
        req_bytes = req.encode(r_pwd.encode())
        res.stage = "ice"
        tr.sendto(req_bytes)
        res.ice_tx += 1
        rto, next_tx = 0.25, time.monotonic() + 0.25
        while True:
            try:
                d = await asyncio.wait_for(cl.q.get(), max(0.02, min(next_tx, deadline) - time.monotonic()))
            except asyncio.TimeoutError:
                if time.monotonic() > deadline:
                    raise
                tr.sendto(req_bytes)
                res.ice_tx += 1
                rto = min(rto * 2, 2.0)
                next_tx = time.monotonic() + rto
                continue
            res.datagrams += 1
            if S.is_stun(d):
                m = S.StunMessage.decode(d)
                if m.type == S.BINDING_SUCCESS and m.tid == req.tid:
                    if not m.check_integrity(r_pwd.encode()):
                        raise RuntimeError("bad MESSAGE-INTEGRITY in binding response")
                    break
        res.stage = "dtls"
        for dg in dtls.start():
            tr.sendto(dg)
        while not dtls.handshake_done:
            try:
                d = await asyncio.wait_for(cl.q.get(), 0.1)
            except asyncio.TimeoutError:
                for dg in dtls.tick():
                    tr.sendto(dg)
                if time.monotonic() > deadline:
                    raise RuntimeError("DTLS handshake timed out")
                continue
            if 20 <= d[0] <= 63:
                for dg in dtls.feed(d):
                    tr.sendto(dg)
            if dtls.failed:
                raise RuntimeError("DTLS failed: " + dtls.error)
        if dtls.peer_fingerprint.lower() != r_fp.lower():
            raise RuntimeError("server fingerprint mismatch")
        km = dtls.export_srtp_keys()
        rx_ctx: dict[int, object] = {}  # one SRTP receive context per SSRC (own rollover counter)

        def rx_for(pkt: bytes):
            ssrc = struct.unpack_from("!I", pkt, 4 if 192 <= pkt[1] <= 223 else 8)[0]
            if ssrc not in rx_ctx:
                rx_ctx[ssrc] = N.net.SrtpSession(km[16:32], km[46:60])  # server -> client
            return rx_ctx[ssrc]
        tx = N.net.SrtpSession(km[0:16], km[32:46])   # client -> server (RTCP)
        res.connect_ms = (time.monotonic() - t0) * 1000
        dc = None
        dc_id = -1
        app = next((m for m in ans.media if m.kind == "application" and m.port), None)

        def sctp_out(packets) -> None:
            for p in packets:
                for dg in dtls.write(p):
                    tr.sendto(dg)
        if dc_messages is not None:
            if app is None:
                raise RuntimeError("remote SDP has no data channel section")
            dc = N.net.DataChannelEndpoint(False, 5000, int(app.attr("sctp-port") or 5000))
            out = dc.connect()
            more = []
            if server_channel is None:
                dc_id, more = dc.open("input")
                if dc_audio_chunks:
                    _aid, amore = dc.open("audio", "", False, 0)
                    more += amore
                for msg in dc_messages:
                    more += dc.send(dc_id, msg.encode(), False)
                res.dc_sent = len(dc_messages)
            sctp_out(out + more)

        def on_dtls(d: bytes) -> None:
            nonlocal dc_id
            sctp_out_raw = dtls.feed(d)
            for dg in sctp_out_raw:
                tr.sendto(dg)
            for p in dtls.take_app_data():
                if dc is not None:
                    sctp_out(dc.feed(p))
            if dc is not None:
                for kind, cid, label, _proto, binary, data in dc.take_events():
                    if kind == 0 and server_channel is not None and label == server_channel and dc_id < 0:
                        dc_id = cid
                        more = []
                        for msg in dc_messages:
                            more += dc.send(cid, msg.encode(), False)
                        res.dc_sent = len(dc_messages)
                        res.dc_labels.append(label)
                        sctp_out(more)
                    elif kind == 1 and binary:
                        res.dc_audio.append(data)
                    elif kind == 1:
                        res.dc_received.append(data.decode("utf-8", "replace"))

        def dc_pending() -> bool:
            if dc is None:
                return False
            if dc.buffered_amount or not dc.is_open(dc_id) or len(res.dc_audio) < dc_audio_chunks:
                return True
            return dc_wait_stats and not any('"stats"' in m for m in res.dc_received)
        last_tick = time.monotonic()
        my_ssrc = secrets.randbits(32)
        hevc = " H265/90000" in res.answer
        vp8 = " VP8/90000" in res.answer

        def new_depk():
            return R.Vp8Depacketizer() if vp8 else (R.H265Depacketizer() if hevc else R.H264Depacketizer())
        depk = new_depk()
        pending: dict[int, bytes] = {}
        next_seq = None
        n_pkts = 0
        sent_pli = False
        nacked: set[int] = set()
        auto_nacked: set[int] = set()
        import random

        loss_rng = random.Random(1234)
        media_ssrc = 0
        gap_since = None       # when the oldest hole in `pending` appeared
        await_idr = False      # after giving up on a hole: drop AUs until the next IDR

        def dist(a: int, b: int) -> int:
            return (a - b) & 0xFFFF

        def is_idr(au: bytes) -> bool:
            if vp8:  # frame tag bit 0: 0 = key frame
                return len(au) > 0 and not au[0] & 1
            for n in N.net.split_annexb(au):
                t = (n[0] >> 1) & 0x3F if hevc else n[0] & 0x1F
                if (16 <= t <= 21) if hevc else t == 5:
                    return True
            return False

        def deliver() -> None:
            nonlocal next_seq, await_idr, sent_pli
            while next_seq in pending:  # in-order delivery to the depacketizer
                pk = pending.pop(next_seq)
                au = depk.push(pk)
                next_seq = (next_seq + 1) & 0xFFFF
                if au is None:
                    continue
                if await_idr and not is_idr(au):
                    res.dropped_aus += 1
                    continue
                await_idr = False
                if len(res.aus) >= n_frames:  # one burst can complete several AUs: keep exactly n
                    continue
                res.aus.append(au)
                res.rtp_ts.append(R.rtp_header(pk)["ts"])
                res.arrival_us.append(time.monotonic_ns() // 1000)
                res.arrival_wall.append(time.time())
                if pli_after and len(res.aus) == pli_after and not sent_pli:
                    tr.sendto(tx.protect_rtcp(R.build_pli(my_ssrc, media_ssrc)))
                    sent_pli = True

        def repair() -> None:
            """Generic NACK for every hole below the newest packet (once), as browsers do; a
            hole still open after 300 ms is abandoned: PLI, resync at the next IDR."""
            nonlocal gap_since, next_seq, await_idr, depk
            if not pending:
                gap_since = None
                return
            now = time.monotonic()
            if gap_since is None:
                gap_since = now
            if now - gap_since > 0.3:
                res.gave_up += 1
                tr.sendto(tx.protect_rtcp(R.build_pli(my_ssrc, media_ssrc)))
                next_seq = min(pending, key=lambda q: dist(q, next_seq))
                depk = new_depk()
                await_idr = True
                gap_since = None
                deliver()
                return
            hi = max(pending, key=lambda q: dist(q, next_seq))
            new = [q for q in ((next_seq + k) & 0xFFFF for k in range(dist(hi, next_seq)))
                   if q not in pending and q not in nacked and q not in auto_nacked]
            for i in range(0, len(new), 64):
                tr.sendto(tx.protect_rtcp(R.build_nack(my_ssrc, media_ssrc, new[i:i + 64])))
            auto_nacked.update(new)
            res.nacked += len(new)

        res.stage = "media"
        lite_ts = None       # lite: timestamp of the frame being received, its next expected seq
        lite_next = None
        lite_ok = True
        if lite == "native" and dc is None:
            # hand the socket to the native receive loop: stop the event loop's reader, count the
            # datagrams it already queued here, then recvmmsg() with the GIL released
            sock = tr.get_extra_info("socket")
            # (the transport owns the fd: the public remove_reader refuses it, and datagram
            # transports have no pause_reading -- the selector loop's own removal)
            loop._remove_reader(sock.fileno())
            rtcp = []
            while not cl.q.empty():
                d = cl.q.get_nowait()
                if not 128 <= d[0] <= 191:
                    continue
                if 192 <= d[1] <= 223:
                    rtcp.append(d)
                    continue
                if d[1] & 0x7F == 0:
                    continue
                seq, ts = struct.unpack_from("!HI", d, 2)
                res.packets += 1
                if ts != lite_ts:
                    lite_ts, lite_ok = ts, lite_next is None or seq == lite_next
                elif seq != lite_next:
                    lite_ok = False
                if lite_next is not None and seq != lite_next and ((seq - lite_next) & 0xFFFF) < 0x8000:
                    res.lost += (seq - lite_next) & 0xFFFF
                lite_next = (seq + 1) & 0xFFFF
                if d[1] & 0x80:
                    if lite_ok and len(res.aus) < n_frames:
                        res.aus.append(b"")
                        res.rtp_ts.append(ts)
                        res.arrival_us.append(time.monotonic_ns() // 1000)
                        res.arrival_wall.append(time.time())
                    lite_ts = None
            left = n_frames - len(res.aus)
            r = await loop.run_in_executor(
                None, lambda: N.net.count_rtp_frames(sock.fileno(), left, max(0.1, deadline - time.monotonic()),
                                                     -1 if lite_ts is None else lite_ts,
                                                     -1 if lite_next is None else lite_next, lite_ok))
            res.aus += [b""] * len(r["rtp_ts"])
            res.rtp_ts += r["rtp_ts"]
            res.arrival_us += r["arrival_us"]
            res.arrival_wall += r["arrival_wall"]
            res.packets += r["packets"]
            res.lost += r["lost"]
            res.datagrams += r["datagrams"]
            for d in rtcp + list(r["rtcp"]):  # the sender reports: RTP time <-> wall time
                p = rx_for(d).unprotect_rtcp(d)
                for x in (R.parse_rtcp(p) if p else []):
                    if x["pt"] == 200:
                        res.srs += 1
                        if "ntp" in x:
                            res.sr_map = (x["ntp"], x["rtp_ts"])
            if r["timed_out"]:
                raise asyncio.TimeoutError()
            res.stream = b""
            return
        while len(res.aus) < n_frames or dc_pending():
            if dc is not None and time.monotonic() - last_tick > 0.05:
                sctp_out(dc.tick())
                last_tick = time.monotonic()
            try:
                d = await asyncio.wait_for(cl.q.get(), 0.05)
            except asyncio.TimeoutError:
                if time.monotonic() > deadline:
                    raise
                if next_seq is not None:
                    repair()
                continue
            if time.monotonic() > deadline:
                raise asyncio.TimeoutError()
            if 20 <= d[0] <= 63:
                on_dtls(d)
                continue
            if not 128 <= d[0] <= 191:
                continue
            if 192 <= d[1] <= 223:
                p = rx_for(d).unprotect_rtcp(d)
                for x in (R.parse_rtcp(p) if p else []):
                    if x["pt"] == 200:
                        res.srs += 1
                        if "ntp" in x and x["ssrc"] == media_ssrc:  # the video sender's SR
                            res.sr_map = (x["ntp"], x["rtp_ts"])
                continue
            if lite:
                pt = d[1] & 0x7F
                if pt == 0:  # PCMU audio
                    continue
                seq, ts, ssrc = struct.unpack_from("!HII", d, 2)
                media_ssrc = ssrc
                res.packets += 1
                if ts != lite_ts:  # a new frame begins
                    lite_ts, lite_ok = ts, lite_next is None or seq == lite_next
                elif seq != lite_next:
                    lite_ok = False
                if lite_next is not None and seq != lite_next:
                    res.lost += (seq - lite_next) & 0xFFFF if ((seq - lite_next) & 0xFFFF) < 0x8000 else 0
                lite_next = (seq + 1) & 0xFFFF
                if d[1] & 0x80:  # marker: the frame's last packet
                    if lite_ok and len(res.aus) < n_frames:
                        res.aus.append(b"")
                        res.rtp_ts.append(ts)
                        res.arrival_us.append(time.monotonic_ns() // 1000)
                        res.arrival_wall.append(time.time())
                    lite_ts = None
                continue
            p = rx_for(d).unprotect_rtp(d)
            if not p:
                raise RuntimeError("SRTP authentication failed")
            h = R.rtp_header(p)
            if h["pt"] == 0:  # PCMU audio
                res.audio_payloads.append(h["payload"])
                res.audio_seqs.append(h["seq"])
                continue
            res.packets += 1
            media_ssrc = h["ssrc"]
            seq = h["seq"]
            if next_seq is None:
                next_seq = seq
            if seq in pending or ((seq - next_seq) & 0xFFFF) > 0x8000:
                continue  # duplicate / already delivered
            n_pkts += 1
            if simulate_loss and loss_rng.random() < simulate_loss and seq not in auto_nacked:
                continue  # lost on the "network": no test-mode NACK, the repair logic must notice
            if drop_seq_every and n_pkts % drop_seq_every == 0 and seq not in nacked:
                res.lost += 1
                nacked.add(seq)
                tr.sendto(tx.protect_rtcp(R.build_nack(my_ssrc, media_ssrc, [seq])))
                continue
            if seq in nacked:
                res.rtx += 1
            if seq in auto_nacked:
                res.recovered += 1
            pending[seq] = p
            deliver()
            repair()
        res.stream = b"".join(res.aus)
    finally:
        tr.close()
def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(description="headless WHEP viewer")
    ap.add_argument("url")
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--user")
    ap.add_argument("--password")
    a = ap.parse_args(argv)
    import aiohttp

    auth = aiohttp.BasicAuth(a.user, a.password) if a.user else None
    r = asyncio.run(whep_view(a.url, a.frames, auth))
    print(f"frames={len(r.aus)} packets={r.packets} bytes={len(r.stream)} connect_ms={r.connect_ms:.1f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
