"""WebRTC media transport (replaces GStreamer webrtcbin + libnice + libsrtp
of the reference's selkies pipeline, Dockerfile:439-444).

* Signalling: WHEP-style HTTP offer/answer (``POST /whep`` with the browser's SDP offer ->
  201 + SDP answer, ``DELETE /whep/<id>``); the selkies WebSocket relay (``/ws``) stays
  available for selkies-style clients.
* ICE-lite (RFC 8445 §2.5): one host candidate; connectivity checks answered with
  MESSAGE-INTEGRITY/FINGERPRINT-protected Binding responses; the browser (full agent,
  controlling) nominates.  TURN relays work because the browser allocates the relay.
* DTLS-SRTP (RFC 5764): native OpenSSL endpoint (server role, ``a=setup:passive``), peer
  certificate checked against the offer's ``a=fingerprint``; AES_CM_128_HMAC_SHA1_80 keys.
* Media: native RFC 6184 packetizer (STAP-A / FU-A), native SRTP, 90 kHz timestamps from
  the capture clock; RTCP PLI/FIR -> IDR, generic NACK -> retransmission from a packet
  history, periodic SR + SDES.
* Data channels (RFC 8831/8832 over SCTP over DTLS, RFC 8261): native SCTP association
  (``csrc/net/sctp.cpp``) on the same DTLS session; the browser opens the channel (selkies
  names it ``input``) and its text messages go through the same input parser as the
  WebSocket control channel (keyboard / mouse / clipboard / gamepad / bitrate); the server
  answers with ``{"type": "stats", ...}`` once a second.  A browser-opened ``audio`` channel
  (unordered, no retransmissions) receives 48 kHz stereo PCM chunks -- full-band audio
  without Opus, which the image lacks; PCMU over RTP remains for plain WHEP players.
"""
from __future__ import annotations

import asyncio
import logging
import os
import re
import secrets
import socket
import struct
import time
from collections import OrderedDict
from dataclasses import dataclass, field

from ..utils.tracing import trace
from . import rtp as R
from . import stun as S

log = logging.getLogger("mxdesk.webrtc")


def _native():
    from .. import native

    return native()


# ------------------------------------------------------------------ SDP
@dataclass
class MediaDesc:
    kind: str
    port: int
    proto: str
    fmts: list[str]
    attrs: list[str] = field(default_factory=list)

    def attr(self, name: str) -> str | None:
        for a in self.attrs:
            if a == name or a.startswith(name + ":"):
                return a[len(name) + 1:] if ":" in a else ""
        return None

    def attrs_named(self, name: str) -> list[str]:
        return [a[len(name) + 1:] for a in self.attrs if a.startswith(name + ":")]


@dataclass
class Sdp:
    session: list[str]
    media: list[MediaDesc]

    def attr(self, name: str) -> str | None:
        for line in self.session:
            if line.startswith("a=" + name + ":"):
                return line[len(name) + 3:]
        return None


def parse_sdp(text: str) -> Sdp:
    session: list[str] = []
    media: list[MediaDesc] = []
    for line in text.replace("\r\n", "\n").split("\n"):
        line = line.strip()
        if not line:
            continue
        if line.startswith("m="):
            kind, port, proto, *fmts = line[2:].split()
            media.append(MediaDesc(kind, int(port), proto, fmts))
        elif media:
            if line.startswith("a="):
                media[-1].attrs.append(line[2:])
        else:
            session.append(line)
    return Sdp(session, media)


def pick_h264(md: MediaDesc) -> str | None:
    """Payload type of a packetization-mode=1 H.264 codec the browser accepts for our
    Constrained Baseline stream (profile-level-id 42xxxx, preferring 42e0xx)."""
    h264 = [r.split()[0] for r in md.attrs_named("rtpmap") if re.search(r"\sH264/90000", r, re.I)]
    best = None
    for pt in h264:
        fmtp = next((f[len(pt) + 1:] for f in md.attrs_named("fmtp") if f.split()[0] == pt), "")
        params = dict(kv.split("=", 1) for kv in fmtp.split(";") if "=" in kv)
        if params.get("packetization-mode", "0") != "1":
            continue
        pli = params.get("profile-level-id", "42e01f").lower()
        if pli.startswith("42"):
            if pli.startswith("42e0"):
                return pt
            best = best or pt
    return best


def pick_h265(md: MediaDesc) -> str | None:
    """Payload type of an H.265 (RFC 7798) codec whose profile is Main (profile-id 1 or
    absent) for our Main-profile HEVC stream."""
    for pt in [r.split()[0] for r in md.attrs_named("rtpmap") if re.search(r"\sH265/90000", r, re.I)]:
        fmtp = next((f[len(pt) + 1:] for f in md.attrs_named("fmtp") if f.split()[0] == pt), "")
        params = dict(kv.strip().split("=", 1) for kv in fmtp.split(";") if "=" in kv)
        if params.get("profile-id", "1") == "1" and params.get("tx-mode", "SRST").upper() == "SRST":
            return pt
    return None


def pick_vp8(md: MediaDesc) -> str | None:
    """Payload type of the offer's VP8 (RFC 7741) codec."""
    return next((r.split()[0] for r in md.attrs_named("rtpmap") if re.search(r"\sVP8/90000", r, re.I)), None)


_PICKERS = {"h264": pick_h264, "hevc": pick_h265, "vp8": pick_vp8}
_MISSING = {"h264": "offer has no H.264 (packetization-mode=1, baseline-compatible) video section",
            "hevc": "offer has no H.265 (Main profile) video section",
            "vp8": "offer has no VP8 video section"}


def codec_sdp(codec: str, level_idc: int) -> tuple[str, str]:
    """(rtpmap, fmtp) of the stream's codec; an empty fmtp means no a=fmtp line (VP8)."""
    if codec == "hevc":
        return "H265/90000", f"profile-id=1;tier-flag=0;level-id={level_idc};tx-mode=SRST"
    if codec == "vp8":
        return "VP8/90000", ""
    return "H264/90000", f"level-asymmetry-allowed=1;packetization-mode=1;profile-level-id=42e0{level_idc:02x}"


@dataclass
class Answer:
    sdp: str
    pt: int
    mid: str
    remote_ufrag: str
    remote_pwd: str
    remote_fingerprint: str
    audio_pt: int | None = None  # PCMU (0) when the offer has an audio section and audio is on
    audio_mid: str | None = None
    dc_mid: str | None = None        # accepted m=application (SCTP data channels)
    remote_sctp_port: int = 5000


def _has_pcmu(md: MediaDesc) -> bool:
    return "0" in md.fmts or any(re.search(r"\sPCMU/8000", r, re.I) for r in md.attrs_named("rtpmap"))


def build_answer(offer_text: str, ice_ufrag: str, ice_pwd: str, fingerprint: str, host: str, port: int, ssrc: int,
                 level_idc: int = 0x2A, audio_ssrc: int | None = None, extra_hosts: list[str] | None = None,
                 codec: str = "h264", datachannel: bool = True, max_message: int = 262144,
                 relay_candidates: list[str] | None = None) -> Answer:
    """Answer one video section in the stream's codec (H.264 packetization-mode 1, H.265 with
    ``codec="hevc"`` -- ``level_idc`` is then general_level_idc -- or VP8) and, with ``audio_ssrc``,
    one PCMU audio section, and with ``datachannel`` one ``UDP/DTLS/SCTP webrtc-datachannel``
    section (RFC 8841); everything else is rejected with port 0.  All accepted sections are
    BUNDLEd onto the single ICE-lite host candidate."""
    pick = _PICKERS[codec]
    rtpmap, fmtp = codec_sdp(codec, level_idc)
    offer = parse_sdp(offer_text)
    lines = ["v=0", f"o=mxdesk {secrets.randbelow(1 << 62)} 2 IN IP4 {host}", "s=mxdesk", "t=0 0", "a=ice-lite",
             "a=msid-semantic: WMS mxdesk"]
    out_media: list[str] = []
    chosen = None
    audio = None  # (pt, mid)
    dc = None     # (mid, remote sctp-port)
    bundle: list[str] = []
    hosts = [host] + [h for h in (extra_hosts or []) if h != host]
    cands = [f"a=candidate:{k + 1} 1 udp {2130706431 - k} {h} {port} typ host" for k, h in enumerate(hosts)]
    cands += list(relay_candidates or [])
    transport = [f"c=IN IP4 {host}", *cands, "a=end-of-candidates",
                 f"a=ice-ufrag:{ice_ufrag}", f"a=ice-pwd:{ice_pwd}", f"a=fingerprint:{fingerprint}", "a=setup:passive"]
    for md in offer.media:
        mid = md.attr("mid") or str(len(bundle) + len(out_media))
        pt = pick(md) if (md.kind == "video" and chosen is None) else None
        ufrag = md.attr("ice-ufrag") or offer.attr("ice-ufrag")
        pwd = md.attr("ice-pwd") or offer.attr("ice-pwd")
        fp = md.attr("fingerprint") or offer.attr("fingerprint")
        if pt is not None:
            chosen = Answer("", int(pt), mid, ufrag or "", pwd or "", fp or "")
            bundle.append(mid)
            out_media += [f"m=video {port} UDP/TLS/RTP/SAVPF {pt}", *transport,
                          f"a=mid:{mid}", "a=sendonly", "a=rtcp-mux", "a=rtcp-rsize",
                          f"a=rtpmap:{pt} {rtpmap}", f"a=rtcp-fb:{pt} nack", f"a=rtcp-fb:{pt} nack pli",
                          f"a=rtcp-fb:{pt} ccm fir", f"a=rtcp-fb:{pt} goog-remb",
                          *([f"a=fmtp:{pt} {fmtp}"] if fmtp else []),
                          f"a=ssrc:{ssrc} cname:mxdesk", f"a=ssrc:{ssrc} msid:mxdesk video0"]
            continue
        if md.kind == "audio" and audio is None and audio_ssrc is not None and _has_pcmu(md):
            audio = (0, mid)
            bundle.append(mid)
            out_media += [f"m=audio {port} UDP/TLS/RTP/SAVPF 0", *transport,
                          f"a=mid:{mid}", "a=sendonly", "a=rtcp-mux", "a=rtpmap:0 PCMU/8000",
                          f"a=ssrc:{audio_ssrc} cname:mxdesk", f"a=ssrc:{audio_ssrc} msid:mxdesk audio0"]
            continue
        if md.kind == "application" and dc is None and datachannel and md.proto.upper().endswith("DTLS/SCTP") \
                and "webrtc-datachannel" in md.fmts:
            dc = (mid, int(md.attr("sctp-port") or 5000))
            bundle.append(mid)
            out_media += [f"m=application {port} UDP/DTLS/SCTP webrtc-datachannel", *transport,
                          f"a=mid:{mid}", "a=sctp-port:5000", f"a=max-message-size:{max_message}"]
            continue
        # reject (legacy SCTP syntax, second video, audio when disabled)
        out_media += [f"m={md.kind} 0 {md.proto} {md.fmts[0] if md.fmts else '0'}", "c=IN IP4 0.0.0.0",
                      f"a=mid:{mid}", "a=inactive"]
    if chosen is None:
        raise ValueError(_MISSING[codec])
    if audio is not None:
        chosen.audio_pt, chosen.audio_mid = audio
    if dc is not None:
        chosen.dc_mid, chosen.remote_sctp_port = dc
    lines.insert(4, "a=group:BUNDLE " + " ".join(bundle))
    chosen.sdp = "\r\n".join(lines + out_media) + "\r\n"
    return chosen


def build_offer(ice_ufrag: str, ice_pwd: str, fingerprint: str, host: str, port: int, ssrc: int,
                level_idc: int = 0x2A, audio_ssrc: int | None = None, extra_hosts: list[str] | None = None,
                codec: str = "h264", datachannel: bool = True, max_message: int = 262144,
                relay_candidates: list[str] | None = None, video_pt: int = 96) -> str:
    """Server-side OFFER for the selkies signalling protocol, where the streaming peer offers
    (upstream webrtcbin): one sendonly video section in the stream's codec, optionally one
    PCMU audio section and one SCTP data-channel section, all BUNDLEd on the ICE-lite host
    candidate(s), DTLS ``actpass`` (browsers answer ``active``: we stay the DTLS server)."""
    rtpmap, fmtp = codec_sdp(codec, level_idc)
    hosts = [host] + [h for h in (extra_hosts or []) if h != host]
    cands = [f"a=candidate:{k + 1} 1 udp {2130706431 - k} {h} {port} typ host" for k, h in enumerate(hosts)]
    cands += list(relay_candidates or [])
    transport = [f"c=IN IP4 {host}", *cands, "a=end-of-candidates",
                 f"a=ice-ufrag:{ice_ufrag}", f"a=ice-pwd:{ice_pwd}", f"a=fingerprint:{fingerprint}", "a=setup:actpass"]
    pt = video_pt
    mids = ["0"]
    media = [f"m=video {port} UDP/TLS/RTP/SAVPF {pt}", *transport, "a=mid:0", "a=sendonly", "a=rtcp-mux",
             "a=rtcp-rsize", f"a=rtpmap:{pt} {rtpmap}", f"a=rtcp-fb:{pt} nack", f"a=rtcp-fb:{pt} nack pli",
             f"a=rtcp-fb:{pt} ccm fir", f"a=rtcp-fb:{pt} goog-remb", *([f"a=fmtp:{pt} {fmtp}"] if fmtp else []),
             f"a=ssrc:{ssrc} cname:mxdesk", f"a=ssrc:{ssrc} msid:mxdesk video0"]
    if audio_ssrc is not None:
        mids.append(str(len(mids)))
        media += [f"m=audio {port} UDP/TLS/RTP/SAVPF 0", *transport, f"a=mid:{mids[-1]}", "a=sendonly", "a=rtcp-mux",
                  "a=rtpmap:0 PCMU/8000", f"a=ssrc:{audio_ssrc} cname:mxdesk", f"a=ssrc:{audio_ssrc} msid:mxdesk audio0"]
    if datachannel:
        mids.append(str(len(mids)))
        media += [f"m=application {port} UDP/DTLS/SCTP webrtc-datachannel", *transport, f"a=mid:{mids[-1]}",
                  "a=sctp-port:5000", f"a=max-message-size:{max_message}"]
    lines = ["v=0", f"o=mxdesk {secrets.randbelow(1 << 62)} 2 IN IP4 {host}", "s=mxdesk", "t=0 0", "a=ice-lite",
             "a=group:BUNDLE " + " ".join(mids), "a=msid-semantic: WMS mxdesk"]
    return "\r\n".join(lines + media) + "\r\n"


def parse_answer(answer_text: str, video_pt: int) -> tuple[Answer, str]:
    """The browser's ANSWER to build_offer(): negotiated sections, its ICE / DTLS parameters and
    its DTLS role (``a=setup``)."""
    ans = parse_sdp(answer_text)
    chosen = None
    audio = dc = None
    setup = ans.attr("setup") or ""
    for md in ans.media:
        if md.port == 0:
            continue
        mid = md.attr("mid") or ""
        setup = md.attr("setup") or setup
        if md.kind == "video" and chosen is None:
            if str(video_pt) not in md.fmts:
                raise ValueError("answer does not accept the offered video format")
            chosen = Answer(answer_text, video_pt, mid, md.attr("ice-ufrag") or ans.attr("ice-ufrag") or "",
                            md.attr("ice-pwd") or ans.attr("ice-pwd") or "",
                            md.attr("fingerprint") or ans.attr("fingerprint") or "")
        elif md.kind == "audio" and audio is None and "0" in md.fmts:
            audio = (0, mid)
        elif md.kind == "application" and dc is None:
            dc = (mid, int(md.attr("sctp-port") or 5000))
    if chosen is None:
        raise ValueError("answer rejected the video section")
    if audio is not None:
        chosen.audio_pt, chosen.audio_mid = audio
    if dc is not None:
        chosen.dc_mid, chosen.remote_sctp_port = dc
    return chosen, setup.strip()


def local_ips() -> list[str]:
    """Non-loopback IPv4 addresses of this host (one ICE host candidate each)."""
    try:
        import psutil

        out = [a.address for addrs in psutil.net_if_addrs().values() for a in addrs
               if a.family == socket.AF_INET and not a.address.startswith("127.")]
        return sorted(set(out))
    except Exception:
        return []


def local_ip() -> str:
    env = os.environ.get("MXDESK_WEBRTC_HOST")
    if env:
        return env
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.connect(("10.255.255.255", 1))
        ip = s.getsockname()[0]
        s.close()
        return ip
    except OSError:
        return "127.0.0.1"


# ------------------------------------------------------------------ congestion control
class CongestionController:
    """``SELKIES_CONGESTION_CONTROL``: steer the encoder's CBR target from the receiver's
    feedback -- REMB estimates (upper bound) and RTCP receiver-report loss (multiplicative
    decrease above 10 % loss, +8 % additive-style probe below 2 %), never above the configured
    bitrate."""

    def __init__(self, pipeline, enabled: bool, min_kbps: int = 500):
        self.pipeline = pipeline
        self.enabled = enabled
        self.max_kbps = int(getattr(pipeline, "bitrate_kbps", 0) or 8000)
        self.kbps = self.max_kbps
        self.min_kbps = min_kbps
        self.remb_kbps: int | None = None

    def _apply(self, kbps: float) -> None:
        cap = min(self.max_kbps, self.remb_kbps or self.max_kbps)
        new = int(max(self.min_kbps, min(cap, kbps)))
        if self.enabled and abs(new - self.kbps) >= max(50, self.kbps // 50):
            self.pipeline.set_bitrate(new)
        self.kbps = new

    def on_remb(self, bps: int) -> None:
        self.remb_kbps = max(self.min_kbps, int(bps * 0.95) // 1000)
        self._apply(self.kbps)

    def on_loss(self, fraction: float) -> None:
        if fraction > 0.10:
            self._apply(self.kbps * (1.0 - 0.5 * fraction))
        elif fraction < 0.02:
            self._apply(self.kbps * 1.08)


class RelayAddr(tuple):
    """A browser address reached through our TURN allocation (sends go via the relay)."""


def turn_relay_settings(cfg) -> dict | None:
    """Server-side TURN relay settings from the TURN_* config (shared-secret HMAC or legacy
    credentials), or None when no TURN server is configured / MXDESK_TURN_RELAY=false."""
    if cfg is None or not getattr(cfg, "turn_host", None) or not getattr(cfg, "turn_relay", True):
        return None
    from .turn import hmac_credentials

    if getattr(cfg, "turn_shared_secret", None):
        user, pw = hmac_credentials(cfg.turn_shared_secret, "mxdesk-server")
    elif getattr(cfg, "turn_username", None) and getattr(cfg, "turn_password", None):
        user, pw = cfg.turn_username, cfg.turn_password
    else:
        return None
    return {"host": cfg.turn_host, "port": int(cfg.turn_port or 3478), "username": user, "password": pw,
            "protocol": (cfg.turn_protocol or "udp").lower(), "tls": bool(cfg.turn_tls)}


# ------------------------------------------------------------------ peer
class WebRtcPeer(asyncio.DatagramProtocol):
    HISTORY = 1024

    def __init__(self, pipeline, offer_sdp: str | None, host: str | None = None, port: int = 0, level_idc: int = 0x2A,
                 audio=None, congestion_control: bool = False, on_input=None, turn: dict | None = None,
                 server_channels: tuple[str, ...] = ()):
        """``offer_sdp``: the browser's offer (WHEP, we answer); None for the selkies protocol,
        where we offer (start_offer / accept_answer).  ``server_channels``: data channels we open
        once SCTP is up (selkies opens ``input`` from the server side)."""
        N = _native()
        self.server_channels = tuple(server_channels)
        self.video_pt = 96
        self.turn = turn          # server-side relay settings (host, port, username, password, protocol, tls)
        self.relay = None         # TurnClient once allocated
        self.on_input = on_input  # callback(str) for data-channel text messages
        self.dc = None            # DataChannelEndpoint once DTLS is up and the offer had m=application
        self.dc_channels: dict[int, str] = {}
        self.pipeline = pipeline
        self.audio = audio
        self.audio_ssrc = (secrets.randbits(32) | 1) if audio is not None else None
        self.srtp_tx_audio = None
        self.asub = None
        self.id = secrets.token_hex(8)
        self.ufrag = secrets.token_hex(4)
        self.pwd = secrets.token_hex(16)
        self.dtls = N.net.DtlsEndpoint(True)
        self.ssrc = secrets.randbits(32) | 1
        explicit = host or os.environ.get("MXDESK_WEBRTC_HOST")
        self.host = explicit or local_ip()
        # no explicit host: listen on all interfaces and offer every address as a candidate
        self.bind_host = self.host if explicit else "0.0.0.0"
        self.extra_hosts = [] if explicit else local_ips()
        self.bind_port = port
        self.level_idc = level_idc
        self.offer_sdp = offer_sdp
        self.transport: asyncio.DatagramTransport | None = None
        self.remote: tuple[str, int] | None = None
        self.srtp_tx = None
        self.srtp_rx = None
        self.pkt = None
        self.history: OrderedDict[int, bytes] = OrderedDict()
        # native send path (packetize + NACK history + SRTP + sendto in one GIL-free call) for a
        # direct UDP remote; relayed remotes keep the Python path
        self._tx_peer = None  # (remote, net.UdpPeer)
        self._tx_hist = None  # net.RtpHistory
        self.answer: Answer | None = None
        self.sub = None
        self.tasks: list[asyncio.Task] = []
        self.closed = asyncio.Event()
        self.stats = {"stun": 0, "dtls_in": 0, "rtp_out": 0, "rtcp_in": 0, "pli": 0, "nack": 0, "rtx": 0,
                      "dc_in": 0, "dc_out": 0}
        self.last_consent = time.monotonic()
        self.ts0: int | None = None
        self.cc = CongestionController(pipeline, enabled=congestion_control)

    async def _bind(self) -> int:
        loop = asyncio.get_running_loop()
        self.transport, _ = await loop.create_datagram_endpoint(lambda: self,
                                                                local_addr=(self.bind_host, self.bind_port))
        port = self.transport.get_extra_info("sockname")[1]
        try:  # an IDR is a burst of hundreds of packets: room in the kernel queue instead of drops
            sock = self.transport.get_extra_info("socket")
            sock.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
            sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 20)
        except OSError:
            pass
        return port

    def _codec_level(self) -> tuple[str, int]:
        codec = getattr(self.pipeline, "codec", "h264")
        level = self.level_idc
        if codec == "hevc":
            p = self.pipeline
            level = _native().hevc_level(p.out_w, p.out_h, p.fps)
        return codec, level

    def _media_ready(self, codec: str) -> None:
        net = _native().net
        if codec == "vp8":
            self.pkt = net.RtpVp8Packetizer(self.ssrc, self.answer.pt, 1150, secrets.randbits(16), secrets.randbits(15))
        else:
            packetizer = net.RtpH265Packetizer if codec == "hevc" else net.RtpH264Packetizer
            self.pkt = packetizer(self.ssrc, self.answer.pt, 1150, secrets.randbits(16))
        self.tasks.append(asyncio.create_task(self._timers()))

    async def start(self) -> str:
        """WHEP: answer the browser's offer."""
        port = await self._bind()
        codec, level = self._codec_level()
        relay_cands = []
        if self.turn:
            relay_cands = await self._allocate_relay()
        self.answer = build_answer(self.offer_sdp, self.ufrag, self.pwd, self.dtls.fingerprint, self.host, port,
                                   self.ssrc, level, self.audio_ssrc, self.extra_hosts, codec=codec,
                                   relay_candidates=relay_cands)
        self._media_ready(codec)
        return self.answer.sdp

    async def start_offer(self) -> str:
        """selkies protocol: our offer (the answer comes back through accept_answer)."""
        port = await self._bind()
        codec, level = self._codec_level()
        relay_cands = []
        if self.turn:
            relay_cands = await self._allocate_relay()
        self.local_offer = build_offer(self.ufrag, self.pwd, self.dtls.fingerprint, self.host, port, self.ssrc, level,
                                       self.audio_ssrc, self.extra_hosts, codec=codec, relay_candidates=relay_cands,
                                       video_pt=self.video_pt)
        self._codec = codec
        return self.local_offer

    async def accept_answer(self, answer_sdp: str) -> None:
        answer, setup = parse_answer(answer_sdp, self.video_pt)
        if setup == "passive":  # our certificate / fingerprint is the DTLS server's
            raise ValueError("answer asks us to be the DTLS client (a=setup:passive); answer with active")
        self.answer = answer
        self.offer_sdp = answer_sdp  # remote description (TURN permissions for its candidates)
        self._media_ready(self._codec)
        if self.relay is not None:
            await self.add_remote_candidates(answer_sdp)

    async def _allocate_relay(self) -> list[str]:
        """TURN allocation + permissions for the offer's candidates -> relay candidate lines."""
        from .turn_client import TurnClient, TurnError, offer_candidate_ips

        t = self.turn
        self.relay = TurnClient(t["host"], t["port"], t["username"], t["password"], t.get("protocol", "udp"),
                                bool(t.get("tls", False)), on_data=self._on_relay_data)
        try:
            rip, rport = await asyncio.wait_for(self.relay.allocate(), float(t.get("timeout", 5.0)))
            ips = offer_candidate_ips(self.offer_sdp) if self.offer_sdp else []
            if ips:
                await self.relay.create_permission(ips)
        except (TurnError, OSError, asyncio.TimeoutError) as e:
            log.warning("TURN relay unavailable (%s); answering with host candidates only", e)
            self.relay.close()
            self.relay = None
            return []
        mip, mport = self.relay.mapped or (rip, rport)
        return [f"a=candidate:9 1 udp 16777215 {rip} {rport} typ relay raddr {mip} rport {mport}"]

    # ------------------------------------------------------------------ datagrams
    def datagram_received(self, data: bytes, addr) -> None:
        if not data:
            return
        b = data[0]
        try:
            if b < 4 and S.is_stun(data):
                self._on_stun(data, addr)
            elif 20 <= b <= 63:
                self.stats["dtls_in"] += 1
                self._send_all(self.dtls.feed(data), addr)
                if self.dtls.handshake_done and self.srtp_tx is None:
                    self._on_dtls_done()
                for pkt in self.dtls.take_app_data():
                    self._on_sctp(pkt, addr)
            elif 128 <= b <= 191 and len(data) > 1 and 192 <= data[1] <= 223:
                self._on_rtcp(data)
        except Exception:
            log.exception("bad datagram from %s", addr)

    def _send_all(self, dgrams, addr) -> None:
        for d in dgrams:
            self._sendto(d, addr)

    def _sendto(self, data: bytes, addr) -> None:
        if isinstance(addr, RelayAddr):
            if self.relay is not None:
                self.relay.send(data, tuple(addr))
        elif self.transport is not None:
            self.transport.sendto(data, addr)

    def _on_relay_data(self, payload: bytes, peer) -> None:
        self.datagram_received(payload, RelayAddr(peer))

    def _on_stun(self, data: bytes, addr) -> None:
        m = S.StunMessage.decode(data)
        if m.type != S.BINDING_REQUEST:
            return
        user = (m.get(S.A_USERNAME) or b"").decode(errors="replace")
        if not user.startswith(self.ufrag + ":") or not m.check_integrity(self.pwd.encode()):
            err = S.StunMessage(S.BINDING_ERROR, m.tid, [(S.A_ERROR_CODE, struct.pack("!HBB", 0, 4, 1) + b"Unauthorized")])
            self._sendto(err.encode(), addr)
            return
        self.stats["stun"] += 1
        self.last_consent = time.monotonic()
        resp = S.StunMessage(S.BINDING_SUCCESS, m.tid, [(S.A_XOR_MAPPED_ADDRESS, S.xor_address(addr[0], addr[1], m.tid))])
        self._sendto(resp.encode(self.pwd.encode()), addr)
        if self.remote is None or m.get(S.A_USE_CANDIDATE) is not None:
            if isinstance(addr, RelayAddr) and addr != self.remote and self.relay is not None:
                # nominated through our relay: bind a channel (4-byte framing per packet)
                self.tasks.append(asyncio.ensure_future(self._bind_channel(tuple(addr))))
            self.remote = addr

    def _on_dtls_done(self) -> None:
        N = _native()
        fp = self.dtls.peer_fingerprint
        want = (self.answer.remote_fingerprint or "").strip()
        if want and fp.lower() != want.lower():
            log.error("DTLS fingerprint mismatch: %s != %s", fp, want)
            self.close()
            return
        km = self.dtls.export_srtp_keys()
        ck, sk, cs, ss = km[:16], km[16:32], km[32:46], km[46:60]
        self.srtp_tx = N.net.SrtpSession(sk, ss)
        self.srtp_rx = N.net.SrtpSession(ck, cs)
        log.info("WebRTC peer %s: DTLS-SRTP up (%s)", self.id, self.dtls.srtp_profile)
        self.sub = self.pipeline.subscribe(asyncio.get_running_loop())
        self.tasks.append(asyncio.create_task(self._send_loop()))
        if self.answer.audio_pt is not None and self.audio is not None:
            # separate SRTP context per SSRC (own rollover counter / SRTCP index), same keys
            self.srtp_tx_audio = N.net.SrtpSession(sk, ss)
            self.asub = self.audio.subscribe(asyncio.get_running_loop())
            self.tasks.append(asyncio.create_task(self._audio_loop()))

    async def _bind_channel(self, peer) -> None:
        from .turn_client import TurnError

        try:
            await self.relay.channel_bind(peer)
        except (TurnError, OSError) as e:
            log.warning("TURN ChannelBind failed (Send indications stay in use): %s", e)

    async def add_remote_candidates(self, sdp_fragment: str) -> int:
        """Trickled browser candidates (WHEP PATCH): TURN permissions for their addresses."""
        from .turn_client import TurnError, offer_candidate_ips

        ips = offer_candidate_ips(sdp_fragment)
        if ips and self.relay is not None:
            try:
                await self.relay.create_permission(ips)
            except (TurnError, OSError) as e:
                log.warning("TURN CreatePermission failed: %s", e)
        return len(ips)

    # ------------------------------------------------------------------ data channels
    def _sctp_out(self, packets, addr=None) -> None:
        addr = addr or self.remote
        if addr is None:
            return
        for p in packets:
            self._send_all(self.dtls.write(p), addr)

    def _on_sctp(self, pkt: bytes, addr) -> None:
        if self.dc is None:
            if self.answer is None or self.answer.dc_mid is None:
                return
            # we are the DTLS server: odd stream ids for channels we open; the browser opens
            self.dc = _native().net.DataChannelEndpoint(True, 5000, self.answer.remote_sctp_port)
            for label in self.server_channels:  # queued until the association is up
                cid, out = self.dc.open(label)
                self.dc_channels[cid] = label
                self._sctp_out(out, addr)
        self._sctp_out(self.dc.feed(pkt), addr)
        self._dc_events()

    def _dc_events(self) -> None:
        for kind, cid, label, _proto, binary, data in self.dc.take_events():
            if kind == 0:
                self.dc_channels[cid] = label
                log.info("WebRTC peer %s: data channel %d '%s' open", self.id, cid, label)
                if label == "audio" and self.audio is not None:
                    self.tasks.append(asyncio.ensure_future(self._dc_audio_loop(cid)))
            elif kind == 1:
                self.stats["dc_in"] += 1
                if self.on_input is not None and not binary:
                    try:
                        self.on_input(data.decode("utf-8", "replace"))
                    except Exception:
                        log.exception("data-channel message %r", data[:64])
            elif kind == 2:
                self.dc_channels.pop(cid, None)

    async def _dc_audio_loop(self, cid: int) -> None:
        """48 kHz stereo PCM (``MXA1`` chunks, 10 ms) on a browser-opened ``audio`` channel --
        full-band audio for WebRTC viewers without an Opus encoder; the browser opens it
        unordered with maxRetransmits 0, so late chunks are dropped, never waited for."""
        from ..audio.pipeline import audio_message

        sub = self.audio.subscribe(asyncio.get_running_loop())
        try:
            while not self.closed.is_set() and cid in self.dc_channels:
                ch = await sub.queue.get()
                if self.dc.buffered_amount > 256 * 1024:  # congested: real-time audio is dropped, not queued
                    self.stats["dc_audio_drop"] = self.stats.get("dc_audio_drop", 0) + 1
                    continue
                self._sctp_out(self.dc.send(cid, audio_message(ch), True))
                self.stats["dc_audio"] = self.stats.get("dc_audio", 0) + 1
        finally:
            self.audio.unsubscribe(sub)

    def dc_send(self, text: str, label: str | None = None) -> bool:
        """Send one text message on the first open channel (or the one named ``label``)."""
        if self.dc is None:
            return False
        for cid, lab in self.dc_channels.items():
            if (label is None or lab == label) and self.dc.is_open(cid):
                self._sctp_out(self.dc.send(cid, text.encode(), False))
                self.stats["dc_out"] += 1
                return True
        return False

    def _dc_stats(self) -> str:
        import json

        m = getattr(self.pipeline, "metrics", None)
        snap = m.summary() if m is not None and hasattr(m, "summary") else {}
        return json.dumps({"type": "stats", "rtp_out": self.stats["rtp_out"], "rtx": self.stats["rtx"],
                           "kbps": self.cc.kbps, **{k: v for k, v in snap.items() if isinstance(v, (int, float))}})

    def _on_rtcp(self, data: bytes) -> None:
        if self.srtp_rx is None:
            return
        pkt = self.srtp_rx.unprotect_rtcp(data)
        if not pkt:
            return
        self.stats["rtcp_in"] += 1
        for p in R.parse_rtcp(pkt):
            if p["pt"] == 206 and p["fmt"] in (1, 4):  # PLI / FIR
                self.stats["pli"] += 1
                self.pipeline.request_idr("pli" if p["fmt"] == 1 else "fir")
            elif "remb_bps" in p:
                self.cc.on_remb(p["remb_bps"])
            elif p["pt"] in (200, 201) and p.get("reports"):
                for rb in p["reports"]:
                    if rb["ssrc"] == self.ssrc:
                        self.cc.on_loss(rb["fraction_lost"])
            elif p["pt"] == 205 and p["fmt"] == 1:
                self.stats["nack"] += 1
                for seq in p.get("nack", []):
                    raw = self._tx_hist.get(seq) if self._tx_hist is not None else None
                    if raw is None:
                        raw = self.history.get(seq)
                    if raw is not None and self.remote is not None:
                        self._sendto(self.srtp_tx.protect_rtp(raw), self.remote)
                        self.stats["rtx"] += 1

    # ------------------------------------------------------------------ media
    async def _send_loop(self) -> None:
        while not self.closed.is_set():
            fr = await self.sub.queue.get()
            if self.remote is None:
                continue
            if self.ts0 is None:
                self.ts0 = fr.t_capture_us
            ts = ((fr.t_capture_us - self.ts0) * 9 // 100) & 0xFFFFFFFF  # 90 kHz
            peer = self._native_peer()
            if peer is not None:
                with trace("mxdesk.webrtc.send_au(native)"):
                    self.stats["rtp_out"] += _native().net.send_au(self.pkt, self.srtp_tx, self._tx_hist, peer,
                                                                   fr.au, ts)
                self.last_ts = ts
                continue
            with trace("mxdesk.webrtc.packetize+srtp+send"):
                for raw in self.pkt.packetize(fr.au, ts):
                    seq = struct.unpack_from("!H", raw, 2)[0]
                    self.history[seq] = raw
                    if len(self.history) > self.HISTORY:
                        self.history.popitem(last=False)
                    self._sendto(self.srtp_tx.protect_rtp(raw), self.remote)
                    self.stats["rtp_out"] += 1
            self.last_ts = ts

    def _native_peer(self):
        """net.UdpPeer for the current remote when it is a direct UDP address (None: relayed or
        no socket -- the Python path sends)."""
        r = self.remote
        if r is None or isinstance(r, RelayAddr) or self.transport is None:
            return None
        if self._tx_peer is None or self._tx_peer[0] != r:
            sock = self.transport.get_extra_info("socket")
            if sock is None:
                return None
            try:
                peer = _native().net.UdpPeer(sock.fileno(), str(r[0]), int(r[1]))
            except (ValueError, OSError):
                return None
            self._tx_peer = (r, peer)
            if self._tx_hist is None:
                self._tx_hist = _native().net.RtpHistory(self.HISTORY)
        return self._tx_peer[1]

    async def _audio_loop(self) -> None:
        """48 kHz stereo chunks -> 8 kHz mono (native FIR decimator) -> 20 ms PCMU packets."""
        import numpy as np

        A = _native().audio
        dec = A.Decimator(6, 2)
        pending = np.zeros(0, np.int16)
        seq = secrets.randbits(16)
        ts = secrets.randbits(32)
        first = True
        self.audio_packets = 0
        while not self.closed.is_set():
            ch = await self.asub.queue.get()
            pending = np.concatenate([pending, dec.process(ch.pcm)])
            while len(pending) >= 160 and self.remote is not None:
                frame, pending = pending[:160], pending[160:]
                hdr = struct.pack("!BBHII", 0x80, (0x80 if first else 0) | self.answer.audio_pt, seq, ts,
                                  self.audio_ssrc)
                self._sendto(self.srtp_tx_audio.protect_rtp(hdr + A.encode_ulaw(frame)), self.remote)
                first = False
                seq = (seq + 1) & 0xFFFF
                ts = (ts + 160) & 0xFFFFFFFF
                self.audio_packets += 1
                self.audio_octets = getattr(self, "audio_octets", 0) + 160
                self.audio_ts = ts

    async def _timers(self) -> None:
        last_sr = 0.0
        while not self.closed.is_set():
            await asyncio.sleep(0.05)
            if self.remote is not None and not self.dtls.handshake_done:
                self._send_all(self.dtls.tick(), self.remote)
            now = time.monotonic()
            if self.dc is not None:
                self._sctp_out(self.dc.tick())
                self._dc_events()
                if now - getattr(self, "_last_dc_stats", 0.0) > 1.0 and self.dc_channels:
                    self.dc_send(self._dc_stats())
                    self._last_dc_stats = now
            if self.srtp_tx is not None and self.remote is not None and now - last_sr > 1.0:
                # the SR's RTP timestamp is the RTP clock NOW (capture clock, 90 kHz), so a receiver
                # maps any frame's timestamp to the wall clock (A/V sync; end-to-end latency)
                rtp_now = ((_native().now_us() - self.ts0) * 9 // 100) & 0xFFFFFFFF if self.ts0 is not None else 0
                sr = R.build_sr(self.ssrc, rtp_now, self.pkt.packets, self.pkt.octets)
                self._sendto(self.srtp_tx.protect_rtcp(sr), self.remote)
                if self.srtp_tx_audio is not None and getattr(self, "audio_packets", 0):
                    asr = R.build_sr(self.audio_ssrc, self.audio_ts, self.audio_packets, self.audio_octets)
                    self._sendto(self.srtp_tx_audio.protect_rtcp(asr), self.remote)
                last_sr = now
            if now - self.last_consent > 30.0:  # consent freshness (RFC 7675)
                log.info("WebRTC peer %s: consent expired", self.id)
                self.close()

    def close(self) -> None:
        if self.closed.is_set():
            return
        self.closed.set()
        if self.sub is not None:
            self.pipeline.unsubscribe(self.sub)
        if self.asub is not None:
            self.audio.unsubscribe(self.asub)
        for t in self.tasks:
            t.cancel()
        if self.transport is not None:
            self.transport.close()
        if self.relay is not None:
            try:
                asyncio.get_running_loop().create_task(self.relay.aclose())
            except RuntimeError:
                self.relay.close()


class WhepEndpoint:
    """``POST /whep`` (application/sdp offer) -> 201 answer; ``DELETE /whep/{id}``."""

    def __init__(self, pipeline, host: str | None = None, udp_port: int = 0, level_idc: int = 0x2A, audio=None,
                 congestion_control: bool = False, on_input=None, turn: dict | None = None):
        self.pipeline = pipeline
        self.on_input = on_input
        self.turn = turn
        self.audio = audio
        self.congestion_control = congestion_control
        self.host = host
        self.udp_port = udp_port
        self.level_idc = level_idc
        self.peers: dict[str, WebRtcPeer] = {}
        self.last_peer: WebRtcPeer | None = None

    def routes(self, app) -> None:
        app.router.add_post("/whep", self.post)
        app.router.add_delete("/whep/{pid}", self.delete)
        app.router.add_patch("/whep/{pid}", self.patch)

    async def post(self, request):
        from aiohttp import web

        offer = await request.text()
        peer = WebRtcPeer(self.pipeline, offer, self.host, self.udp_port, self.level_idc, audio=self.audio,
                          congestion_control=self.congestion_control, on_input=self.on_input, turn=self.turn)
        try:
            answer = await peer.start()
        except ValueError as e:
            peer.close()
            raise web.HTTPBadRequest(text=str(e))
        self.peers[peer.id] = peer
        self.last_peer = peer
        return web.Response(status=201, text=answer, content_type="application/sdp",
                            headers={"Location": f"/whep/{peer.id}"})

    async def patch(self, request):
        """Trickle ICE (RFC 9725 §4.3): ``application/trickle-ice-sdpfrag`` with the browser's
        late candidates; they become TURN permissions on our relay."""
        from aiohttp import web

        peer = self.peers.get(request.match_info["pid"])
        if peer is None:
            raise web.HTTPNotFound()
        await peer.add_remote_candidates(await request.text())
        return web.Response(status=204)

    async def delete(self, request):
        from aiohttp import web

        peer = self.peers.pop(request.match_info["pid"], None)
        if peer is None:
            raise web.HTTPNotFound()
        peer.close()
        return web.Response(status=200)

    def close_all(self) -> None:
        for p in list(self.peers.values()):
            p.close()
        self.peers.clear()
