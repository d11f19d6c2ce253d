"""Headless selkies web-client stand-in: speaks the selkies signalling protocol on ``/ws``
(``HELLO 1 <meta>`` -> waits for the server's offer -> answers) and then plays the browser's
media role (full ICE agent, DTLS client, SRTP receiver with NACK / PLI, SCTP with the
server-opened ``input`` channel) through the same session code as the WHEP viewer.  Used by
the loopback tests and as a CLI smoke check: ``python -m mxdesk.server.selkies_client ws://host:8080/ws``.

Reference: the selkies-gstreamer web app (installed at reference Dockerfile:472) against the
streaming app started by selkies-gstreamer-entrypoint.sh:44-47.
"""
from __future__ import annotations

import asyncio
import base64
import json
import secrets
import time

from .webrtc import parse_sdp
from .whep_client import WhepResult, _native, media_session


def make_answer(offer_sdp: str, ufrag: str, pwd: str, fingerprint: str) -> str:
    """A browser-style answer: accept the H.264 / H.265 video section (recvonly), a PCMU audio
    section and the SCTP data-channel section, BUNDLEd, DTLS ``active`` (we are the client)."""
    off = parse_sdp(offer_sdp)
    mids, media = [], []
    for md in off.media:
        mid = md.attr("mid") or str(len(mids))
        common = ["c=IN IP4 0.0.0.0", f"a=ice-ufrag:{ufrag}", f"a=ice-pwd:{pwd}", f"a=fingerprint:{fingerprint}",
                  "a=setup:active", f"a=mid:{mid}"]
        if md.kind == "video":
            pt = md.fmts[0]
            rtpmap = next((r for r in md.attrs_named("rtpmap") if r.split()[0] == pt), f"{pt} H264/90000")
            fmtp = next((f for f in md.attrs_named("fmtp") if f.split()[0] == pt), None)
            media += [f"m=video 9 UDP/TLS/RTP/SAVPF {pt}", *common, "a=recvonly", "a=rtcp-mux", "a=rtcp-rsize",
                      f"a=rtpmap:{rtpmap}", f"a=rtcp-fb:{pt} nack", f"a=rtcp-fb:{pt} nack pli"]
            if fmtp:
                media.append(f"a=fmtp:{fmtp}")
        elif md.kind == "audio":
            media += ["m=audio 9 UDP/TLS/RTP/SAVPF 0", *common, "a=recvonly", "a=rtcp-mux", "a=rtpmap:0 PCMU/8000"]
        elif md.kind == "application":
            media += ["m=application 9 UDP/DTLS/SCTP webrtc-datachannel", *common, "a=sctp-port:5000",
                      "a=max-message-size:262144"]
        else:
            media += [f"m={md.kind} 0 {md.proto} {md.fmts[0] if md.fmts else '0'}", f"a=mid:{mid}"]
            continue
        mids.append(mid)
    lines = ["v=0", f"o=- {secrets.randbelow(1 << 62)} 2 IN IP4 127.0.0.1", "s=-", "t=0 0",
             "a=group:BUNDLE " + " ".join(mids), "a=msid-semantic: WMS"]
    return "\r\n".join(lines + media) + "\r\n"


async def selkies_view(ws_url: str, n_frames: int, uid: str = "1", dc_messages: list[str] | None = None,
                       timeout: float = 30.0, auth=None, pli_after: int = 0) -> WhepResult:
    """Register as ``uid``, take the server's offer, answer, receive ``n_frames`` access units;
    ``dc_messages`` are sent on the server-opened ``input`` channel."""
    import aiohttp

    N = _native()
    dtls = N.net.DtlsEndpoint(False)
    ufrag, pwd = secrets.token_hex(4), secrets.token_hex(12)
    res = WhepResult()
    t0 = time.monotonic()
    headers = {"Authorization": auth.encode()} if auth else None
    async with aiohttp.ClientSession(headers=headers) as s:
        async with s.ws_connect(ws_url) as ws:
            meta = base64.b64encode(json.dumps({"res": "1920x1080", "scale": 1}).encode()).decode()
            await ws.send_str(f"HELLO {uid} {meta}")
            offer = None
            deadline = time.monotonic() + timeout
            while offer is None:
                msg = await asyncio.wait_for(ws.receive(), max(0.1, deadline - time.monotonic()))
                if msg.type != aiohttp.WSMsgType.TEXT:
                    raise RuntimeError(f"signalling closed: {msg.type}")
                if msg.data == "HELLO" or msg.data.startswith("SESSION_OK"):
                    continue
                if msg.data.startswith("ERROR"):
                    raise RuntimeError(msg.data)
                data = json.loads(msg.data)
                if "sdp" in data and data["sdp"].get("type") == "offer":
                    offer = data["sdp"]["sdp"]
            answer = make_answer(offer, ufrag, pwd, dtls.fingerprint)
            await ws.send_str(json.dumps({"sdp": {"type": "answer", "sdp": answer}}))
            await ws.send_str(json.dumps({"ice": {"candidate": "candidate:1 1 udp 2122260223 127.0.0.1 9 typ host",
                                                  "sdpMLineIndex": 0}}))
            res.answer = offer  # the remote description (here: the server's offer)
            await media_session(res, offer, dtls, ufrag, N, n_frames, t0, timeout=timeout, pli_after=pli_after,
                                dc_messages=dc_messages, server_channel="input" if dc_messages is not None else None)
    return res


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(description="headless selkies signalling client")
    ap.add_argument("url", help="ws://host:port/ws")
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--uid", default="1")
    a = ap.parse_args(argv)
    r = asyncio.run(selkies_view(a.url, a.frames, a.uid))
    print(f"frames={len(r.aus)} packets={r.packets} bytes={len(r.stream)} connect_ms={r.connect_ms:.1f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
