"""The streaming side of the selkies WebRTC protocol.

Upstream (reference selkies-gstreamer-entrypoint.sh:44-47, web app installed at
Dockerfile:472), the selkies streaming application registers on the signalling server as
uid 0, links itself to the browser, creates the offer with webrtcbin and opens the ``input``
data channel from the server side.  A stock selkies web client therefore only registers
(``HELLO 1 <meta>``) and waits for an offer.  ``SelkiesServerPeer`` plays that role on
mxdesk's own ``/ws`` relay: for every browser that registers it

  * creates a ``WebRtcPeer`` in offer mode (ICE-lite, DTLS-SRTP, SCTP data channels -- the
    same transport as the WHEP endpoint) and sends ``{"sdp": {"type": "offer", "sdp": ...}}``;
  * takes ``{"sdp": {"type": "answer", ...}}`` and trickled ``{"ice": {...}}`` messages;
  * opens the ``input`` data channel, whose messages (selkies input protocol: ``m,x,y,...``,
    ``kd,keysym``, ``cw,<b64>``, ``vb,kbps``, ...) go to the MediaServer's input handler.
"""
from __future__ import annotations

import json
import logging

log = logging.getLogger("mxdesk.selkies")


class SelkiesServerPeer:
    def __init__(self, relay, make_peer, uid: str = "0"):
        """``make_peer()`` -> a new WebRtcPeer(pipeline, None, ..., server_channels=("input",))."""
        self.relay = relay
        self.make_peer = make_peer
        self.uid = uid
        self.sessions: dict[str, object] = {}

    async def on_join(self, client: str) -> None:
        old = self.sessions.pop(client, None)
        if old is not None:
            old.close()
        peer = self.make_peer()
        self.sessions[client] = peer
        try:
            offer = await peer.start_offer()
        except Exception:
            log.exception("selkies peer for %s: offer failed", client)
            self.sessions.pop(client, None)
            peer.close()
            return
        log.info("selkies: offering a stream to %s (peer %s)", client, peer.id)
        await self.relay.send_to(client, json.dumps({"sdp": {"type": "offer", "sdp": offer}}))

    async def on_message(self, client: str, text: str) -> None:
        peer = self.sessions.get(client)
        if peer is None:
            return
        msg = json.loads(text)
        if "sdp" in msg:
            sdp = msg["sdp"] or {}
            if sdp.get("type") != "answer":
                raise ValueError(f"expected an SDP answer, got {sdp.get('type')!r}")
            await peer.accept_answer(sdp.get("sdp", ""))
        elif "ice" in msg:
            cand = (msg["ice"] or {}).get("candidate") or ""
            if cand:
                await peer.add_remote_candidates("a=" + cand if not cand.startswith("a=") else cand)

    def on_leave(self, client: str) -> None:
        peer = self.sessions.pop(client, None)
        if peer is not None:
            log.info("selkies: %s left, closing peer %s", client, peer.id)
            peer.close()

    def close_all(self) -> None:
        for c in list(self.sessions):
            self.on_leave(c)
