"""selkies-compatible WebSocket signalling relay.

Protocol (selkies-gstreamer ``webrtc_signalling.py`` [UP], derived from the GStreamer
webrtc "sendrecv" demo): a peer connects to ``/ws`` and sends ``HELLO <uid> [meta]``; the
server answers ``HELLO``.  ``SESSION <peer_uid>`` links two peers (``SESSION_OK`` /
``ERROR peer <uid> not found``); afterwards every message (JSON ``{"sdp": ...}`` /
``{"ice": ...}``) is relayed verbatim to the linked peer.  Disconnects notify the peer.
"""
from __future__ import annotations

import asyncio
import logging

from aiohttp import WSMsgType, web

log = logging.getLogger("mxdesk.signalling")


class SignallingRelay:
    def __init__(self):
        self.peers: dict[str, web.WebSocketResponse] = {}
        self.sessions: dict[str, str] = {}
        self.lock = asyncio.Lock()

    async def handler(self, request: web.Request) -> web.WebSocketResponse:
        ws = web.WebSocketResponse(heartbeat=10)
        await ws.prepare(request)
        uid = None
        try:
            async for msg in ws:
                if msg.type != WSMsgType.TEXT:
                    continue
                text = msg.data
                if uid is None:
                    parts = text.split(" ", 2)
                    if len(parts) < 2 or parts[0] != "HELLO":
                        await ws.send_str("ERROR invalid protocol: expected HELLO")
                        continue
                    uid = parts[1]
                    async with self.lock:
                        if uid in self.peers:
                            await ws.send_str(f"ERROR uid {uid} already in use")
                            uid = None
                            continue
                        self.peers[uid] = ws
                    await ws.send_str("HELLO")
                    continue
                if text.startswith("SESSION "):
                    other = text.split(" ", 1)[1].strip()
                    async with self.lock:
                        if other not in self.peers:
                            await ws.send_str(f"ERROR peer {other!r} not found")
                            continue
                        self.sessions[uid] = other
                        self.sessions[other] = uid
                    await ws.send_str("SESSION_OK")
                    continue
                other = self.sessions.get(uid)
                if other is None or other not in self.peers:
                    await ws.send_str("ERROR no session")
                    continue
                await self.peers[other].send_str(text)
        finally:
            if uid is not None:
                async with self.lock:
                    self.peers.pop(uid, None)
                    other = self.sessions.pop(uid, None)
                    if other is not None:
                        self.sessions.pop(other, None)
                        peer = self.peers.get(other)
                        if peer is not None and not peer.closed:
                            await peer.send_str(f"ERROR peer {uid} disconnected")
        return ws
