"""selkies-compatible WebSocket signalling with an in-process streaming peer.

Protocol (selkies-gstreamer ``webrtc_signalling.py`` [UP], derived from the GStreamer webrtc
"sendrecv" demo): a peer connects to ``/ws`` and sends ``HELLO <uid> [meta]``; the server
answers ``HELLO``.  ``SESSION <peer_uid>`` links two peers (``SESSION_OK`` /
``ERROR peer <uid> not found``); afterwards every message (JSON ``{"sdp": ...}`` /
``{"ice": ...}``) is relayed verbatim to the linked peer.  Disconnects notify the peer.

Upstream, the streaming application itself registers on the signalling server (uid 0), links
itself to the browser (uid 1) and sends the SDP offer (reference
selkies-gstreamer-entrypoint.sh:44-47 starts it).  Here that streaming peer lives in-process
(``attach_server``, mxdesk.server.selkies_peer): every browser that registers is offered a
stream by it, and browser -> server messages are handed to it with the sender's uid, so one
streaming peer serves several browsers.  Browser <-> browser sessions still relay as before.
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
        self.server = None  # in-process streaming peer (uid, on_join / on_message / on_leave)
        self.tasks: set[asyncio.Task] = set()

    def attach_server(self, server) -> None:
        self.server = server

    async def send_to(self, uid: str, text: str) -> bool:
        ws = self.peers.get(uid)
        if ws is None or ws.closed:
            return False
        await ws.send_str(text)
        return True

    def _spawn(self, coro) -> None:
        t = asyncio.ensure_future(coro)
        self.tasks.add(t)
        t.add_done_callback(self.tasks.discard)

    def _link_server(self, uid: str) -> None:
        self.sessions[uid] = self.server.uid
        self._spawn(self.server.on_join(uid))

    async def handler(self, request: web.Request) -> web.WebSocketResponse:
        ws = web.WebSocketResponse(heartbeat=10)
        await ws.prepare(request)
        uid = None
        srv = self.server
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
                        if uid in self.peers or (srv is not None and uid == srv.uid):
                            await ws.send_str(f"ERROR uid {uid} already in use")
                            uid = None
                            continue
                        self.peers[uid] = ws
                    await ws.send_str("HELLO")
                    if srv is not None:  # the streaming peer links itself and offers
                        self._link_server(uid)
                    continue
                if text.startswith("SESSION "):
                    other = text.split(" ", 1)[1].strip()
                    if srv is not None and other == srv.uid:
                        await ws.send_str("SESSION_OK")
                        if self.sessions.get(uid) != srv.uid:
                            self._link_server(uid)
                        continue
                    async with self.lock:
                        if other not in self.peers:
                            await ws.send_str(f"ERROR peer {other!r} not found")
                            continue
                        # both browsers leave the streaming peer they were linked to (otherwise
                        # the peer's socket, timers and pipeline consumer would be orphaned)
                        for u in (uid, other):
                            if srv is not None and self.sessions.get(u) == srv.uid:
                                srv.on_leave(u)
                            prev = self.sessions.get(u)
                            if prev is not None and prev not in (srv.uid if srv else None, uid, other):
                                self.sessions.pop(prev, None)  # a third browser loses its link
                        self.sessions[uid] = other
                        self.sessions[other] = uid
                    await ws.send_str("SESSION_OK")
                    continue
                other = self.sessions.get(uid)
                if srv is not None and other == srv.uid:
                    try:
                        await srv.on_message(uid, text)
                    except Exception as e:  # bad SDP / ICE from this browser: tell it, keep the socket
                        log.warning("streaming peer rejected a message from %s: %s", uid, e)
                        await ws.send_str(f"ERROR {e}")
                    continue
                if other is None or other not in self.peers:
                    await ws.send_str("ERROR no session")
                    continue
                await self.peers[other].send_str(text)
        finally:
            if uid is not None:
                async with self.lock:
                    self.peers.pop(uid, None)
                    other = self.sessions.pop(uid, None)
                    if srv is not None and other == srv.uid:
                        srv.on_leave(uid)
                    elif other is not None and self.sessions.get(other) == uid:
                        self.sessions.pop(other, None)
                        peer = self.peers.get(other)
                        if peer is not None and not peer.closed:
                            await peer.send_str(f"ERROR peer {uid} disconnected")
        return ws
