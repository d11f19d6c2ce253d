"""Server-side TURN client (RFC 8656): the server allocates its own relay so browsers reach it
through a TURN server even when the desktop pod is not directly reachable -- what the
reference's webrtcbin does with the ``TURN_*`` settings (README.md:65-143, xgl.yml:85-109).

* Allocate with long-term credentials (401 -> REALM/NONCE -> MESSAGE-INTEGRITY keyed by
  MD5(user:realm:pass); 438 stale nonce retried), REQUESTED-TRANSPORT UDP.
* CreatePermission for the browser's candidate addresses (from the offer / trickle PATCH),
  ChannelBind for the nominated peer (4-byte ChannelData framing instead of 36-byte
  Send/Data indications), periodic Refresh of allocation, permissions and channels.
* Transports to the TURN server: UDP, TCP (RFC 8656 §5 framing, ChannelData padded to 4),
  TLS over TCP (``TURN_TLS``).

Relayed payloads are handed to ``on_data(payload, (peer_ip, peer_port))``; ``send`` relays
one datagram to a peer.
"""
from __future__ import annotations

import asyncio
import hashlib
import logging
import ssl
import struct
import time
from typing import Callable

from . import stun as S

log = logging.getLogger("mxdesk.turn")

ALLOCATE, REFRESH, SEND, DATA, CREATE_PERMISSION, CHANNEL_BIND = 0x003, 0x004, 0x006, 0x007, 0x008, 0x009
REQUEST, INDICATION, SUCCESS, ERROR = 0x000, 0x010, 0x100, 0x110
A_CHANNEL_NUMBER, A_LIFETIME, A_XOR_PEER_ADDRESS, A_DATA = 0x000C, 0x000D, 0x0012, 0x0013
A_REALM, A_NONCE, A_XOR_RELAYED_ADDRESS, A_REQUESTED_TRANSPORT, A_SOFTWARE = 0x0014, 0x0015, 0x0016, 0x0019, 0x8022


def method_of(mtype: int) -> int:
    return mtype & 0x3EEF


def class_of(mtype: int) -> int:
    return mtype & 0x0110


def error_code(m: S.StunMessage) -> int:
    v = m.get(S.A_ERROR_CODE)
    return (v[2] & 7) * 100 + v[3] if v and len(v) >= 4 else 0


def channel_data(channel: int, data: bytes, pad: bool = False) -> bytes:
    out = struct.pack("!HH", channel, len(data)) + data
    return out + b"\0" * ((4 - len(data) % 4) % 4) if pad else out


class TurnError(RuntimeError):
    pass


class TurnClient:
    CHANNEL_BASE = 0x4000

    def __init__(self, host: str, port: int, username: str, password: str, protocol: str = "udp",
                 tls: bool = False, on_data: Callable[[bytes, tuple[str, int]], None] | None = None,
                 ssl_context: ssl.SSLContext | None = None, lifetime: int = 600):
        self.server = (host, int(port))
        self.username, self.password = username, password
        self.protocol = "tcp" if tls else protocol.lower()
        self.tls = tls
        self.ssl_context = ssl_context
        self.on_data = on_data
        self.lifetime = lifetime
        self.realm: bytes | None = None
        self.nonce: bytes | None = None
        self.key: bytes | None = None
        self.relayed: tuple[str, int] | None = None
        self.mapped: tuple[str, int] | None = None
        self.permissions: dict[str, float] = {}
        self.channels: dict[tuple[str, int], int] = {}
        self._peers_by_channel: dict[int, tuple[str, int]] = {}
        self._pending: dict[bytes, asyncio.Future] = {}
        self._transport = None
        self._writer: asyncio.StreamWriter | None = None
        self._tasks: list[asyncio.Task] = []
        self.closed = False
        self.stats = {"sent": 0, "received": 0, "channel_sent": 0, "channel_received": 0}

    # ------------------------------------------------------------------ transport
    async def connect(self) -> None:
        loop = asyncio.get_running_loop()
        if self.protocol == "udp":
            client = self

            class _Proto(asyncio.DatagramProtocol):
                def datagram_received(self, data, addr):
                    client._on_packet(data)

            self._transport, _ = await loop.create_datagram_endpoint(_Proto, remote_addr=self.server)
        else:
            ctx = None
            if self.tls:
                ctx = self.ssl_context or ssl.create_default_context()
            reader, self._writer = await asyncio.open_connection(*self.server, ssl=ctx)
            self._tasks.append(asyncio.create_task(self._tcp_reader(reader)))

    async def _tcp_reader(self, reader: asyncio.StreamReader) -> None:
        try:
            while True:
                hdr = await reader.readexactly(4)
                if 0x40 <= hdr[0] <= 0x7F:  # ChannelData, padded to 4 over stream transports
                    n = struct.unpack_from("!H", hdr, 2)[0]
                    body = await reader.readexactly(n + (4 - n % 4) % 4)
                    self._on_packet(hdr + body[:n])
                else:
                    n = struct.unpack_from("!H", hdr, 2)[0]
                    self._on_packet(hdr + await reader.readexactly(16 + n))
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError):
            pass

    def _write(self, data: bytes) -> None:
        if self.closed:
            return
        if self._transport is not None:
            self._transport.sendto(data)
        elif self._writer is not None:
            self._writer.write(data)

    # ------------------------------------------------------------------ incoming
    def _on_packet(self, data: bytes) -> None:
        if len(data) >= 4 and 0x40 <= data[0] <= 0x7F:
            ch, n = struct.unpack_from("!HH", data)
            peer = self._peers_by_channel.get(ch)
            if peer is not None and self.on_data is not None:
                self.stats["channel_received"] += 1
                self.on_data(data[4:4 + n], peer)
            return
        if not S.is_stun(data):
            return
        try:
            m = S.StunMessage.decode(data)
        except ValueError:
            return
        if class_of(m.type) == INDICATION and method_of(m.type) == DATA:
            pa, payload = m.get(A_XOR_PEER_ADDRESS), m.get(A_DATA)
            if pa is not None and payload is not None and self.on_data is not None:
                self.stats["received"] += 1
                self.on_data(payload, S.parse_xor_address(pa, m.tid))
            return
        fut = self._pending.pop(m.tid, None)
        if fut is not None and not fut.done():
            fut.set_result(m)

    # ------------------------------------------------------------------ requests
    def _auth_attrs(self) -> list[tuple[int, bytes]]:
        if self.realm is None:
            return []
        return [(S.A_USERNAME, self.username.encode()), (A_REALM, self.realm), (A_NONCE, self.nonce)]

    async def _request(self, method: int, attrs, timeout: float = 5.0) -> S.StunMessage:
        """``attrs``: attribute list, or a function of the transaction id returning one (XOR
        addresses of IPv6 peers depend on it)."""
        for _attempt in range(3):
            m = S.StunMessage(method | REQUEST, None, [])
            m.attrs = (attrs(m.tid) if callable(attrs) else list(attrs)) + self._auth_attrs()
            fut = asyncio.get_running_loop().create_future()
            self._pending[m.tid] = fut
            raw = m.encode(self.key if self.realm is not None else None, fingerprint=False)
            deadline = time.monotonic() + timeout
            rto = 0.25
            resp = None
            while resp is None:  # retransmit over UDP (RFC 8489 §6.2.1); once over TCP
                self._write(raw)
                try:
                    resp = await asyncio.wait_for(asyncio.shield(fut), min(rto, max(0.01, deadline - time.monotonic()))
                                                  if self.protocol == "udp" else timeout)
                except asyncio.TimeoutError:
                    if time.monotonic() >= deadline:
                        self._pending.pop(m.tid, None)
                        raise TurnError(f"TURN {method:#x}: no response from {self.server}")
                    rto = min(rto * 2, 2.0)
            if class_of(resp.type) == SUCCESS:
                if self.key is not None and resp.get(S.A_MESSAGE_INTEGRITY) is not None \
                        and not resp.check_integrity(self.key):
                    raise TurnError(f"TURN {method:#x}: bad MESSAGE-INTEGRITY in the response")
                return resp
            code = error_code(resp)
            if code in (401, 438) and resp.get(A_NONCE) is not None:
                first = self.realm is None
                self.nonce = resp.get(A_NONCE)
                if resp.get(A_REALM) is not None:
                    self.realm = resp.get(A_REALM)
                self.key = hashlib.md5(self.username.encode() + b":" + self.realm + b":" +
                                       self.password.encode()).digest()
                if code == 438 or first:
                    continue
            raise TurnError(f"TURN {method:#x} failed: {code} "
                            f"{(resp.get(S.A_ERROR_CODE) or b'')[4:].decode(errors='replace')}")
        raise TurnError(f"TURN {method:#x}: authentication failed")

    async def allocate(self) -> tuple[str, int]:
        if self._transport is None and self._writer is None:
            await self.connect()
        r = await self._request(ALLOCATE, [(A_REQUESTED_TRANSPORT, bytes([17, 0, 0, 0])),
                                           (A_LIFETIME, struct.pack("!I", self.lifetime)),
                                           (A_SOFTWARE, b"mxdesk")])
        self.relayed = S.parse_xor_address(r.get(A_XOR_RELAYED_ADDRESS), r.tid)
        xm = r.get(S.A_XOR_MAPPED_ADDRESS)
        self.mapped = S.parse_xor_address(xm, r.tid) if xm else None
        lt = r.get(A_LIFETIME)
        if lt:
            self.lifetime = struct.unpack("!I", lt)[0]
        self._tasks.append(asyncio.create_task(self._refresher()))
        log.info("TURN relay %s:%d via %s:%d/%s", *self.relayed, *self.server, self.protocol)
        return self.relayed

    async def create_permission(self, ips) -> None:
        ips = sorted({ip for ip in ips if ip})
        if not ips:
            return
        await self._request(CREATE_PERMISSION, lambda tid: [(A_XOR_PEER_ADDRESS, S.xor_address(ip, 0, tid))
                                                            for ip in ips])
        now = time.monotonic()
        for ip in ips:
            self.permissions[ip] = now

    async def channel_bind(self, peer: tuple[str, int]) -> int:
        peer = (peer[0], int(peer[1]))
        ch = self.channels.get(peer)
        if ch is None:
            ch = self.CHANNEL_BASE + len(self.channels)
        await self._request(CHANNEL_BIND, lambda tid: [(A_CHANNEL_NUMBER, struct.pack("!HH", ch, 0)),
                                                       (A_XOR_PEER_ADDRESS, S.xor_address(peer[0], peer[1], tid))])
        self.channels[peer] = ch
        self._peers_by_channel[ch] = peer
        self.permissions[peer[0]] = time.monotonic()
        return ch

    def send(self, data: bytes, peer: tuple[str, int]) -> None:
        peer = (peer[0], int(peer[1]))
        ch = self.channels.get(peer)
        if ch is not None:
            self.stats["channel_sent"] += 1
            self._write(channel_data(ch, data, pad=self.protocol != "udp"))
            return
        self.stats["sent"] += 1
        m = S.StunMessage(SEND | INDICATION, None, [])
        m.attrs = [(A_XOR_PEER_ADDRESS, S.xor_address(peer[0], peer[1], m.tid)), (A_DATA, data)]
        self._write(m.encode(None, fingerprint=False))

    # ------------------------------------------------------------------ lifetime
    async def _refresher(self) -> None:
        try:
            while not self.closed:
                await asyncio.sleep(min(240.0, max(1.0, self.lifetime / 2)))
                await self._request(REFRESH, [(A_LIFETIME, struct.pack("!I", self.lifetime))])
                if self.permissions:  # permissions last 300 s (RFC 8656 §9)
                    await self.create_permission(list(self.permissions))
                for peer in list(self.channels):  # channel bindings last 600 s
                    await self.channel_bind(peer)
        except asyncio.CancelledError:
            pass
        except TurnError as e:
            log.warning("TURN refresh failed: %s", e)

    async def aclose(self) -> None:
        if self.closed:
            return
        try:
            if self.relayed is not None:
                await self._request(REFRESH, [(A_LIFETIME, struct.pack("!I", 0))], timeout=1.0)
        except (TurnError, OSError):
            pass
        self.close()

    def close(self) -> None:
        self.closed = True
        for t in self._tasks:
            t.cancel()
        if self._transport is not None:
            self._transport.close()
        if self._writer is not None:
            self._writer.close()
        for f in self._pending.values():
            if not f.done():
                f.cancel()


def offer_candidate_ips(sdp: str) -> list[str]:
    """Peer IPs of the browser's ICE candidates in an offer or trickle fragment (mDNS
    ``.local`` names are skipped: a TURN permission needs an IP)."""
    out = []
    for line in sdp.replace("\r\n", "\n").split("\n"):
        line = line.strip()
        if line.startswith("a=candidate:"):
            parts = line[len("a=candidate:"):].split()
            if len(parts) >= 6 and parts[2].lower() == "udp" and not parts[4].endswith(".local"):
                out.append(parts[4])
    return out
