"""A small RFC 8656 TURN server over UDP for the TURN-client tests: long-term credentials
(401 with REALM/NONCE, MD5 key), Allocate / Refresh / CreatePermission / ChannelBind, Send
and Data indications, ChannelData, permission enforcement on both directions."""
import asyncio
import hashlib
import os
import struct

from mxdesk.server import stun as S
from mxdesk.server import turn_client as T


class MiniTurnServer:
    REALM = b"mxdesk.test"

    def __init__(self, users: dict[str, str]):
        self.users = users
        self.nonce = os.urandom(8).hex().encode()
        self.allocs = {}  # client addr -> Allocation
        self.transport = None
        self.log = []
        self.relayed_in = self.relayed_out = self.dropped = 0

    async def start(self, host="127.0.0.1"):
        loop = asyncio.get_running_loop()
        srv = self

        class P(asyncio.DatagramProtocol):
            def datagram_received(self, data, addr):
                srv._on_client(data, addr)

        self.transport, _ = await loop.create_datagram_endpoint(P, local_addr=(host, 0))
        return self.transport.get_extra_info("sockname")[1]

    def close(self):
        for a in self.allocs.values():
            a["relay"].close()
        self.transport.close()

    def _key(self, user):
        return hashlib.md5(user.encode() + b":" + self.REALM + b":" + self.users[user].encode()).digest()

    def _reply(self, addr, m, cls, attrs, key=None):
        r = S.StunMessage(T.method_of(m.type) | cls, m.tid, attrs)
        self.transport.sendto(r.encode(key, fingerprint=False), addr)

    def _err(self, addr, m, code, reason=b""):
        attrs = [(S.A_ERROR_CODE, struct.pack("!HBB", 0, code // 100, code % 100) + reason)]
        if code in (401, 438):
            attrs += [(T.A_REALM, self.REALM), (T.A_NONCE, self.nonce)]
        self._reply(addr, m, T.ERROR, attrs)

    def _on_client(self, data, addr):
        if 0x40 <= data[0] <= 0x7F:
            ch, n = struct.unpack_from("!HH", data)
            a = self.allocs.get(addr)
            peer = a and a["channels"].get(ch)
            if peer and peer[0] in a["perms"]:
                a["relay"].sendto(data[4:4 + n], peer)
                self.relayed_out += 1
            return
        m = S.StunMessage.decode(data)
        meth, cls = T.method_of(m.type), T.class_of(m.type)
        self.log.append((meth, cls))
        a = self.allocs.get(addr)
        if cls == T.INDICATION and meth == T.SEND:
            peer = S.parse_xor_address(m.get(T.A_XOR_PEER_ADDRESS), m.tid)
            if a and peer[0] in a["perms"]:
                a["relay"].sendto(m.get(T.A_DATA), peer)
                self.relayed_out += 1
            else:
                self.dropped += 1
            return
        user = (m.get(S.A_USERNAME) or b"").decode()
        if user not in self.users or m.get(S.A_MESSAGE_INTEGRITY) is None:
            return self._err(addr, m, 401)
        if m.get(T.A_NONCE) != self.nonce:
            return self._err(addr, m, 438)
        key = self._key(user)
        if not m.check_integrity(key):
            return self._err(addr, m, 401)
        if meth == T.ALLOCATE:
            if a is None:
                a = {"perms": set(), "channels": {}, "bychan": {}}
                loop = asyncio.get_running_loop()
                srv = self

                class R(asyncio.DatagramProtocol):
                    def datagram_received(self, d, peer, a=a, client=addr):
                        srv._on_peer(a, client, d, peer)

                fut = loop.create_datagram_endpoint(R, local_addr=("127.0.0.1", 0))
                task = asyncio.ensure_future(fut)

                def done(t, a=a, m=m, addr=addr, key=key):
                    a["relay"] = t.result()[0]
                    self.allocs[addr] = a
                    port = a["relay"].get_extra_info("sockname")[1]
                    self._reply(addr, m, T.SUCCESS, [(T.A_XOR_RELAYED_ADDRESS, S.xor_address("127.0.0.1", port, m.tid)),
                                                     (S.A_XOR_MAPPED_ADDRESS, S.xor_address(addr[0], addr[1], m.tid)),
                                                     (T.A_LIFETIME, struct.pack("!I", 600))], key)
                task.add_done_callback(done)
                return
            return self._err(addr, m, 437)
        if a is None:
            return self._err(addr, m, 437)
        if meth == T.REFRESH:
            self._reply(addr, m, T.SUCCESS, [(T.A_LIFETIME, m.get(T.A_LIFETIME) or struct.pack("!I", 600))], key)
        elif meth == T.CREATE_PERMISSION:
            for t, v in m.attrs:
                if t == T.A_XOR_PEER_ADDRESS:
                    a["perms"].add(S.parse_xor_address(v, m.tid)[0])
            self._reply(addr, m, T.SUCCESS, [], key)
        elif meth == T.CHANNEL_BIND:
            ch = struct.unpack("!H", m.get(T.A_CHANNEL_NUMBER)[:2])[0]
            peer = S.parse_xor_address(m.get(T.A_XOR_PEER_ADDRESS), m.tid)
            a["channels"][ch] = peer
            a["bychan"][peer] = ch
            a["perms"].add(peer[0])
            self._reply(addr, m, T.SUCCESS, [], key)
        else:
            self._err(addr, m, 400)

    def _on_peer(self, a, client, data, peer):
        if peer[0] not in a["perms"]:
            self.dropped += 1
            return
        self.relayed_in += 1
        ch = a["bychan"].get(peer)
        if ch is not None:
            self.transport.sendto(T.channel_data(ch, data), client)
        else:
            ind = S.StunMessage(T.DATA | T.INDICATION, None, [])
            ind.attrs = [(T.A_XOR_PEER_ADDRESS, S.xor_address(peer[0], peer[1], ind.tid)), (T.A_DATA, data)]
            self.transport.sendto(ind.encode(None, fingerprint=False), client)
