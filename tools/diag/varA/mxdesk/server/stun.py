"""STUN (RFC 5389) messages for ICE-lite connectivity checks (RFC 8445 §2.5)."""
from __future__ import annotations

import hashlib
import hmac
import ipaddress
import os
import struct
import zlib

MAGIC = 0x2112A442
BINDING_REQUEST = 0x0001
BINDING_SUCCESS = 0x0101
BINDING_ERROR = 0x0111
A_USERNAME = 0x0006
A_MESSAGE_INTEGRITY = 0x0008
A_ERROR_CODE = 0x0009
A_XOR_MAPPED_ADDRESS = 0x0020
A_PRIORITY = 0x0024
A_USE_CANDIDATE = 0x0025
A_FINGERPRINT = 0x8028
A_ICE_CONTROLLED = 0x8029
A_ICE_CONTROLLING = 0x802A
FINGERPRINT_XOR = 0x5354554E


def is_stun(data: bytes) -> bool:
    return len(data) >= 20 and data[0] < 4 and struct.unpack_from("!I", data, 4)[0] == MAGIC


class StunMessage:
    def __init__(self, mtype: int, tid: bytes | None = None, attrs: list[tuple[int, bytes]] | None = None):
        self.type = mtype
        self.tid = tid or os.urandom(12)
        self.attrs = attrs or []

    def get(self, t: int) -> bytes | None:
        for a, v in self.attrs:
            if a == t:
                return v
        return None

    @staticmethod
    def _attr(t: int, v: bytes) -> bytes:
        return struct.pack("!HH", t, len(v)) + v + b"\x00" * ((4 - len(v) % 4) % 4)

    def encode(self, integrity_key: bytes | None = None, fingerprint: bool = True) -> bytes:
        body = b"".join(self._attr(t, v) for t, v in self.attrs)
        if integrity_key is not None:
            hdr = struct.pack("!HHI", self.type, len(body) + 24, MAGIC) + self.tid
            mac = hmac.new(integrity_key, hdr + body, hashlib.sha1).digest()
            body += self._attr(A_MESSAGE_INTEGRITY, mac)
        if fingerprint:
            hdr = struct.pack("!HHI", self.type, len(body) + 8, MAGIC) + self.tid
            crc = (zlib.crc32(hdr + body) & 0xFFFFFFFF) ^ FINGERPRINT_XOR
            body += self._attr(A_FINGERPRINT, struct.pack("!I", crc))
        return struct.pack("!HHI", self.type, len(body), MAGIC) + self.tid + body

    @classmethod
    def decode(cls, data: bytes) -> "StunMessage":
        mtype, ln, magic = struct.unpack_from("!HHI", data)
        if magic != MAGIC or 20 + ln > len(data):
            raise ValueError("not a STUN message")
        m = cls(mtype, data[8:20])
        off = 20
        while off + 4 <= 20 + ln:
            t, n = struct.unpack_from("!HH", data, off)
            m.attrs.append((t, data[off + 4: off + 4 + n]))
            off += 4 + n + ((4 - n % 4) % 4)
        m.raw = data[: 20 + ln]
        return m

    def check_integrity(self, key: bytes) -> bool:
        """Verify MESSAGE-INTEGRITY (and FINGERPRINT if present) of a decoded message."""
        raw = self.raw
        off = 20
        mi_off = None
        while off + 4 <= len(raw):
            t, n = struct.unpack_from("!HH", raw, off)
            if t == A_MESSAGE_INTEGRITY:
                mi_off = off
                break
            off += 4 + n + ((4 - n % 4) % 4)
        if mi_off is None:
            return False
        hdr = struct.pack("!HHI", self.type, mi_off - 20 + 24, MAGIC) + self.tid
        mac = hmac.new(key, hdr + raw[20:mi_off], hashlib.sha1).digest()
        if not hmac.compare_digest(mac, raw[mi_off + 4: mi_off + 24]):
            return False
        fp = self.get(A_FINGERPRINT)
        if fp is not None:
            fp_off = len(raw) - 8
            hdr = struct.pack("!HHI", self.type, fp_off - 20 + 8, MAGIC) + self.tid
            if (zlib.crc32(hdr + raw[20:fp_off]) & 0xFFFFFFFF) ^ FINGERPRINT_XOR != struct.unpack("!I", fp)[0]:
                return False
        return True


def xor_address(host: str, port: int, tid: bytes) -> bytes:
    ip = ipaddress.ip_address(host)
    xport = port ^ (MAGIC >> 16)
    if ip.version == 4:
        xaddr = int(ip) ^ MAGIC
        return struct.pack("!BBHI", 0, 1, xport, xaddr)
    key = struct.pack("!I", MAGIC) + tid
    xaddr = bytes(a ^ b for a, b in zip(ip.packed, key))
    return struct.pack("!BBH", 0, 2, xport) + xaddr


def parse_xor_address(v: bytes, tid: bytes) -> tuple[str, int]:
    fam, xport = v[1], struct.unpack_from("!H", v, 2)[0]
    port = xport ^ (MAGIC >> 16)
    if fam == 1:
        return str(ipaddress.IPv4Address(struct.unpack_from("!I", v, 4)[0] ^ MAGIC)), port
    key = struct.pack("!I", MAGIC) + tid
    return str(ipaddress.IPv6Address(bytes(a ^ b for a, b in zip(v[4:20], key)))), port
