"""RTP/RTCP helpers in Python: H.264 / H.265 / VP8 depacketizers (RFC 6184 / 7798 / 7741) for test peers and RTCP
packet builders/parsers (RFC 3550 SR/RR/SDES, RFC 4585 generic NACK + PLI, RFC 5104 FIR,
REMB receiver bandwidth estimates)."""
from __future__ import annotations

import struct
import time

NTP_EPOCH_OFFSET = 2208988800


def rtp_header(pkt: bytes) -> dict:
    b0, b1, seq, ts, ssrc = struct.unpack_from("!BBHII", pkt)
    cc = b0 & 0x0F
    off = 12 + 4 * cc
    if b0 & 0x10:
        _, ln = struct.unpack_from("!HH", pkt, off)
        off += 4 + 4 * ln
    return {"version": b0 >> 6, "marker": bool(b1 & 0x80), "pt": b1 & 0x7F, "seq": seq, "ts": ts, "ssrc": ssrc,
            "payload": pkt[off:]}


class H264Depacketizer:
    """Reassembles Annex-B access units from RTP packets (single NAL, STAP-A, FU-A)."""

    def __init__(self):
        self.nals: list[bytes] = []
        self.fu: bytearray | None = None
        self.last_seq: int | None = None
        self.lost = 0

    def push(self, pkt: bytes) -> bytes | None:
        h = rtp_header(pkt)
        if self.last_seq is not None and ((h["seq"] - self.last_seq) & 0xFFFF) != 1:
            self.lost += 1
        self.last_seq = h["seq"]
        p = h["payload"]
        t = p[0] & 0x1F
        if 1 <= t <= 23:
            self.nals.append(p)
        elif t == 24:  # STAP-A
            off = 1
            while off + 2 <= len(p):
                n = struct.unpack_from("!H", p, off)[0]
                self.nals.append(p[off + 2: off + 2 + n])
                off += 2 + n
        elif t == 28:  # FU-A
            fu = p[1]
            if fu & 0x80:
                self.fu = bytearray([(p[0] & 0xE0) | (fu & 0x1F)])
            if self.fu is not None:
                self.fu += p[2:]
                if fu & 0x40:
                    self.nals.append(bytes(self.fu))
                    self.fu = None
        if h["marker"]:
            au = b"".join(b"\x00\x00\x00\x01" + n for n in self.nals)
            self.nals = []
            return au
        return None


class H265Depacketizer:
    """Reassembles Annex-B access units from RFC 7798 packets (single NAL, AP, FU; no DONL)."""

    def __init__(self):
        self.nals: list[bytes] = []
        self.fu: bytearray | None = None
        self.last_seq: int | None = None
        self.lost = 0

    def push(self, pkt: bytes) -> bytes | None:
        h = rtp_header(pkt)
        if self.last_seq is not None and ((h["seq"] - self.last_seq) & 0xFFFF) != 1:
            self.lost += 1
        self.last_seq = h["seq"]
        p = h["payload"]
        t = (p[0] >> 1) & 0x3F
        if t < 48:
            self.nals.append(p)
        elif t == 48:  # aggregation packet
            off = 2
            while off + 2 <= len(p):
                n = struct.unpack_from("!H", p, off)[0]
                self.nals.append(p[off + 2: off + 2 + n])
                off += 2 + n
        elif t == 49:  # fragmentation unit
            fu = p[2]
            if fu & 0x80:
                self.fu = bytearray([(p[0] & 0x81) | ((fu & 0x3F) << 1), p[1]])
            if self.fu is not None:
                self.fu += p[3:]
                if fu & 0x40:
                    self.nals.append(bytes(self.fu))
                    self.fu = None
        if h["marker"]:
            au = b"".join(b"\x00\x00\x00\x01" + n for n in self.nals)
            self.nals = []
            return au
        return None


class Vp8Depacketizer:
    """Reassembles VP8 frames from RFC 7741 packets: parses the payload descriptor (X, N, S, PID
    and the optional PictureID / TL0PICIDX / TID / KEYIDX extensions), starts a frame at S = 1 with
    PID 0, ends it at the marker bit.  A frame with a lost packet is dropped."""

    def __init__(self):
        self.buf: bytearray | None = None
        self.last_seq: int | None = None
        self.lost = 0
        self.picture_ids: list[int] = []

    @staticmethod
    def descriptor(p: bytes) -> tuple[int, dict]:
        b0 = p[0]
        d = {"N": bool(b0 & 0x20), "S": bool(b0 & 0x10), "PID": b0 & 0x07, "picture_id": None}
        off = 1
        if b0 & 0x80:  # X
            x = p[off]
            off += 1
            if x & 0x80:  # I
                if p[off] & 0x80:  # M: 15-bit picture id
                    d["picture_id"] = ((p[off] & 0x7F) << 8) | p[off + 1]
                    off += 2
                else:
                    d["picture_id"] = p[off] & 0x7F
                    off += 1
            if x & 0x40:  # L: TL0PICIDX
                off += 1
            if x & 0x30:  # T or K: TID|Y|KEYIDX byte
                off += 1
        return off, d

    def push(self, pkt: bytes) -> bytes | None:
        h = rtp_header(pkt)
        gap = self.last_seq is not None and ((h["seq"] - self.last_seq) & 0xFFFF) != 1
        if gap:
            self.lost += 1
            self.buf = None
        self.last_seq = h["seq"]
        off, d = self.descriptor(h["payload"])
        if d["S"] and d["PID"] == 0:
            self.buf = bytearray()
            self.picture_ids.append(d["picture_id"])
        if self.buf is not None:
            self.buf += h["payload"][off:]
        if h["marker"] and self.buf is not None:
            frame, self.buf = bytes(self.buf), None
            return frame
        return None


def ntp_now() -> tuple[int, int]:
    t = time.time() + NTP_EPOCH_OFFSET
    sec = int(t)
    return sec, int((t - sec) * (1 << 32)) & 0xFFFFFFFF


def build_sr(ssrc: int, rtp_ts: int, packets: int, octets: int, cname: str = "mxdesk") -> bytes:
    sec, frac = ntp_now()
    sr = struct.pack("!BBHIIIIII", 0x80, 200, 6, ssrc, sec, frac, rtp_ts & 0xFFFFFFFF, packets & 0xFFFFFFFF,
                     octets & 0xFFFFFFFF)
    c = cname.encode()
    item = bytes([1, len(c)]) + c + b"\x00"
    item += b"\x00" * ((4 - (4 + len(item)) % 4) % 4)
    sdes = struct.pack("!BBHI", 0x81, 202, (4 + len(item)) // 4, ssrc) + item
    return sr + sdes


def build_pli(sender_ssrc: int, media_ssrc: int) -> bytes:
    return struct.pack("!BBHII", 0x81, 206, 2, sender_ssrc, media_ssrc)


def build_rr(sender_ssrc: int, media_ssrc: int, fraction_lost: float, cum_lost: int = 0, ext_seq: int = 0) -> bytes:
    lost = (int(max(0.0, min(fraction_lost, 255 / 256)) * 256) << 24) | (cum_lost & 0xFFFFFF)
    return struct.pack("!BBHI", 0x81, 201, 7, sender_ssrc) + struct.pack("!IIIIII", media_ssrc, lost, ext_seq, 0, 0, 0)


def build_remb(sender_ssrc: int, media_ssrc: int, bps: int) -> bytes:
    exp = 0
    while bps >> exp > 0x3FFFF:
        exp += 1
    mant = bps >> exp
    fci = b"REMB" + struct.pack("!BBBBI", 1, (exp << 2) | (mant >> 16), (mant >> 8) & 0xFF, mant & 0xFF, media_ssrc)
    return struct.pack("!BBHII", 0x8F, 206, 2 + len(fci) // 4, sender_ssrc, 0) + fci


def build_nack(sender_ssrc: int, media_ssrc: int, seqs: list[int]) -> bytes:
    fci = b""
    seqs = sorted(set(s & 0xFFFF for s in seqs))
    i = 0
    while i < len(seqs):
        pid, blp = seqs[i], 0
        j = i + 1
        while j < len(seqs) and 0 < ((seqs[j] - pid) & 0xFFFF) <= 16:
            blp |= 1 << (((seqs[j] - pid) & 0xFFFF) - 1)
            j += 1
        fci += struct.pack("!HH", pid, blp)
        i = j
    return struct.pack("!BBHII", 0x81, 205, 2 + len(fci) // 4, sender_ssrc, media_ssrc) + fci


def parse_rtcp(buf: bytes) -> list[dict]:
    """Parse a compound RTCP packet into a list of {'pt', 'fmt', ...}."""
    out = []
    off = 0
    while off + 4 <= len(buf):
        b0, pt, ln = struct.unpack_from("!BBH", buf, off)
        end = off + 4 * (ln + 1)
        body = buf[off + 4: end]
        fmt = b0 & 0x1F
        d = {"pt": pt, "fmt": fmt}
        if pt in (205, 206) and len(body) >= 8:
            d["sender_ssrc"], d["media_ssrc"] = struct.unpack_from("!II", body)
            if pt == 205 and fmt == 1:
                seqs = []
                for k in range(8, len(body) - 3, 4):
                    pid, blp = struct.unpack_from("!HH", body, k)
                    seqs.append(pid)
                    seqs += [(pid + i + 1) & 0xFFFF for i in range(16) if blp & (1 << i)]
                d["nack"] = seqs
            if pt == 206 and fmt == 15 and len(body) >= 16 and body[8:12] == b"REMB":
                # draft-alvestrand-rmcat-remb: receiver estimated maximum bitrate
                n, b1, b2, b3 = struct.unpack_from("!BBBB", body, 12)
                exp, mant = b1 >> 2, ((b1 & 3) << 16) | (b2 << 8) | b3
                d["remb_bps"] = mant << exp
        elif pt in (200, 201) and len(body) >= 4:
            d["ssrc"] = struct.unpack_from("!I", body)[0]
            if pt == 200 and len(body) >= 24:  # sender info: NTP <-> RTP time of one instant
                ntp_s, ntp_f, d["rtp_ts"], d["packets"], d["octets"] = struct.unpack_from("!IIIII", body, 4)
                d["ntp"] = ntp_s + ntp_f / 2.0 ** 32
            blocks = []
            k = 24 if pt == 200 else 4
            for _ in range(fmt):  # report blocks (fmt = reception report count)
                if k + 24 > len(body):
                    break
                ssrc, lost_word, hseq, jitter, lsr, dlsr = struct.unpack_from("!IIIIII", body, k)
                blocks.append({"ssrc": ssrc, "fraction_lost": (lost_word >> 24) / 256.0,
                               "cum_lost": lost_word & 0xFFFFFF, "jitter": jitter, "lsr": lsr, "dlsr": dlsr})
                k += 24
            d["reports"] = blocks
        out.append(d)
        off = end
    return out
