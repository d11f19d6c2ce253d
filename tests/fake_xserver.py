"""A minimal X11 protocol server for tests (there is no X server in the image or on the GPU box).

It speaks enough of the core protocol and of the MIT-SHM, DAMAGE and XFIXES extensions for the
real libX11 / libXext / libXdamage / libXfixes that ``mxdesk/models/x11.py`` drives through
ctypes: connection setup (one 24-bit TrueColor screen), QueryExtension, GetProperty,
GetInputFocus (XSync), ShmQueryVersion / ShmAttach / ShmDetach / ShmGetImage (pixels written into
the client's SysV segment at the request's offset), DamageQueryVersion / Create / Subtract /
Destroy with DamageNotify events, XFixesQueryVersion / CreateRegion / FetchRegion /
DestroyRegion.  The framebuffer is a numpy (H, W, 4) BGRx array; ``draw()`` changes it and
accumulates damage like a real server.  Listens on TCP 127.0.0.1:6000+N (display
``127.0.0.1:N``).
"""
from __future__ import annotations

import ctypes
import socket
import struct
import threading

import numpy as np

SHM_OP, DAMAGE_OP, XFIXES_OP, XTEST_OP = 130, 131, 132, 133
DAMAGE_EVENT = 90
ROOT, VISUAL, COLORMAP = 0x100, 0x21, 0x20
EXTENSIONS = {b"MIT-SHM": (SHM_OP, 0, 128), b"DAMAGE": (DAMAGE_OP, DAMAGE_EVENT, 140),
              b"XFIXES": (XFIXES_OP, 100, 150), b"XTEST": (XTEST_OP, 0, 0)}
# core keyboard map: keycode -> (unshifted, shifted) keysyms
KEYMAP = {38: (0x61, 0x41), 36: (0xFF0D, 0), 50: (0xFFE1, 0), 9: (0xFF1B, 0)}
MIN_KEYCODE, MAX_KEYCODE = 8, 255


def _pad(n: int) -> int:
    return (4 - n % 4) % 4


class FakeXServer:
    def __init__(self, width: int = 320, height: int = 192):
        self.w, self.h = width, height
        self.fb = np.zeros((height, width, 4), np.uint8)
        self.lock = threading.Lock()
        self.damage_rects: list[tuple[int, int, int, int]] = []
        self.damages: dict[int, object] = {}
        self.regions: dict[int, list] = {}
        self.segments: dict[int, int] = {}  # shmseg -> attached address in this process
        self.requests: list[tuple[int, int]] = []  # (major, minor) of every request
        self.getimage_rows = 0
        self.fake_inputs: list[tuple[int, int, int, int]] = []  # XTestFakeInput (type, detail, x, y)
        self.cursor = None  # (xhot, yhot, serial, (h, w) uint32 ARGB) for XFixesGetCursorImage
        self.seq: dict[socket.socket, int] = {}  # last request sequence per connection (events carry it)
        self.send_lock = threading.Lock()  # replies (server threads) and events (draw) never interleave
        self.libc = ctypes.CDLL("libc.so.6", use_errno=True)
        self.libc.shmat.restype = ctypes.c_void_p
        self.libc.shmat.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        self.libc.shmdt.argtypes = [ctypes.c_void_p]
        self.sock = None
        for n in range(40, 140):
            # no SO_REUSEADDR: with it two processes (pytest-xdist workers) could both bind a port
            # before either listens, and the second listen() would fail; busy ports are skipped
            s = socket.socket()
            try:
                s.bind(("127.0.0.1", 6000 + n))
                s.listen(4)
            except OSError:
                s.close()
                continue
            self.sock, self.display = s, f"127.0.0.1:{n}"
            break
        if self.sock is None:
            raise OSError("no free X display port")
        self.conns: list[socket.socket] = []
        self._stop = False
        self.thread = threading.Thread(target=self._accept, daemon=True)
        self.thread.start()

    # ------------------------------------------------------------------ test API
    def draw(self, x: int, y: int, w: int, h: int, value) -> None:
        """Fill a rectangle (BGRx bytes or a scalar) and damage it (DamageNotify to clients)."""
        with self.lock:
            self.fb[y:y + h, x:x + w] = value
            self.damage_rects.append((x, y, w, h))
            targets = list(self.damages.items())
        for did, conn in targets:
            ev = struct.pack("<BBHIIIhhHHhhHH", DAMAGE_EVENT, 3, self.seq.get(conn, 0), ROOT, did, 0, x, y, w, h, 0, 0,
                             self.w, self.h)
            try:
                with self.send_lock:
                    conn.sendall(ev)
            except OSError:
                pass

    def close(self) -> None:
        self._stop = True
        for c in self.conns:
            try:
                c.shutdown(socket.SHUT_RDWR)
                c.close()
            except OSError:
                pass
        self.sock.close()
        for addr in self.segments.values():
            self.libc.shmdt(ctypes.c_void_p(addr))

    # ------------------------------------------------------------------ protocol
    def _accept(self) -> None:
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            self.conns.append(c)
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    @staticmethod
    def _recv(c: socket.socket, n: int) -> bytes:
        b = b""
        while len(b) < n:
            chunk = c.recv(n - len(b))
            if not chunk:
                raise EOFError
            b += chunk
        return b

    def _setup_reply(self) -> bytes:
        vendor = b"mxdesk-test"
        formats = struct.pack("<BBB5x", 1, 1, 32) + struct.pack("<BBB5x", 24, 32, 32)
        visual = struct.pack("<IBBHIII4x", VISUAL, 4, 8, 256, 0xFF0000, 0x00FF00, 0x0000FF)
        depth = struct.pack("<BxH4x", 24, 1) + visual
        screen = struct.pack("<IIIIIHHHHHHIBBBB", ROOT, COLORMAP, 0xFFFFFF, 0, 0, self.w, self.h, 300, 200, 1, 1,
                             VISUAL, 0, 0, 24, 1) + depth
        body = struct.pack("<IIIIHHBBBBBBBB4x", 1, 0x00400000, 0x001FFFFF, 0, len(vendor), 65535, 1, 2, 0, 0, 32, 32,
                           MIN_KEYCODE, MAX_KEYCODE)
        body += vendor + b"\0" * _pad(len(vendor)) + formats + screen
        return struct.pack("<BxHHH", 1, 11, 0, len(body) // 4) + body

    def _serve(self, c: socket.socket) -> None:
        try:
            hdr = self._recv(c, 12)
            if hdr[0:1] != b"l":
                return  # little-endian clients only
            n_name, n_data = struct.unpack_from("<HH", hdr, 6)
            self._recv(c, n_name + _pad(n_name) + n_data + _pad(n_data))
            with self.send_lock:
                c.sendall(self._setup_reply())
            seq = 0
            while True:
                h = self._recv(c, 4)
                op, data, length = struct.unpack("<BBH", h)
                body = self._recv(c, length * 4 - 4) if length > 1 else b""
                seq = (seq + 1) & 0xFFFF
                self.seq[c] = seq
                self.requests.append((op, data))
                reply = self._handle(c, op, data, body, seq)
                if reply:
                    with self.send_lock:
                        c.sendall(reply)
        except (EOFError, OSError):
            pass

    @staticmethod
    def _reply(seq: int, data: int = 0, payload: bytes = b"", extra: bytes = b"") -> bytes:
        payload = payload + b"\0" * (24 - len(payload))
        return struct.pack("<BBHI", 1, data, seq, len(extra) // 4) + payload + extra

    def _handle(self, c, op: int, data: int, body: bytes, seq: int) -> bytes | None:
        if op == 98:  # QueryExtension
            n = struct.unpack_from("<H", body, 0)[0]
            name = body[4:4 + n]
            major, ev, err = EXTENSIONS.get(name, (0, 0, 0))
            return self._reply(seq, 0, struct.pack("<BBBB", int(major != 0), major, ev, err))
        if op == 20:  # GetProperty: no such property
            return self._reply(seq, 0, struct.pack("<III", 0, 0, 0))
        if op == 43:  # GetInputFocus (XSync)
            return self._reply(seq, 1, struct.pack("<I", ROOT))
        if op == SHM_OP:
            return self._shm(data, body, seq)
        if op == DAMAGE_OP:
            return self._damage(c, data, body, seq)
        if op == XFIXES_OP:
            return self._xfixes(data, body, seq)
        if op == XTEST_OP:
            if data == 0:  # XTestGetVersion
                return self._reply(seq, 2, struct.pack("<H", 2))
            if data == 2:  # XTestFakeInput
                typ, detail = body[0], body[1]
                rx, ry = struct.unpack_from("<hh", body, 20) if typ == 6 else (0, 0)  # root x/y: motion only
                self.fake_inputs.append((typ, detail, rx, ry))
            return None
        if op == 101:  # GetKeyboardMapping(first, count)
            first, count = body[0], body[1]
            syms = b"".join(struct.pack("<II", *KEYMAP.get(k, (0, 0))) for k in range(first, first + count))
            return self._reply(seq, 2, b"", syms)
        if op == 119:  # GetModifierMapping: one keycode per modifier, shift = 50
            return self._reply(seq, 1, b"", struct.pack("<8B", 50, 0, 0, 0, 0, 0, 0, 0))
        return None  # requests without replies (or not modelled) are accepted silently

    def _shm(self, minor: int, body: bytes, seq: int) -> bytes | None:
        if minor == 0:  # ShmQueryVersion
            return self._reply(seq, 0, struct.pack("<HHHHB", 1, 2, 0, 0, 2))
        if minor == 1:  # ShmAttach
            shmseg, shmid = struct.unpack_from("<II", body, 0)
            addr = self.libc.shmat(shmid, None, 0)
            if addr in (None, ctypes.c_void_p(-1).value):
                raise OSError("shmat failed in the fake server")
            self.segments[shmseg] = addr
            return None
        if minor == 2:  # ShmDetach
            shmseg = struct.unpack_from("<I", body, 0)[0]
            addr = self.segments.pop(shmseg, None)
            if addr:
                self.libc.shmdt(ctypes.c_void_p(addr))
            return None
        if minor == 4:  # ShmGetImage
            _, x, y, w, h, _, _, shmseg, offset = struct.unpack_from("<IhhHHIB3xII", body, 0)
            with self.lock:
                px = np.ascontiguousarray(self.fb[y:y + h, x:x + w])
            self.getimage_rows += h
            ctypes.memmove(self.segments[shmseg] + offset, px.ctypes.data, px.nbytes)
            return self._reply(seq, 24, struct.pack("<II", VISUAL, px.nbytes))
        return None

    def _damage(self, c, minor: int, body: bytes, seq: int) -> bytes | None:
        if minor == 0:  # DamageQueryVersion
            return self._reply(seq, 0, struct.pack("<II", 1, 1))
        if minor == 1:  # DamageCreate
            did = struct.unpack_from("<I", body, 0)[0]
            with self.lock:
                self.damages[did] = c
            return None
        if minor == 2:  # DamageDestroy
            with self.lock:
                self.damages.pop(struct.unpack_from("<I", body, 0)[0], None)
            return None
        if minor == 3:  # DamageSubtract(damage, repair = None, parts)
            _, repair, parts = struct.unpack_from("<III", body, 0)
            with self.lock:
                rects, self.damage_rects = self.damage_rects, []
            if parts:
                self.regions[parts] = rects
            return None
        return None

    def _xfixes(self, minor: int, body: bytes, seq: int) -> bytes | None:
        if minor == 0:  # XFixesQueryVersion
            return self._reply(seq, 0, struct.pack("<II", 5, 0))
        if minor == 5:  # CreateRegion(region, rects...)
            rid = struct.unpack_from("<I", body, 0)[0]
            self.regions[rid] = [struct.unpack_from("<hhHH", body, 4 + 8 * i) for i in range((len(body) - 4) // 8)]
            return None
        if minor == 10:  # DestroyRegion
            self.regions.pop(struct.unpack_from("<I", body, 0)[0], None)
            return None
        if minor in (4, 25) and self.cursor is not None:  # GetCursorImage (AndName)
            xhot, yhot, serial, px = self.cursor
            hh, ww = px.shape
            head = struct.pack("<hhHHHHI", 10, 20, ww, hh, xhot, yhot, serial)
            pixels = np.ascontiguousarray(px, np.uint32).tobytes()
            if minor == 4:
                return self._reply(seq, 0, head, pixels)
            name = b"left_ptr"
            head += struct.pack("<IHH", 0, len(name), 0)
            return self._reply(seq, 0, head, pixels + name + b"\0" * _pad(len(name)))
        if minor == 19:  # FetchRegion -> extents + rectangles
            rects = self.regions.get(struct.unpack_from("<I", body, 0)[0], [])
            if rects:
                x0 = min(r[0] for r in rects)
                y0 = min(r[1] for r in rects)
                x1 = max(r[0] + r[2] for r in rects)
                y1 = max(r[1] + r[3] for r in rects)
                ext = struct.pack("<hhHH", x0, y0, x1 - x0, y1 - y0)
            else:
                ext = struct.pack("<hhHH", 0, 0, 0, 0)
            extra = b"".join(struct.pack("<hhHH", *r) for r in rects)
            return self._reply(seq, 0, ext, extra)
        return None
