"""RFB 3.8 (VNC) server + WebSocket bridge: the noVNC fallback front end
(reference entrypoint.sh:120-125 runs ``x11vnc -shared -forever
-passwd $BASIC_AUTH_PASSWORD [-viewpasswd $NOVNC_VIEWPASS] -rfbport 5900`` behind
``novnc_proxy --listen 8080``).

* Security: VNC authentication (DES challenge, RFC 6143 §7.2.2) with the full-access
  password and an optional view-only password (input is ignored for view-only clients);
  ``None`` when no password is configured.
* Encodings: ZRLE (native C++ encoder, csrc/rfb/zrle.cpp: solid / packed-palette / RLE /
  palette-RLE / raw 64x64 tiles over a per-connection zlib stream), Raw, and the
  DesktopSize pseudo-encoding.  Updates carry only the 64x64 tiles that changed since the
  last frame sent to that client (incremental updates), merged into row spans.
* Pixel formats: 32 bpp true colour with any byte permutation of R/G/B (noVNC asks for
  RGBX; the server-native format is BGRX).
* Transports: plain TCP (:5900) and WebSocket (``/websockify``, subprotocol ``binary``),
  which is what a stock noVNC client connects to.
"""
from __future__ import annotations

import asyncio
import logging
import os
import struct
import time
from typing import Any, Callable

import numpy as np
from aiohttp import WSMsgType, web

from .. import native

from .des import vnc_response
from .input import InputEvent

log = logging.getLogger("mxdesk.rfb")

ENC_RAW, ENC_COPYRECT, ENC_ZRLE, ENC_DESKTOPSIZE = 0, 1, 16, -223
TILE = 64


# ClientCutText cap (RFC 6143 7.5.6 has a u32 length; 1 MiB is ample for a clipboard)
MAX_CUT_TEXT = 1 << 20

class FrameCache:
    """Latest desktop frame (H, W, 4 BGRx), rendered at most `fps` times per second and
    shared by all RFB connections."""

    def __init__(self, grab: Callable[[], np.ndarray], fps: float = 30.0):
        self.grab = grab
        self.period = 1.0 / fps
        self.frame: np.ndarray | None = None
        self.gen = 0
        self.t = 0.0
        self.lock = asyncio.Lock()

    async def latest(self) -> tuple[np.ndarray, int]:
        async with self.lock:
            now = time.monotonic()
            if self.frame is None or now - self.t >= self.period:
                self.frame = await asyncio.get_running_loop().run_in_executor(None, self.grab)
                self.gen += 1
                self.t = now
            return self.frame, self.gen


class _Stream:
    """Byte-stream adapter over asyncio streams or an aiohttp WebSocket."""

    def __init__(self, reader=None, writer=None, ws: web.WebSocketResponse | None = None):
        self.reader, self.writer, self.ws = reader, writer, ws
        self.buf = bytearray()

    async def read(self, n: int) -> bytes:
        if self.ws is None:
            return await self.reader.readexactly(n)
        while len(self.buf) < n:
            msg = await self.ws.receive()
            if msg.type == WSMsgType.BINARY:
                self.buf += msg.data
            elif msg.type == WSMsgType.TEXT:
                self.buf += msg.data.encode("latin-1")
            else:
                raise ConnectionError("websocket closed")
        out = bytes(self.buf[:n])
        del self.buf[:n]
        return out

    async def write(self, data: bytes) -> None:
        if self.ws is None:
            self.writer.write(data)
            await self.writer.drain()
        else:
            await self.ws.send_bytes(data)


def pixel_format_bytes() -> bytes:
    # bpp 32, depth 24, little endian, true colour, max 255, shifts R16 G8 B0 (BGRX in memory)
    return struct.pack(">BBBBHHHBBB3x", 32, 24, 0, 1, 255, 255, 255, 16, 8, 0)


class RfbConnection:
    def __init__(self, server: "RfbServer", stream: _Stream):
        self.srv, self.s = server, stream
        self.view_only = False
        self.encodings: list[int] = [ENC_RAW]
        self.perm = None  # byte permutation from BGRX to the client format
        self.last: np.ndarray | None = None
        self.zrle = native().rfb.ZrleEncoder(6)  # one zlib stream per connection (RFC 6143 §7.7.6)
        self.pending: tuple[int, int, int, int, int] | None = None
        self.w, self.h = server.width, server.height

    # ------------------------------------------------------------------ handshake
    async def handshake(self) -> bool:
        await self.s.write(b"RFB 003.008\n")
        ver = await self.s.read(12)
        if not ver.startswith(b"RFB 003."):
            return False
        minor = int(ver[8:11])
        pw, vpw = self.srv.password, self.srv.view_password
        sec = 2 if (pw or vpw) else 1
        if minor >= 7:
            await self.s.write(bytes([1, sec]))
            chosen = (await self.s.read(1))[0]
            if chosen != sec:
                await self.s.write(struct.pack(">I", 1) + self._reason("unsupported security type"))
                return False
        else:
            await self.s.write(struct.pack(">I", sec))
        if sec == 2:
            challenge = os.urandom(16)
            await self.s.write(challenge)
            resp = await self.s.read(16)
            if pw and resp == vnc_response(pw, challenge):
                self.view_only = False
            elif vpw and resp == vnc_response(vpw, challenge):
                self.view_only = True
            else:
                await self.s.write(struct.pack(">I", 1) + (self._reason("authentication failed") if minor >= 8 else b""))
                return False
        if sec == 2 or minor >= 8:
            await self.s.write(struct.pack(">I", 0))
        await self.s.read(1)  # ClientInit shared flag (always shared, like x11vnc -shared)
        name = self.srv.name.encode()
        await self.s.write(struct.pack(">HH", self.w, self.h) + pixel_format_bytes() + struct.pack(">I", len(name)) +
                           name)
        return True

    @staticmethod
    def _reason(text: str) -> bytes:
        b = text.encode()
        return struct.pack(">I", len(b)) + b

    # ------------------------------------------------------------------ messages
    async def run(self) -> None:
        if not await self.handshake():
            return
        updater = asyncio.create_task(self._update_loop())
        try:
            while True:
                t = (await self.s.read(1))[0]
                if t == 0:  # SetPixelFormat
                    d = await self.s.read(19)
                    bpp, depth, be, tc, rmax, gmax, bmax, rs, gs, bs = struct.unpack(">3xBBBBHHHBBB3x", d)
                    if bpp != 32 or not tc or be or sorted((rs, gs, bs)) != [0, 8, 16]:
                        raise ConnectionError("unsupported pixel format")
                    # output byte index i holds channel with shift 8*i; server BGRX has B@0 G@1 R@2
                    src = {bs: 0, gs: 1, rs: 2}
                    self.perm = None if (rs, gs, bs) == (16, 8, 0) else [src[0], src[8], src[16], 3]
                elif t == 2:  # SetEncodings
                    _, n = struct.unpack(">BH", await self.s.read(3))
                    self.encodings = list(struct.unpack(f">{n}i", await self.s.read(4 * n))) if n else []
                elif t == 3:  # FramebufferUpdateRequest
                    inc, x, y, w, h = struct.unpack(">BHHHH", await self.s.read(9))
                    self.pending = (inc, x, y, w, h)
                elif t == 4:  # KeyEvent
                    down, _, key = struct.unpack(">BHI", await self.s.read(7))
                    if not self.view_only:
                        self.srv.inject(InputEvent("key", keysym=key, down=bool(down)))
                elif t == 5:  # PointerEvent
                    mask, x, y = struct.unpack(">BHH", await self.s.read(5))
                    if not self.view_only:
                        scroll = 1 if mask & 8 else (-1 if mask & 16 else 0)
                        self.srv.inject(InputEvent("mouse", x, y, mask & 7, scroll))
                elif t == 6:  # ClientCutText
                    _, n = struct.unpack(">3sI", await self.s.read(7))
                    if n > MAX_CUT_TEXT:  # attacker-chosen u32: never buffer it
                        raise ConnectionError(f"ClientCutText of {n} bytes exceeds {MAX_CUT_TEXT}")
                    text = (await self.s.read(n)).decode("latin-1")
                    if not self.view_only and self.srv.clipboard_in:
                        self.srv.inject(InputEvent("clipboard", text=text))
                else:
                    raise ConnectionError(f"unknown client message {t}")
        except (asyncio.IncompleteReadError, ConnectionError, ConnectionResetError):
            pass
        finally:
            updater.cancel()

    async def _update_loop(self) -> None:
        while True:
            if self.pending is None:
                await asyncio.sleep(0.005)
                continue
            inc = self.pending[0]
            frame, _ = await self.srv.frames.latest()
            rects = self._dirty_rects(frame, incremental=bool(inc))
            if not rects:
                await asyncio.sleep(self.srv.frames.period / 2)
                continue
            self.pending = None
            await self.s.write(self._encode_update(frame, rects))
            self.last = frame

    # ------------------------------------------------------------------ encoding
    def _dirty_rects(self, frame: np.ndarray, incremental: bool) -> list[tuple[int, int, int, int]]:
        h, w = frame.shape[:2]
        if not incremental or self.last is None or self.last.shape != frame.shape:
            return [(0, 0, w, h)]
        th, tw = (h + TILE - 1) // TILE, (w + TILE - 1) // TILE
        tiles = native().rfb.tile_diff(np.ascontiguousarray(frame), np.ascontiguousarray(self.last), TILE)
        rects = []
        for ty in range(th):
            tx = 0
            while tx < tw:
                if tiles[ty, tx]:
                    x0 = tx
                    while tx < tw and tiles[ty, tx]:
                        tx += 1
                    x, y = x0 * TILE, ty * TILE
                    rects.append((x, y, min(tx * TILE, w) - x, min(TILE, h - y)))
                else:
                    tx += 1
        return rects

    def _pixels(self, region: np.ndarray) -> np.ndarray:
        return region if self.perm is None else region[..., self.perm]

    def _encode_update(self, frame: np.ndarray, rects: list[tuple[int, int, int, int]]) -> bytes:
        zrle = ENC_ZRLE in self.encodings
        out = [struct.pack(">BxH", 0, len(rects))]
        frame = np.ascontiguousarray(frame)
        perm = list(self.perm[:3]) if self.perm is not None else [0, 1, 2]
        for x, y, w, h in rects:
            if zrle:  # native ZRLE: all tile subencodings, persistent zlib stream
                out.append(struct.pack(">HHHHi", x, y, w, h, ENC_ZRLE) + self.zrle.encode(frame, x, y, w, h, perm))
            else:
                px = self._pixels(frame[y:y + h, x:x + w])
                out.append(struct.pack(">HHHHi", x, y, w, h, ENC_RAW) + np.ascontiguousarray(px).tobytes())
        return b"".join(out)


class RfbServer:
    def __init__(self, grab: Any, password: str | None, view_password: str | None = None,
                 width: int | None = None, height: int | None = None, fps: float = 30.0, name: str = "mxdesk",
                 injector: Any = None, clipboard_in: bool = True):
        """``grab`` is a callable returning an (H, W, 4) BGRx frame, or a StreamPipeline (its
        desktop is then rendered/captured through ``FrameGrabber``)."""
        if not callable(grab):
            from .framegrab import FrameGrabber

            fg = FrameGrabber.for_pipeline(grab)
            width, height, fps, grab = fg.width, fg.height, fg.fps, fg.grab
            if injector is None:
                from .input import SyntheticInjector

                injector = SyntheticInjector(fg, width, height)
        self.frames = FrameCache(grab, fps)
        self.password = password or None
        self.view_password = view_password or None
        self.width, self.height = width, height
        self.name = name
        self.injector = injector
        self.clipboard_in = clipboard_in
        self.connections = 0

    def inject(self, ev: InputEvent) -> None:
        if self.injector is not None:
            self.injector.apply(ev)

    async def handle_stream(self, stream: _Stream) -> None:
        self.connections += 1
        try:
            await RfbConnection(self, stream).run()
        finally:
            self.connections -= 1

    async def ws_handler(self, request: web.Request) -> web.WebSocketResponse:
        ws = web.WebSocketResponse(protocols=("binary",), heartbeat=10, max_msg_size=16 * 1024 * 1024)
        await ws.prepare(request)
        await self.handle_stream(_Stream(ws=ws))
        await ws.close()
        return ws

    async def serve_tcp(self, host: str = "127.0.0.1", port: int = 5900) -> asyncio.AbstractServer:
        async def cb(reader, writer):
            try:
                await self.handle_stream(_Stream(reader, writer))
            finally:
                writer.close()

        return await asyncio.start_server(cb, host, port)
