"""RFB 3.8 server (noVNC fallback): DES vectors, VNC auth (full / view-only / wrong),
pixel-format negotiation, ZRLE + Raw updates checked pixel-exactly, incremental dirty
tiles, input injection, and the WebSocket (``/websockify``) transport."""
import asyncio
import struct
import zlib

import aiohttp
import numpy as np
import pytest

from mxdesk.server.des import des_encrypt_block, vnc_response
from mxdesk.server.rfb import RfbServer


def test_des_fips_vector():
    assert des_encrypt_block(bytes.fromhex("133457799BBCDFF1"), bytes.fromhex("0123456789ABCDEF")).hex() == \
        "85e813540f0ab405"


class Frames:
    def __init__(self, w=130, h=70):
        self.w, self.h = w, h
        self.n = 0

    def __call__(self):
        img = np.zeros((self.h, self.w, 4), np.uint8)
        img[..., 0] = 10  # B
        img[..., 1] = 20  # G
        img[..., 2] = 30  # R
        img[5:15, 70:90, :3] = (200, 100, 50)
        if self.n > 0:  # second frame: one small change (one dirty tile)
            img[66:69, 128:130, :3] = 255
        self.n += 1
        return img


class Inj:
    def __init__(self):
        self.events = []

    def apply(self, ev):
        self.events.append(ev)


async def _client(reader, writer, password, pixfmt_rgbx=True, encodings=(16, 0)):
    assert await reader.readexactly(12) == b"RFB 003.008\n"
    writer.write(b"RFB 003.008\n")
    n = (await reader.readexactly(1))[0]
    types = await reader.readexactly(n)
    writer.write(bytes([types[0]]))
    if types[0] == 2:
        ch = await reader.readexactly(16)
        writer.write(vnc_response(password, ch))
    res = struct.unpack(">I", await reader.readexactly(4))[0]
    if res != 0:
        return None
    writer.write(b"\x01")
    w, h = struct.unpack(">HH", await reader.readexactly(4))
    await reader.readexactly(16)
    nl = struct.unpack(">I", await reader.readexactly(4))[0]
    name = await reader.readexactly(nl)
    if pixfmt_rgbx:
        writer.write(b"\x00\x00\x00\x00" + struct.pack(">BBBBHHHBBB3x", 32, 24, 0, 1, 255, 255, 255, 0, 8, 16))
    writer.write(struct.pack(">BxH", 2, len(encodings)) + struct.pack(f">{len(encodings)}i", *encodings))
    return w, h, name


def _cpixels(raw, off, n):
    return np.frombuffer(raw[off:off + 3 * n], np.uint8).reshape(n, 3), off + 3 * n


def _run(raw, off):
    n = 1
    while raw[off] == 255:
        n += 255
        off += 1
    return n + raw[off], off + 1


def zrle_tile(raw, off, tw, th):
    """Independent ZRLE tile decoder (RFC 6143 §7.7.6), 3-byte CPIXELs -> (th, tw, 3)."""
    sub = raw[off]
    off += 1
    n = tw * th
    if sub == 0:
        px, off = _cpixels(raw, off, n)
    elif sub == 1:
        c, off = _cpixels(raw, off, 1)
        px = np.repeat(c, n, axis=0)
    elif 2 <= sub <= 16:
        pal, off = _cpixels(raw, off, sub)
        bits = 1 if sub == 2 else 2 if sub <= 4 else 4
        rowb = (tw * bits + 7) // 8
        idx = []
        for r in range(th):
            row = raw[off:off + rowb]
            off += rowb
            v = int.from_bytes(row, "big")
            tot = rowb * 8
            idx += [(v >> (tot - bits * (c + 1))) & ((1 << bits) - 1) for c in range(tw)]
        px = pal[np.array(idx)]
    elif sub == 128:
        out = []
        while len(out) < n:
            c, off = _cpixels(raw, off, 1)
            ln, off = _run(raw, off)
            out += [c[0]] * ln
        assert len(out) == n
        px = np.array(out)
    elif sub >= 130:
        pal, off = _cpixels(raw, off, sub - 128)
        out = []
        while len(out) < n:
            b = raw[off]
            off += 1
            if b & 128:
                ln, off = _run(raw, off)
                out += [pal[b & 127]] * ln
            else:
                out.append(pal[b])
        assert len(out) == n
        px = np.array(out)
    else:
        raise AssertionError(f"bad subencoding {sub}")
    return px.reshape(th, tw, 3), off


async def _read_update(reader, w, h, fb, zd):
    t = (await reader.readexactly(1))[0]
    assert t == 0
    await reader.readexactly(1)
    n = struct.unpack(">H", await reader.readexactly(2))[0]
    rects = []
    for _ in range(n):
        x, y, rw, rh, enc = struct.unpack(">HHHHi", await reader.readexactly(12))
        rects.append((x, y, rw, rh, enc))
        if enc == 16:
            ln = struct.unpack(">I", await reader.readexactly(4))[0]
            raw = zd.decompress(await reader.readexactly(ln))
            off = 0
            for ty in range(y, y + rh, 64):
                for tx in range(x, x + rw, 64):
                    tw, th = min(64, x + rw - tx), min(64, y + rh - ty)
                    fb[ty:ty + th, tx:tx + tw], off = zrle_tile(raw, off, tw, th)
            assert off == len(raw)
        else:
            assert enc == 0
            fb[y:y + rh, x:x + rw] = np.frombuffer(await reader.readexactly(rw * rh * 4), np.uint8).reshape(rh, rw, 4)[..., :3]
    return rects


def _tiles_frame(rng):
    """Frame whose 64x64 tiles exercise every ZRLE subencoding."""
    f = np.zeros((130, 330, 4), np.uint8)
    f[:64, 0:64, :3] = (1, 2, 3)                                        # solid
    f[:64, 64:128, :3] = rng.choice([0, 255], (64, 64, 1))              # 2 colours, noisy -> packed
    f[:64, 128:192, :3] = np.array([[9, 9, 9], [200, 1, 1], [1, 200, 1], [5, 6, 7], [90, 90, 9]])[
        rng.integers(0, 5, (64, 64))]                                   # 5 colours -> packed 4 bit
    f[:64, 192:256, :3] = np.repeat(np.arange(64, dtype=np.uint8)[:, None, None] * 3, 64, axis=1)  # 64 colours, long runs
    f[:64, 256:320, :3] = rng.integers(0, 256, (64, 64, 3))             # raw
    f[64:, :, :3] = np.where((np.arange(330) // 17 % 2)[None, :, None] == 0, 40, 220)  # 2 colours in runs
    f[64:, 300:330, :3] = 77
    return f


@pytest.mark.parametrize("perm", [[0, 1, 2], [2, 1, 0]])
def test_native_zrle_all_subencodings_roundtrip(native, perm):
    import zlib

    rng = np.random.default_rng(5)
    frame = _tiles_frame(rng)
    enc = native.rfb.ZrleEncoder(6)
    zd = zlib.decompressobj()
    for rect in [(0, 0, 330, 130), (64, 0, 200, 64), (3, 70, 61, 60)]:
        x, y, w, h = rect
        body = enc.encode(frame, x, y, w, h, perm)
        ln = struct.unpack(">I", body[:4])[0]
        assert ln == len(body) - 4
        raw = zd.decompress(body[4:])
        off, got = 0, np.zeros((h, w, 3), np.uint8)
        for ty in range(0, h, 64):
            for tx in range(0, w, 64):
                tw, th = min(64, w - tx), min(64, h - ty)
                got[ty:ty + th, tx:tx + tw], off = zrle_tile(raw, off, tw, th)
        assert off == len(raw)
        assert np.array_equal(got, frame[y:y + h, x:x + w][..., perm])
    st = enc.stats
    assert st[1] and st[0] and st[128] + sum(st[130:]) > 0 and sum(st[2:17]) > 0


def test_native_tile_diff(native):
    a = np.zeros((130, 200, 4), np.uint8)
    b = a.copy()
    b[129, 199, 1] = 1
    b[0, 64, 0] = 1
    fl = native.rfb.tile_diff(b, a, 64)
    assert fl.shape == (3, 4) and fl.sum() == 2 and fl[2, 3] == 1 and fl[0, 1] == 1


@pytest.mark.parametrize("encodings", [(16, 0), (0,)])
def test_rfb_tcp_auth_updates_input(encodings):
    frames = Frames()
    inj = Inj()
    srv = RfbServer(frames, "pw", "view", 130, 70, fps=1000, injector=inj)

    async def go():
        server = await srv.serve_tcp("127.0.0.1", 0)
        port = server.sockets[0].getsockname()[1]
        try:
            # wrong password
            r, w = await asyncio.open_connection("127.0.0.1", port)
            assert await _client(r, w, "nope") is None
            w.close()
            # full access
            r, w = await asyncio.open_connection("127.0.0.1", port)
            wh = await _client(r, w, "pw", encodings=encodings)
            assert wh[:2] == (130, 70) and wh[2] == b"mxdesk"
            fb = np.zeros((70, 130, 3), np.uint8)
            zd = zlib.decompressobj()
            w.write(struct.pack(">BBHHHH", 3, 0, 0, 0, 130, 70))
            await _read_update(r, 130, 70, fb, zd)
            ref = frames.__class__()()  # first frame, converted to RGBX
            assert np.array_equal(fb, ref[..., [2, 1, 0]])
            w.write(struct.pack(">BBHHHH", 3, 1, 0, 0, 130, 70))  # incremental
            rects = await _read_update(r, 130, 70, fb, zd)
            assert rects == [(128, 64, 2, 6, rects[0][4])]  # only the changed 64x64 tile (clipped)
            assert np.all(fb[66:69, 128:130] == 255)
            w.write(struct.pack(">BBHH", 5, 1, 40, 30) + struct.pack(">BBxxI", 4, 1, 0xff0d))
            await w.drain()
            await asyncio.sleep(0.1)
            w.close()
            # view-only: input ignored
            r, w = await asyncio.open_connection("127.0.0.1", port)
            await _client(r, w, "view", encodings=encodings)
            w.write(struct.pack(">BBHH", 5, 0, 1, 1))
            await w.drain()
            await asyncio.sleep(0.1)
            w.close()
        finally:
            server.close()

    asyncio.run(go())
    kinds = [(e.kind, e.x, e.y, e.buttons) if e.kind == "mouse" else (e.kind, e.keysym, e.down) for e in inj.events]
    assert kinds == [("mouse", 40, 30, 1), ("key", 0xff0d, True)]


def test_rfb_over_websocket():
    from aiohttp import web

    frames = Frames()
    srv = RfbServer(frames, None, None, 130, 70, fps=1000)

    async def go():
        app = web.Application()
        app.router.add_get("/websockify", srv.ws_handler)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        try:
            async with aiohttp.ClientSession() as s:
                async with s.ws_connect(f"http://127.0.0.1:{port}/websockify", protocols=("binary",)) as ws:
                    assert ws.protocol == "binary"
                    got = (await ws.receive()).data
                    assert got == b"RFB 003.008\n"
                    await ws.send_bytes(b"RFB 003.008\n")
                    assert (await ws.receive()).data == bytes([1, 1])  # no password -> security None
                    await ws.send_bytes(b"\x01")
                    assert struct.unpack(">I", (await ws.receive()).data)[0] == 0
                    await ws.send_bytes(b"\x01")
                    init = (await ws.receive()).data
                    assert struct.unpack(">HH", init[:4]) == (130, 70)
        finally:
            await runner.cleanup()

    asyncio.run(go())


def test_rfb_cut_text_capped_and_view_only_ignored():
    """ClientCutText carries an attacker-chosen u32 length -- an oversized one closes
    the connection without buffering; view-only sessions never set the clipboard."""
    import time

    frames = Frames()
    inj = Inj()
    srv = RfbServer(frames, "pw", "view", 130, 70, fps=1000, injector=inj)

    async def go():
        server = await srv.serve_tcp("127.0.0.1", 0)
        port = server.sockets[0].getsockname()[1]
        try:
            r, w = await asyncio.open_connection("127.0.0.1", port)
            await _client(r, w, "pw")
            w.write(struct.pack(">B3sI", 6, b"\0\0\0", 5) + b"hello")
            w.write(struct.pack(">B3sI", 6, b"\0\0\0", 0xFFFFFFF0))  # 4 GiB announced
            await w.drain()
            t0 = time.monotonic()
            assert await asyncio.wait_for(r.read(), 5) is not None  # server closes: EOF
            assert time.monotonic() - t0 < 5
            w.close()
            r, w = await asyncio.open_connection("127.0.0.1", port)
            await _client(r, w, "view")
            w.write(struct.pack(">B3sI", 6, b"\0\0\0", 3) + b"abc")
            await w.drain()
            await asyncio.sleep(0.1)
            w.close()
        finally:
            server.close()

    asyncio.run(go())
    assert [(e.kind, e.text) for e in inj.events] == [("clipboard", "hello")]
