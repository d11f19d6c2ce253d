"""The bundled browser VNC viewer (web/vnc.js, served at / when NOVNC_ENABLE=true) driven
under Node against the RFB server: VNC auth with the JS DES, ZRLE through the JS streaming
inflate (persistent zlib window across updates), pixel-exact framebuffer, input back to the
server.  Skipped when no ``node`` binary exists."""
import asyncio
import hashlib
import json
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from mxdesk.server.rfb import RfbServer

ROOT = Path(__file__).resolve().parent.parent
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


class Desktop:
    """Frames mixing every ZRLE tile type: solid, few-colour (packed palette / palette RLE),
    long runs (plain RLE) and noise (raw)."""

    def __init__(self, w=300, h=170):
        self.w, self.h, self.n = w, h, 0
        rng = np.random.default_rng(5)
        img = np.zeros((h, w, 4), np.uint8)
        img[..., :3] = (40, 80, 120)
        img[10:60, 10:200, :3] = rng.integers(0, 256, (50, 190, 3))          # noise -> raw tiles
        img[70:130, 0:130, :3] = np.array([(0, 0, 255), (0, 255, 0), (255, 255, 255)])[
            (np.arange(130)[None, :] // 7 + np.arange(60)[:, None] // 5) % 3]  # 3 colours
        for k in range(12):                                                     # 12-colour stripes
            img[135:170, 150 + 12 * k:162 + 12 * k, :3] = (20 * k, 255 - 20 * k, 7 * k)
        img[70:130, 200:300, :3] = np.arange(100, dtype=np.uint8)[None, :, None] // 9 * 20  # long runs
        self.base = img

    def __call__(self):
        img = self.base.copy()
        if self.n > 0:  # later frames: something moves
            img[100:140, 40 + 5 * self.n:90 + 5 * self.n, :3] = (250, 10 * self.n, 3)
        self.n += 1
        return img

    def expected_rgba(self, k):
        d = Desktop(self.w, self.h)
        for _ in range(k):
            d()
        img = d()
        out = np.empty_like(img)
        out[..., 0], out[..., 1], out[..., 2], out[..., 3] = img[..., 2], img[..., 1], img[..., 0], 255
        return hashlib.md5(out.tobytes()).hexdigest()


class Inj:
    def __init__(self):
        self.events = []

    def apply(self, ev):
        self.events.append(ev)


def _run(updates, password="secret", server_pw="secret"):
    desk, inj = Desktop(), Inj()
    srv = RfbServer(desk, server_pw, None, desk.w, desk.h, fps=1000, injector=inj)

    async def go():
        server = await srv.serve_tcp("127.0.0.1", 0)
        port = server.sockets[0].getsockname()[1]
        try:
            proc = await asyncio.create_subprocess_exec(
                NODE, str(ROOT / "tools" / "vnc_client_check.js"), str(port), password, str(updates),
                stdout=subprocess.PIPE, stderr=subprocess.PIPE)
            out, err = await asyncio.wait_for(proc.communicate(), 60)
            return json.loads(out.decode().strip().splitlines()[-1]), err.decode()
        finally:
            server.close()

    res, err = asyncio.run(go())
    return desk, inj, res, err


def test_js_client_zrle_pixel_exact_and_input():
    desk, inj, res, err = _run(3)
    assert "error" not in res, (res, err)
    assert (res["width"], res["height"], res["name"]) == (300, 170, "mxdesk")
    # every update leaves the client framebuffer equal to the frame the server encoded
    assert res["digests"][0] == desk.expected_rgba(0)
    assert res["digests"][-1] in {desk.expected_rgba(k) for k in range(1, 8)}
    kinds = [e.kind for e in inj.events]
    assert "mouse" in kinds and "key" in kinds and "clipboard" in kinds
    m = next(e for e in inj.events if e.kind == "mouse")
    assert (m.x, m.y, m.buttons) == (12, 34, 1)
    assert next(e for e in inj.events if e.kind == "clipboard").text == "hi there"


def test_js_client_wrong_password():
    _, inj, res, _ = _run(1, password="nope")
    assert "auth" in res.get("error", "") and not inj.events


def test_js_des_matches_python():
    from mxdesk.server.des import vnc_response

    ch = bytes(range(16))
    js = ("const {vncResponse}=require(%r);process.stdout.write(Buffer.from(vncResponse('pässwörd9', "
          "Uint8Array.from(%r))).toString('hex'))") % (str(ROOT / "web" / "vnc.js"), list(ch))
    out = subprocess.run([NODE, "-e", js], capture_output=True, text=True, timeout=30).stdout
    assert out == vnc_response("pässwörd9", ch).hex()


def test_js_inflate_matches_zlib_across_sync_flushes():
    import zlib

    rng = np.random.default_rng(1)
    pieces = [rng.integers(0, 4, 5000, dtype=np.uint8).tobytes(), b"abc" * 3000, rng.bytes(20000),
              b"abc" * 3000 + rng.bytes(100)]
    c = zlib.compressobj(6)
    chunks = [(c.compress(p) + c.flush(zlib.Z_SYNC_FLUSH)).hex() for p in pieces]
    c9 = zlib.compressobj(9, zlib.DEFLATED, 15, 9, zlib.Z_FIXED)  # fixed-Huffman blocks too
    chunks9 = [(c9.compress(p) + c9.flush(zlib.Z_SYNC_FLUSH)).hex() for p in pieces]
    js = ("const {Inflater}=require(%r);const out=[];for(const set of %s){const f=new Inflater();"
          "for(const h of set){out.push(Buffer.from(f.push(Uint8Array.from(Buffer.from(h,'hex')))).toString('hex'));}}"
          "process.stdout.write(JSON.stringify(out))") % (str(ROOT / "web" / "vnc.js"), json.dumps([chunks, chunks9]))
    r = subprocess.run([NODE, "-e", js], capture_output=True, text=True, timeout=60)
    got = json.loads(r.stdout)
    assert [bytes.fromhex(g) for g in got] == pieces + pieces, r.stderr


def test_novnc_mode_serves_the_vnc_viewer():
    import aiohttp

    from .test_server import free_port, make_server

    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    srv.rfb = RfbServer(Desktop(), None, None, 300, 170)
    from mxdesk.server.app import serve

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            async with aiohttp.ClientSession() as s:
                async with s.get(f"http://127.0.0.1:{port}/") as r:
                    page = await r.text()
                async with s.get(f"http://127.0.0.1:{port}/vnc.js") as r:
                    js = await r.text()
            return page, js
        finally:
            await runner.cleanup()

    page, js = asyncio.run(go())
    assert "vnc.js" in page and "/websockify" in page and "RfbClient" in js
