"""Client-driven resize (RandR planning, live session restart at the new size), remote
clipboard push and cursor images (WEBRTC_ENABLE_RESIZE Dockerfile:211,
xclip/xdotool Dockerfile:428-430)."""
import asyncio
import base64
import io
import json
import types

import aiohttp
import numpy as np
from PIL import Image

from mxdesk.codec.h264_decoder import Decoder
from mxdesk.display.randr import clamp_size, parse_query, plan_resize, resize_display
from mxdesk.models.x11 import argb_longs_to_rgba
from mxdesk.pipeline.stream import parse_frame
from mxdesk.server import desktop_sync as DS
from mxdesk.utils.png import encode_rgba

from .test_server import free_port, make_server

XRANDR_DUMMY = """Screen 0: minimum 8 x 8, current 1920 x 1080, maximum 32767 x 32767
DUMMY0 connected primary 1920x1080+0+0 (normal left inverted right x axis y axis) 0mm x 0mm
   1920x1080R    59.93*+
   1280x720      60.00
DUMMY1 disconnected (normal left inverted right x axis y axis)
"""


def test_clamp_size():
    assert clamp_size(1366, 768) == (1360, 768)
    assert clamp_size(100, 50) == (320, 240)
    assert clamp_size(10000, 9000) == (7680, 4320)
    assert clamp_size(1921, 1081) == (1920, 1080)


def test_parse_query_and_plan_resize():
    outs = parse_query(XRANDR_DUMMY)
    assert [o.name for o in outs] == ["DUMMY0", "DUMMY1"]
    assert outs[0].connected and outs[0].modes == ["1920x1080R", "1280x720"] and outs[0].current == "1920x1080R"
    assert plan_resize(XRANDR_DUMMY, 1920, 1080) == []  # already current
    assert plan_resize(XRANDR_DUMMY, 1280, 720) == [["--output", "DUMMY0", "--mode", "1280x720"]]
    cmds = plan_resize(XRANDR_DUMMY, 1600, 896)
    assert cmds[0][:2] == ["--newmode", "1600x896R"] and cmds[1] == ["--addmode", "DUMMY0", "1600x896R"]
    assert cmds[2] == ["--output", "DUMMY0", "--mode", "1600x896R"]
    # CVT-RB timings: hdisplay/htotal, vdisplay, sync polarities of `cvt -r`
    t = cmds[0][2:]
    assert t[1] == "1600" and int(t[4]) == 1600 + 160 and t[5] == "896" and t[-2:] == ["+hsync", "-vsync"]


def test_resize_display_runs_xrandr(monkeypatch):
    calls = []

    def fake_run(argv, **kw):
        calls.append(argv[1:])
        assert kw["env"]["DISPLAY"] == ":5"
        out = XRANDR_DUMMY if argv[1] == "--query" else ""
        return types.SimpleNamespace(returncode=0, stdout=out, stderr="")
    monkeypatch.setattr("shutil.which", lambda name: "/usr/bin/" + name)
    cmds = resize_display(":5", 1280, 720, run=fake_run)
    assert calls == [["--query"], ["--output", "DUMMY0", "--mode", "1280x720"]] and cmds == calls[1:]


def test_png_roundtrip_and_cursor_conversion():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (24, 17, 4), dtype=np.uint8)
    back = np.asarray(Image.open(io.BytesIO(encode_rgba(img))).convert("RGBA"))
    assert np.array_equal(back, img)
    # premultiplied ARGB in unsigned longs -> straight RGBA
    px = np.array([0xFF112233, 0x80404040, 0x00000000, 0xFFFFFFFF], np.uint64)
    rgba = argb_longs_to_rgba(px, 2, 2)
    assert rgba.shape == (2, 2, 4)
    assert list(rgba[0, 0]) == [0x11, 0x22, 0x33, 0xFF]
    assert list(rgba[0, 1]) == [128, 128, 128, 0x80]  # 0x40 * 255 / 0x80, rounded
    assert list(rgba[1, 0]) == [0, 0, 0, 0] and list(rgba[1, 1]) == [255, 255, 255, 255]
    msg = json.loads(DS.cursor_message(7, 3, 4, rgba))
    assert msg["type"] == "cursor" and msg["data"]["handle"] == 7 and msg["data"]["hotspot"] == {"x": 3, "y": 4}
    assert base64.b64decode(msg["data"]["curdata"]).startswith(b"\x89PNG")


def test_cursor_sync_only_on_new_serial():
    imgs = [(1, 0, 0, np.zeros((2, 2, 4), np.uint8)), (1, 0, 0, np.zeros((2, 2, 4), np.uint8)),
            (2, 1, 1, np.full((2, 2, 4), 255, np.uint8))]
    cap = types.SimpleNamespace(cursor_image=lambda: imgs.pop(0))
    cs = DS.CursorSync(cap)
    assert cs.poll() is not None and cs.poll() is None
    m = cs.poll()
    assert json.loads(m)["data"]["handle"] == 2 and cs.last_message == m


def test_clipboard_sync_xclip(monkeypatch):
    state = {"sel": "first"}
    calls = []

    def fake_run(argv, **kw):
        calls.append(argv[1:])
        if argv[-1] == "-o":
            return types.SimpleNamespace(returncode=0, stdout=state["sel"].encode())
        state["sel"] = kw["input"].decode()
        return types.SimpleNamespace(returncode=0, stdout=b"")
    monkeypatch.setattr("shutil.which", lambda name: "/usr/bin/" + name)
    cb = DS.ClipboardSync(None, ":0", run=fake_run)
    assert cb.mode == "xclip"
    assert cb.poll() is None  # baseline
    state["sel"] = "copied on the remote"
    assert cb.poll() == "copied on the remote" and cb.poll() is None
    cb.write("from the browser")
    assert state["sel"] == "from the browser" and cb.poll() is None  # no echo back to the client
    assert ["-selection", "clipboard", "-i"] in calls


async def _ws_session(url, handler, timeout=20.0):
    async with aiohttp.ClientSession() as s:
        async with s.ws_connect(url) as ws:
            return await asyncio.wait_for(handler(ws), timeout)


def test_live_resize_over_websocket():
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "WEBRTC_ENABLE_RESIZE": "true"})
    from mxdesk.server.app import serve

    async def handler(ws):
        configs, frames = [], []
        async for msg in ws:
            if msg.type == aiohttp.WSMsgType.TEXT:
                m = json.loads(msg.data)
                if m["type"] == "config":
                    configs.append(m)
                    if len(configs) == 1:
                        assert m["resize"] is True
                        await ws.send_str("r,643x250")
            elif msg.type == aiohttp.WSMsgType.BINARY:
                f = parse_frame(msg.data)
                frames.append((len(configs), f))
                if len(configs) == 2 and sum(1 for c, _ in frames if c == 2) >= 3:
                    return configs, frames

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await _ws_session(f"http://127.0.0.1:{port}/mxws", handler)
        finally:
            await runner.cleanup()

    configs, frames = asyncio.run(go())
    assert (configs[0]["width"], configs[0]["height"]) == (320, 96)
    assert (configs[1]["width"], configs[1]["height"]) == (640, 248) and configs[1]["codec"].startswith("avc1.")
    after = [f for c, f in frames if c == 2]
    assert after[0]["key"]  # the new session starts with an IDR
    stream = b"".join(f["au"] for f in after)
    assert (after[0]["width"], after[0]["height"]) == (640, 248)
    dec = Decoder().decode(stream)
    assert dec[0][0].shape == (248, 640)
    assert pipe.resizes == 1 and (srv.injector.w, srv.injector.h) == (640, 248)


def test_resize_ignored_when_disabled():
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    srv._on_client_message("r,640x480")
    assert pipe._pending_resize is None


def test_remote_clipboard_pushed_to_websocket_clients():
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    from mxdesk.server.app import serve

    async def handler(ws):
        await asyncio.sleep(0.3)  # past the baseline poll
        srv.injector.clipboard = "remote ünïcode"
        async for msg in ws:
            if msg.type == aiohttp.WSMsgType.TEXT:
                m = json.loads(msg.data)
                if m["type"] == "clipboard":
                    return base64.b64decode(m["data"]["content"]).decode()

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await _ws_session(f"http://127.0.0.1:{port}/mxws?media=0", handler)
        finally:
            await runner.cleanup()

    assert asyncio.run(go()) == "remote ünïcode"
    # the client's own paste is not echoed back
    srv._on_client_message('{"type": "clipboard", "text": "pasted"}')
    assert srv.clipboard.poll() is None and srv.injector.clipboard == "pasted"


def test_clipboard_direction_modes():
    from mxdesk.utils.config import clipboard_directions

    assert clipboard_directions("true") == (True, True) and clipboard_directions("False") == (False, False)
    assert clipboard_directions("in") == (True, False) and clipboard_directions("OUT") == (False, True)
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "SELKIES_ENABLE_CLIPBOARD": "out"})
    srv._on_client_message('{"type": "clipboard", "text": "blocked"}')
    assert srv.injector.clipboard == "" and srv.clipboard is not None and srv.clipboard_out
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "SELKIES_ENABLE_CLIPBOARD": "false"})
    assert srv.clipboard is None
    srv._on_client_message('{"type": "clipboard", "text": "blocked"}')
    assert srv.injector.clipboard == ""
