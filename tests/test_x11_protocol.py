"""X11Capture (mxdesk/models/x11.py) against the real libX11 / libXext / libXdamage / libXfixes,
talking the X protocol to tests/fake_xserver.py: MIT-SHM capture into a SysV segment, XDamage
bands and the narrowed-image XShmGetImage of only those rows.  Skipped where the X client
libraries are missing."""
from __future__ import annotations

import ctypes.util

import numpy as np
import pytest

from mxdesk.models import x11 as X

pytestmark = pytest.mark.skipif(not (ctypes.util.find_library("X11") and ctypes.util.find_library("Xext")
                                     and ctypes.util.find_library("Xdamage") and ctypes.util.find_library("Xfixes")),
                                reason="X client libraries not installed")


@pytest.fixture
def xserver():
    from tests.fake_xserver import FakeXServer

    s = FakeXServer(320, 192)
    s.fb[:] = np.arange(320 * 4, dtype=np.uint32).astype(np.uint8).reshape(1, 320, 4)
    yield s
    s.close()


def test_shm_capture_full_frame(xserver):
    cap = X.X11Capture(xserver.display)
    assert (cap.w, cap.h) == (320, 192)
    assert cap.shm is not None and cap.pitch == 320 * 4
    img = cap.grab()
    assert img.shape == (192, 320, 4)
    assert np.array_equal(img, xserver.fb)
    addr, pitch = cap.grab_shm()
    assert (addr, pitch) == (cap.shm_buffer()[0], 320 * 4)


def test_damage_capture_grabs_only_changed_bands(xserver):
    cap = X.X11Capture(xserver.display)
    assert cap.enable_damage()
    addr, pitch, bands = cap.grab_shm_damage()
    assert bands == [(0, 192)]  # first grab: everything
    view = cap.view.reshape(192, pitch)[:, : 320 * 4].reshape(192, 320, 4)
    assert np.array_equal(view, xserver.fb)
    rows0 = xserver.getimage_rows

    # nothing drawn: no rows copied
    assert cap.grab_shm_damage()[2] == []
    assert xserver.getimage_rows == rows0

    # two small changes far apart -> two macroblock-row bands, only those rows copied
    xserver.draw(10, 37, 20, 5, 200)
    xserver.draw(100, 150, 8, 8, 17)
    _, _, bands = cap.grab_shm_damage()
    assert bands == [(32, 48), (144, 160)]
    assert xserver.getimage_rows - rows0 == 32
    assert np.array_equal(view, xserver.fb)  # the segment equals the screen again
    assert cap.damage.polls == 3

    # rows outside the bands are not rewritten: poison them in the segment, change one band
    view[0:16] = 0
    xserver.draw(0, 100, 320, 4, 99)
    assert cap.grab_shm_damage()[2] == [(96, 112)]
    assert np.array_equal(view[96:112], xserver.fb[96:112])
    assert not view[0:16].any()
    cap.damage.close()


def test_xtest_injection_reaches_the_server(xserver):
    """Browser input -> XTestInjector -> XTestFakeInput requests: absolute motion, button
    press / release, wheel clicks and a key looked up through the core keyboard map."""
    if not ctypes.util.find_library("Xtst"):
        pytest.skip("libXtst not installed")
    from mxdesk.server.input import InputEvent, XTestInjector

    inj = XTestInjector(xserver.display)
    inj.apply(InputEvent("mouse", x=100, y=50, buttons=1))
    inj.apply(InputEvent("mouse", x=101, y=52, buttons=0, scroll=1))
    inj.apply(InputEvent("key", keysym=0x61, down=True))
    inj.apply(InputEvent("key", keysym=0x61, down=False))
    inj.apply(InputEvent("key", keysym=0xFF0D, down=True))
    inj.x11.XSync.argtypes = [ctypes.c_void_p, ctypes.c_int]
    inj.x11.XSync(inj.dpy, 0)
    MOTION, BPRESS, BRELEASE, KPRESS, KRELEASE = 6, 4, 5, 2, 3
    assert xserver.fake_inputs == [
        (MOTION, 0, 100, 50), (BPRESS, 1, 0, 0),
        (MOTION, 0, 101, 52), (BRELEASE, 1, 0, 0), (BPRESS, 4, 0, 0), (BRELEASE, 4, 0, 0),
        (KPRESS, 38, 0, 0), (KRELEASE, 38, 0, 0), (KPRESS, 36, 0, 0)]


def test_cursor_image_through_xfixes(xserver):
    """X11Capture.cursor_image (remote cursors): XFixesGetCursorImage's premultiplied ARGB
    through libXfixes -> straight RGBA."""
    px = np.array([[0xFF102030, 0x80400000], [0x00000000, 0xFFFFFFFF]], np.uint32)
    xserver.cursor = (1, 0, 7, px)
    cap = X.X11Capture(xserver.display)
    serial, xhot, yhot, rgba = cap.cursor_image()
    assert (serial, xhot, yhot) == (7, 1, 0)
    assert rgba.shape == (2, 2, 4)
    assert rgba[0, 0].tolist() == [0x10, 0x20, 0x30, 255]
    assert rgba[0, 1].tolist() == [0x80, 0, 0, 0x80]  # un-premultiplied
    assert rgba[1, 0, 3] == 0 and rgba[1, 1].tolist() == [255, 255, 255, 255]


def test_serve_pipeline_captures_the_x_display(xserver):
    """`mxdesk serve` wiring with MXDESK_SOURCE=x11: build_pipeline opens the display, turns on
    XDamage (MXDESK_CAPTURE_DAMAGE) and the CPU encoder (x264enc) streams the X framebuffer."""
    from mxdesk.cli import build_pipeline
    from mxdesk.codec.h264_decoder import Decoder
    from mxdesk.models.synthetic import bgrx_to_nv12
    from mxdesk.utils import config as C

    yy, xx = np.mgrid[0:192, 0:320]
    xserver.fb[..., 0] = (xx * 255 // 320).astype(np.uint8)
    xserver.fb[..., 1] = (yy * 255 // 192).astype(np.uint8)
    xserver.fb[..., 2] = 90
    cfg = C.load(env={"ENABLE_BASIC_AUTH": "false", "SIZEW": "320", "SIZEH": "192", "DISPLAY": xserver.display,
                      "MXDESK_SOURCE": "x11", "WEBRTC_ENCODER": "x264enc"}, argv=[])
    pipe = build_pipeline(cfg)
    assert pipe.capture is not None and pipe.capture.damage is not None
    xserver.draw(0, 0, 64, 64, 250)
    stream = b"".join(pipe.step().au for _ in range(2))
    frames = Decoder().decode(stream)
    assert len(frames) == 2
    y_src, _ = bgrx_to_nv12(xserver.fb)
    err = frames[-1][0].astype(np.float64) - y_src.astype(np.float64)
    assert 10 * np.log10(255 ** 2 / max(1e-9, float((err ** 2).mean()))) > 30


def test_full_grab_from_another_thread_keeps_damage_pending(xserver):
    """The RFB server grabs whole frames from its executor thread on the same connection as
    the pipeline's damage polls: those grabs are serialised with the polls, return copies and
    never consume damage, so the video path still uploads every changed band."""
    import threading

    cap = X.X11Capture(xserver.display)
    assert cap.enable_damage()
    cap.grab_shm_damage()
    xserver.draw(0, 40, 50, 10, 123)
    stop = threading.Event()
    errors = []

    def rfb_like():
        try:
            while not stop.is_set():
                f = cap.grab()
                assert f.shape == (192, 320, 4)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    t = threading.Thread(target=rfb_like)
    t.start()
    try:
        f = cap.grab()
        assert np.array_equal(f, xserver.fb)
        assert not np.shares_memory(f, cap.view)  # a copy, not the live segment
        bands = []
        for _ in range(20):
            bands += cap.grab_shm_damage()[2]
    finally:
        stop.set()
        t.join()
    assert not errors
    assert bands == [(32, 64)]  # reported exactly once, to the damage path
