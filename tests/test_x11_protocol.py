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
