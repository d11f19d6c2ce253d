"""Damage-driven X11 capture (mxdesk/models/x11.py): rectangle -> row-band reduction, the
XDamage poll sequence and the banded XShmGetImage, against ctypes-level fakes of libXdamage /
libXfixes / libXext (there is no X server in the image; the GPU side is
tests/test_gpu_pipeline.py::test_damage_driven_capture_matches_full_upload)."""
from __future__ import annotations

import ctypes
from types import SimpleNamespace

import pytest

from mxdesk.models import x11 as X


def test_rects_to_bands_align_merge_clip():
    assert X.rects_to_bands([], 1080) == []
    assert X.rects_to_bands([(0, 0, 0, 5), (3, 4, 5, 0)], 1080) == []  # empty rectangles
    # one cursor-sized rectangle -> its macroblock rows
    assert X.rects_to_bands([(100, 37, 16, 16)], 1080) == [(32, 64)]
    # bands closer than max_gap merge, far ones stay apart; order-independent
    assert X.rects_to_bands([(0, 300, 9, 1), (0, 5, 10, 10), (0, 40, 3, 3)], 1080) == [(0, 48), (288, 304)]
    # clipped to the screen (negative y, past the bottom; 1080 is not a multiple of 16)
    assert X.rects_to_bands([(0, -8, 4, 20), (0, 1070, 4, 40)], 1080) == [(0, 16), (1056, 1080)]


def test_rects_to_bands_caps_band_count_by_merging_closest():
    rects = [(0, 100 * i, 4, 4) for i in range(10)]
    bands = X.rects_to_bands(rects, 1080, max_bands=4)
    assert len(bands) == 4
    covered = set()
    for a, b in bands:
        covered.update(range(a, b))
    assert all(y in covered for i in range(10) for y in range(100 * i, 100 * i + 4))
    assert all(b0[1] <= b1[0] for b0, b1 in zip(bands, bands[1:]))


def _fn(impl):
    def f(*a):
        return impl(*a)
    return f  # plain functions accept the argtypes / restype attributes the tracker sets


class FakeX:
    """Records the Xlib / XDamage / XFixes calls of one display connection."""

    def __init__(self, damage_supported=True):
        self.pending = 0
        self.region_rects: list[tuple[int, int, int, int]] = []
        self.calls: list[str] = []
        self.x11 = SimpleNamespace(XPending=_fn(lambda d: self.pending), XNextEvent=_fn(self._next),
                                   XFree=_fn(lambda p: self.calls.append("XFree")))
        self.xd = SimpleNamespace(
            XDamageQueryExtension=_fn(lambda d, ev, err: int(damage_supported)),
            XDamageCreate=_fn(lambda d, root, level: (self.calls.append(f"create:{level}"), 77)[1]),
            XDamageSubtract=_fn(self._subtract),
            XDamageDestroy=_fn(lambda d, dmg: self.calls.append("destroy")))
        self.xf = SimpleNamespace(XFixesCreateRegion=_fn(lambda d, r, n: 5), XFixesFetchRegion=_fn(self._fetch),
                                  XFixesDestroyRegion=_fn(lambda d, r: None))
        self._fetched: list[tuple[int, int, int, int]] = []

    def _next(self, d, ev):
        self.pending -= 1
        self.calls.append("event")

    def _subtract(self, d, damage, repair, parts):
        assert damage == 77 and repair == 0 and parts == 5
        self._fetched, self.region_rects = self.region_rects, []
        self.calls.append("subtract")

    def _fetch(self, d, region, n):
        rects = self._fetched
        ctypes.cast(n, ctypes.POINTER(ctypes.c_int))[0] = len(rects)
        if not rects:
            return None
        return (X.XRectangle * len(rects))(*[X.XRectangle(x, y, w, h) for x, y, w, h in rects])

    def tracker(self, height=1080):
        return X.DamageTracker(self.x11, 1, 2, height, xdamage=self.xd, xfixes=self.xf)


def test_damage_tracker_poll_sequence():
    fx = FakeX()
    t = fx.tracker()
    assert f"create:{X.XDamageReportNonEmpty}" in fx.calls
    fx.region_rects = [(0, 0, 10, 10)]
    assert t.poll() == [(0, 1080)]  # first poll: the whole screen (segment starts empty)
    assert t.poll() == []  # nothing changed since
    fx.pending = 3
    fx.region_rects = [(500, 200, 30, 20), (0, 1000, 1920, 80)]
    assert t.poll() == [(192, 224), (992, 1080)]
    assert fx.pending == 0 and fx.calls.count("event") == 3  # notify events drained
    t.invalidate()
    assert t.poll() == [(0, 1080)]
    t.resize(720)
    assert t.poll() == [(0, 720)]
    assert t.rows_grabbed == 1080 + 32 + 88 + 1080 + 720
    t.close()
    assert "destroy" in fx.calls


def test_damage_tracker_without_extension():
    with pytest.raises(OSError):
        FakeX(damage_supported=False).tracker()


def test_grab_bands_narrows_and_restores_the_image():
    pitch, h = 64 * 4 + 32, 96
    img = ctypes.pointer(X.XImage(width=64, height=h, data=0x10000, bytes_per_line=pitch))
    seen = []

    def get_image(dpy, root, im, x, y, planes):
        c = im.contents
        seen.append((x, y, c.height, c.data - 0x10000))
        return 1

    xext = SimpleNamespace(XShmGetImage=get_image)
    X.grab_bands(xext, 1, 2, img, 0x10000, pitch, [(0, 16), (48, 96)])
    assert seen == [(0, 0, 16, 0), (0, 48, 48, 48 * pitch)]
    assert img.contents.height == h and img.contents.data == 0x10000
    xext.XShmGetImage = lambda *a: 0
    with pytest.raises(OSError):
        X.grab_bands(xext, 1, 2, img, 0x10000, pitch, [(16, 32)])
    assert img.contents.height == h and img.contents.data == 0x10000  # restored on failure too


def test_capture_damage_grab_and_pipeline_fallbacks():
    """X11Capture.grab_shm_damage returns (addr, pitch, bands); without SHM enable_damage is
    False and the pipeline keeps the full-frame path."""
    import threading

    cap = X.X11Capture.__new__(X.X11Capture)
    cap.shm, cap.damage, cap._lock = None, None, threading.RLock()
    assert cap.enable_damage() is False and cap.grab_shm_damage() is None
    fx = FakeX()
    cap.damage = fx.tracker(96)
    pitch = 64 * 4
    info = X.XShmSegmentInfo(shmaddr=0x20000)
    img = ctypes.pointer(X.XImage(width=64, height=96, data=0x20000, bytes_per_line=pitch))
    grabbed = []
    cap.shm, cap.pitch, cap.dpy, cap.root = (info, img, pitch * 96), pitch, 1, 2
    cap.xext = SimpleNamespace(XShmGetImage=lambda d, r, im, x, y, p: grabbed.append((y, im.contents.height)) or 1)
    assert cap.grab_shm_damage() == (0x20000, pitch, [(0, 96)])
    fx.region_rects = [(3, 70, 2, 2)]
    assert cap.grab_shm_damage() == (0x20000, pitch, [(64, 80)])
    assert grabbed == [(0, 96), (64, 16)]


def test_idle_skip_policy(monkeypatch):
    """Damage-driven frame rate: production pauses after `idle_after` frames without damage and
    resumes on damage, a cursor move, a key-frame request or the heartbeat."""
    from mxdesk.pipeline import stream as S

    now = [100.0]
    monkeypatch.setattr(S.time, "monotonic", lambda: now[0])
    from mxdesk.utils.metrics import SessionMetrics

    p = S.StreamPipeline.__new__(S.StreamPipeline)
    p.metrics = SessionMetrics("t")
    p.idle_after, p.idle_heartbeat_s, p.frames_idle = 3, 1.0, 0
    p._static_frames, p._cursor, p._last_produced_t = 0, (-1, -1), 100.0
    p._idle_cursor = p._cursor
    assert [p._idle_skip([], False) for _ in range(5)] == [False, False, False, True, True]
    assert p.frames_idle == 2
    assert p.metrics.idle.labels("t")._value.get() == 2  # /metrics mxdesk_idle_frames_total
    assert p._idle_skip([(0, 16)], False) is False  # damage resumes at once
    assert [p._idle_skip([], False) for _ in range(4)] == [False, False, False, True]
    assert p._idle_skip([], True) is False  # a key frame is always produced
    p._static_frames = 10
    p._cursor = (5, 5)
    assert p._idle_skip([], False) is False  # the cursor moved (it is drawn into the picture)
    p._static_frames = 10
    now[0] = 101.5  # heartbeat: one frame per idle_heartbeat_s
    assert p._idle_skip([], False) is False
    p.idle_after = 0  # disabled
    now[0] = 100.2
    p._static_frames = 50
    assert p._idle_skip([], False) is False
