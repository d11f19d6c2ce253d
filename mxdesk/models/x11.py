"""X11 MIT-SHM screen capture (replaces GStreamer ``ximagesrc`` with
``use-damage=0`` XShmGetImage capture in the reference's selkies pipeline).

libX11/libXext are loaded with ctypes (their development headers are not in the image);
the frame is grabbed with ``XShmGetImage`` into a SysV shared-memory segment -- zero copies
inside this process -- and returned as an (H, W, 4) BGRx numpy view that the GPU session
uploads from pinned memory (``Session.submit_bgrx``).  Falls back to ``XGetImage`` when the
MIT-SHM extension is unavailable (e.g. remote displays).

Damage-driven capture (``enable_damage``): the reference's ``ximagesrc`` runs with
``use-damage=0`` and copies the whole screen every frame (selkies pipeline,
``/root/reference/entrypoint.sh:110-131`` starts the X server it grabs from).  Here an XDamage
object on the root window accumulates the changed region; each tick subtracts it (before the
grab, so a change racing the grab is reported again next tick), turns its rectangles into a few
row bands, and ``XShmGetImage`` copies only those bands into the SHM segment.  The GPU session
DMAs the same bands into its device-resident screen (``Session.submit_bgrx_damage``), so a
static desktop costs neither X-server copies nor PCIe traffic.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import threading

import numpy as np

ZPixmap = 2
AllPlanes = ctypes.c_ulong(0xFFFFFFFFFFFFFFFF)
IPC_PRIVATE = 0
IPC_CREAT = 0o1000
IPC_RMID = 0


class XShmSegmentInfo(ctypes.Structure):
    _fields_ = [("shmseg", ctypes.c_ulong), ("shmid", ctypes.c_int), ("shmaddr", ctypes.c_void_p),
                ("readOnly", ctypes.c_int)]


class XImage(ctypes.Structure):  # leading fields of Xlib's XImage (x86_64 layout)
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("xoffset", ctypes.c_int),
                ("format", ctypes.c_int), ("data", ctypes.c_void_p), ("byte_order", ctypes.c_int),
                ("bitmap_unit", ctypes.c_int), ("bitmap_bit_order", ctypes.c_int), ("bitmap_pad", ctypes.c_int),
                ("depth", ctypes.c_int), ("bytes_per_line", ctypes.c_int), ("bits_per_pixel", ctypes.c_int)]


class XRectangle(ctypes.Structure):
    _fields_ = [("x", ctypes.c_short), ("y", ctypes.c_short), ("width", ctypes.c_ushort),
                ("height", ctypes.c_ushort)]


XDamageReportNonEmpty = 3  # one event when the damage goes from empty to non-empty


def rects_to_bands(rects, height: int, align: int = 16, max_gap: int = 32, max_bands: int = 16
                   ) -> list[tuple[int, int]]:
    """Damaged rectangles ``(x, y, w, h)`` -> sorted, disjoint row bands ``(y0, y1)``.

    Bands are widened to ``align``-row boundaries (macroblock rows: one DMA per band, and the
    encoder's rows change whole), bands closer than ``max_gap`` rows merge (a DMA costs more
    than a few extra rows), and while more than ``max_bands`` remain the closest pair merges."""
    iv = []
    for x, y, w, h in rects:
        if w <= 0 or h <= 0:
            continue
        y0 = max(0, int(y)) // align * align
        y1 = min(height, -(-(int(y) + int(h)) // align) * align)
        if y1 > y0:
            iv.append((y0, y1))
    iv.sort()
    out: list[list[int]] = []
    for y0, y1 in iv:
        if out and y0 - out[-1][1] < max_gap:
            out[-1][1] = max(out[-1][1], y1)
        else:
            out.append([y0, y1])
    while len(out) > max(1, max_bands):
        i = min(range(len(out) - 1), key=lambda j: out[j + 1][0] - out[j][1])
        out[i][1] = out[i + 1][1]
        del out[i + 1]
    return [(a, b) for a, b in out]


class DamageTracker:
    """XDamage on the root window (libXdamage + libXfixes through ctypes).  ``poll()`` returns
    the row bands changed since the previous poll; the first poll (and the one after
    ``invalidate()``) returns the whole screen."""

    def __init__(self, x11, dpy, root: int, height: int, xdamage=None, xfixes=None):
        self.x11, self.dpy, self.h = x11, dpy, int(height)
        xd = xdamage or ctypes.CDLL(ctypes.util.find_library("Xdamage") or "libXdamage.so.1")
        xf = xfixes or ctypes.CDLL(ctypes.util.find_library("Xfixes") or "libXfixes.so.3")
        ev, err = ctypes.c_int(0), ctypes.c_int(0)
        xd.XDamageQueryExtension.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_int)]
        if not xd.XDamageQueryExtension(dpy, ctypes.byref(ev), ctypes.byref(err)):
            raise OSError("no DAMAGE extension")
        xd.XDamageCreate.restype = ctypes.c_ulong
        xd.XDamageCreate.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int]
        xd.XDamageSubtract.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong]
        xd.XDamageDestroy.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
        xf.XFixesCreateRegion.restype = ctypes.c_ulong
        xf.XFixesCreateRegion.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        xf.XFixesFetchRegion.restype = ctypes.POINTER(XRectangle)
        xf.XFixesFetchRegion.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.POINTER(ctypes.c_int)]
        xf.XFixesDestroyRegion.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
        x11.XPending.argtypes = [ctypes.c_void_p]
        x11.XNextEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        x11.XFree.argtypes = [ctypes.c_void_p]
        self.xd, self.xf = xd, xf
        self.damage = xd.XDamageCreate(dpy, root, XDamageReportNonEmpty)
        self.region = xf.XFixesCreateRegion(dpy, None, 0)
        self._event = ctypes.create_string_buffer(192)  # sizeof(XEvent)
        self.full = True
        self.polls = 0
        self.rows_grabbed = 0

    def invalidate(self) -> None:
        self.full = True

    def resize(self, height: int) -> None:
        self.h = int(height)
        self.full = True

    def poll(self) -> list[tuple[int, int]]:
        while self.x11.XPending(self.dpy):  # the notify events only say "non-empty": drop them
            self.x11.XNextEvent(self.dpy, self._event)
        self.xd.XDamageSubtract(self.dpy, self.damage, 0, self.region)  # clear; region <- damage
        n = ctypes.c_int(0)
        r = self.xf.XFixesFetchRegion(self.dpy, self.region, ctypes.byref(n))
        rects = [(r[i].x, r[i].y, r[i].width, r[i].height) for i in range(n.value)] if r else []
        if r:
            self.x11.XFree(r)
        self.polls += 1
        if self.full:
            self.full = False
            bands = [(0, self.h)]
        else:
            bands = rects_to_bands(rects, self.h)
        self.rows_grabbed += sum(b - a for a, b in bands)
        return bands

    def close(self) -> None:
        self.xf.XFixesDestroyRegion(self.dpy, self.region)
        self.xd.XDamageDestroy(self.dpy, self.damage)


class XFixesCursorImage(ctypes.Structure):
    _fields_ = [("x", ctypes.c_short), ("y", ctypes.c_short), ("width", ctypes.c_ushort),
                ("height", ctypes.c_ushort), ("xhot", ctypes.c_ushort), ("yhot", ctypes.c_ushort),
                ("cursor_serial", ctypes.c_ulong), ("pixels", ctypes.POINTER(ctypes.c_ulong)),
                ("atom", ctypes.c_ulong), ("name", ctypes.c_char_p)]


def grab_bands(xext, dpy, root: int, img, shmaddr: int, pitch: int, bands) -> None:
    """``XShmGetImage`` of row bands into one full-frame SHM image: the image's height and
    data pointer are narrowed to the band (Xlib sends ``data - shmaddr`` as the segment
    offset), then restored."""
    c = img.contents
    full_h, full_data = c.height, c.data
    try:
        for y0, y1 in bands:
            c.height = int(y1 - y0)
            c.data = shmaddr + int(y0) * pitch
            if not xext.XShmGetImage(dpy, root, img, 0, int(y0), AllPlanes):
                raise OSError(f"XShmGetImage failed for rows [{y0}, {y1})")
    finally:
        c.height, c.data = full_h, full_data


def argb_longs_to_rgba(pixels: np.ndarray, width: int, height: int) -> np.ndarray:
    """XFixes cursor pixels (one premultiplied 0xAARRGGBB per ``unsigned long``) -> straight
    RGBA (H, W, 4) uint8, the layout a PNG cursor image needs."""
    p = np.asarray(pixels, np.uint64)[: width * height].astype(np.uint32).reshape(height, width)
    a = (p >> 24) & 0xFF
    rgb = np.stack([(p >> 16) & 0xFF, (p >> 8) & 0xFF, p & 0xFF], axis=-1).astype(np.uint32)
    nz = a > 0
    # un-premultiply (X cursors are premultiplied ARGB)
    rgb[nz] = np.minimum(255, (rgb[nz] * 255 + a[nz, None] // 2) // a[nz, None])
    return np.concatenate([rgb, a[..., None]], axis=-1).astype(np.uint8)


class X11Capture:
    def __init__(self, display: str = ":0", width: int | None = None, height: int | None = None):
        self.x11 = ctypes.CDLL(ctypes.util.find_library("X11") or "libX11.so.6")
        self.libc = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6", use_errno=True)
        x = self.x11
        x.XOpenDisplay.restype = ctypes.c_void_p
        x.XOpenDisplay.argtypes = [ctypes.c_char_p]
        x.XDefaultRootWindow.restype = ctypes.c_ulong
        x.XDefaultRootWindow.argtypes = [ctypes.c_void_p]
        x.XDefaultScreen.argtypes = [ctypes.c_void_p]
        x.XDisplayWidth.argtypes = [ctypes.c_void_p, ctypes.c_int]
        x.XDisplayHeight.argtypes = [ctypes.c_void_p, ctypes.c_int]
        x.XDefaultVisual.restype = ctypes.c_void_p
        x.XDefaultVisual.argtypes = [ctypes.c_void_p, ctypes.c_int]
        x.XDefaultDepth.argtypes = [ctypes.c_void_p, ctypes.c_int]
        x.XGetImage.restype = ctypes.POINTER(XImage)
        x.XGetImage.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int, ctypes.c_int, ctypes.c_uint,
                                ctypes.c_uint, ctypes.c_ulong, ctypes.c_int]
        x.XDestroyImage = getattr(x, "XDestroyImage", None)
        self.display_name = display
        # one connection shared by the pipeline thread and the RFB server's executor thread: Xlib
        # is not thread-safe (no XInitThreads), so every request sequence holds this lock
        self._lock = threading.RLock()
        self.dpy = x.XOpenDisplay(display.encode())
        if not self.dpy:
            raise OSError(f"cannot open X display {display}")
        scr = x.XDefaultScreen(self.dpy)
        self.root = x.XDefaultRootWindow(self.dpy)
        self.w = width or x.XDisplayWidth(self.dpy, scr)
        self.h = height or x.XDisplayHeight(self.dpy, scr)
        self.shm = None
        self.damage: DamageTracker | None = None
        try:
            self._init_shm(scr)
        except OSError:
            self.shm = None

    def enable_damage(self) -> bool:
        """Track XDamage on the root window so ``grab_shm_damage`` grabs only changed row
        bands; False (full-frame capture stays) without the DAMAGE extension or MIT-SHM."""
        if self.shm is None:
            return False
        try:
            with self._lock:
                self.damage = DamageTracker(self.x11, self.dpy, self.root, self.h)
        except (OSError, AttributeError):
            self.damage = None
        return self.damage is not None

    def _init_shm(self, scr: int) -> None:
        xext = ctypes.CDLL(ctypes.util.find_library("Xext") or "libXext.so.6")
        xext.XShmQueryExtension.argtypes = [ctypes.c_void_p]
        if not xext.XShmQueryExtension(self.dpy):
            raise OSError("no MIT-SHM")
        xext.XShmCreateImage.restype = ctypes.POINTER(XImage)
        xext.XShmCreateImage.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_int,
                                         ctypes.c_char_p, ctypes.POINTER(XShmSegmentInfo), ctypes.c_uint,
                                         ctypes.c_uint]
        xext.XShmAttach.argtypes = [ctypes.c_void_p, ctypes.POINTER(XShmSegmentInfo)]
        xext.XShmGetImage.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.POINTER(XImage), ctypes.c_int,
                                      ctypes.c_int, ctypes.c_ulong]
        self.xext = xext
        info = XShmSegmentInfo()
        vis = self.x11.XDefaultVisual(self.dpy, scr)
        depth = self.x11.XDefaultDepth(self.dpy, scr)
        img = xext.XShmCreateImage(self.dpy, vis, depth, ZPixmap, None, ctypes.byref(info), self.w, self.h)
        if not img:
            raise OSError("XShmCreateImage failed")
        size = img.contents.bytes_per_line * self.h
        self.libc.shmget.restype = ctypes.c_int
        self.libc.shmat.restype = ctypes.c_void_p
        self.libc.shmat.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        info.shmid = self.libc.shmget(IPC_PRIVATE, size, IPC_CREAT | 0o600)
        if info.shmid < 0:
            raise OSError("shmget failed")
        info.shmaddr = self.libc.shmat(info.shmid, None, 0)
        img.contents.data = info.shmaddr
        info.readOnly = 0
        if not xext.XShmAttach(self.dpy, ctypes.byref(info)):
            raise OSError("XShmAttach failed")
        self.libc.shmctl(info.shmid, IPC_RMID, None)  # freed when both sides detach
        self.shm = (info, img, size)
        self.view = np.ctypeslib.as_array(ctypes.cast(info.shmaddr, ctypes.POINTER(ctypes.c_uint8)), shape=(size,))
        self.pitch = img.contents.bytes_per_line

    def _release_shm(self) -> None:
        if self.shm is not None:
            info, img, _ = self.shm
            self.xext.XShmDetach.argtypes = [ctypes.c_void_p, ctypes.POINTER(XShmSegmentInfo)]
            self.xext.XShmDetach(self.dpy, ctypes.byref(info))
            self.x11.XSync.argtypes = [ctypes.c_void_p, ctypes.c_int]
            self.x11.XSync(self.dpy, 0)
            self.libc.shmdt.argtypes = [ctypes.c_void_p]
            self.libc.shmdt(info.shmaddr)
            self.shm = None

    def resize(self, width: int, height: int) -> None:
        """Re-create the capture image after the screen changed size (RandR resize)."""
        with self._lock:
            self._resize_locked(width, height)

    def _resize_locked(self, width: int, height: int) -> None:
        self._release_shm()
        self.w, self.h = int(width), int(height)
        try:
            self._init_shm(self.x11.XDefaultScreen(self.dpy))
        except OSError:
            self.shm = None
        if self.damage is not None:
            self.damage.resize(self.h)

    def cursor_image(self):
        """Current cursor as ``(serial, xhot, yhot, rgba)`` via XFixesGetCursorImage, or None
        when XFixes is unavailable (selkies' remote-cursor feature)."""
        if not hasattr(self, "_xfixes"):
            try:
                xf = ctypes.CDLL(ctypes.util.find_library("Xfixes") or "libXfixes.so.3")
                xf.XFixesGetCursorImage.restype = ctypes.POINTER(XFixesCursorImage)
                xf.XFixesGetCursorImage.argtypes = [ctypes.c_void_p]
                self.x11.XFree.argtypes = [ctypes.c_void_p]
                self._xfixes = xf
            except OSError:
                self._xfixes = None
        if self._xfixes is None:
            return None
        if not hasattr(self, "_cursor_dpy"):
            # own connection: Xlib is not thread-safe and grab() runs on the pipeline thread
            self._cursor_dpy = self.x11.XOpenDisplay(self.display_name.encode())
        if not self._cursor_dpy:
            return None
        ci = self._xfixes.XFixesGetCursorImage(self._cursor_dpy)
        if not ci:
            return None
        c = ci.contents
        n = c.width * c.height
        px = np.ctypeslib.as_array(c.pixels, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
        out = (int(c.cursor_serial), int(c.xhot), int(c.yhot), argb_longs_to_rgba(px, c.width, c.height))
        self.x11.XFree(ci)
        return out

    def shm_buffer(self) -> tuple[int, int] | None:
        """(address, size) of the MIT-SHM segment frames land in, or None (XGetImage path)."""
        if self.shm is None:
            return None
        info, _, size = self.shm
        return int(info.shmaddr), int(size)

    def grab_shm(self) -> tuple[int, int] | None:
        """Capture into the SHM segment without touching the pixels on the CPU: returns
        (address, row pitch in bytes) for Session.submit_bgrx_ptr, or None without SHM."""
        if self.shm is None:
            return None
        info, img, _ = self.shm
        with self._lock:
            if not self.xext.XShmGetImage(self.dpy, self.root, img, 0, 0, AllPlanes):
                raise OSError("XShmGetImage failed")
        return int(info.shmaddr), int(self.pitch)

    def grab_shm_damage(self) -> tuple[int, int, list[tuple[int, int]]] | None:
        """Damage-driven grab into the SHM segment: ``(address, pitch, bands)`` where only the
        row bands ``[y0, y1)`` were copied by the X server (the rest of the segment still holds
        the previous frame's pixels); None without SHM or damage tracking."""
        if self.shm is None or self.damage is None:
            return None
        info, img, _ = self.shm
        with self._lock:
            bands = self.damage.poll()  # subtract before grabbing: a racing change is re-reported
            grab_bands(self.xext, self.dpy, self.root, img, int(info.shmaddr), self.pitch, bands)
        return int(info.shmaddr), int(self.pitch), bands

    def grab(self) -> np.ndarray:
        """One frame as an (H, W, 4) uint8 BGRx array (a copy: the SHM segment is rewritten by
        the next grab, possibly from another thread).  It does not consume XDamage: a full grab
        only makes the segment newer, and the damage stays pending for ``grab_shm_damage``."""
        if self.shm is not None:
            info, img, size = self.shm
            with self._lock:
                if not self.xext.XShmGetImage(self.dpy, self.root, img, 0, 0, AllPlanes):
                    raise OSError("XShmGetImage failed")
                return self.view.reshape(self.h, self.pitch)[:, : self.w * 4].reshape(self.h, self.w, 4).copy()
        with self._lock:
            img = self.x11.XGetImage(self.dpy, self.root, 0, 0, self.w, self.h, AllPlanes, ZPixmap)
        if not img:
            raise OSError("XGetImage failed")
        bpl = img.contents.bytes_per_line
        buf = ctypes.string_at(img.contents.data, bpl * self.h)
        if self.x11.XDestroyImage is not None:
            pass  # XDestroyImage is a macro in Xlib; the image is leaked into Xlib's allocator
        return np.frombuffer(buf, np.uint8).reshape(self.h, bpl)[:, : self.w * 4].reshape(self.h, self.w, 4)
