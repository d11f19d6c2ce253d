"""X11 MIT-SHM screen capture (replaces GStreamer ``ximagesrc`` with
``use-damage=0`` XShmGetImage capture in the reference's selkies pipeline).

libX11/libXext are loaded with ctypes (their development headers are not in the image);
the frame is grabbed with ``XShmGetImage`` into a SysV shared-memory segment -- zero copies
inside this process -- and returned as an (H, W, 4) BGRx numpy view that the GPU session
uploads from pinned memory (``Session.submit_bgrx``).  Falls back to ``XGetImage`` when the
MIT-SHM extension is unavailable (e.g. remote displays).
"""
from __future__ import annotations

import ctypes
import ctypes.util

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


class XFixesCursorImage(ctypes.Structure):
    _fields_ = [("x", ctypes.c_short), ("y", ctypes.c_short), ("width", ctypes.c_ushort),
                ("height", ctypes.c_ushort), ("xhot", ctypes.c_ushort), ("yhot", ctypes.c_ushort),
                ("cursor_serial", ctypes.c_ulong), ("pixels", ctypes.POINTER(ctypes.c_ulong)),
                ("atom", ctypes.c_ulong), ("name", ctypes.c_char_p)]


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
        self.dpy = x.XOpenDisplay(display.encode())
        if not self.dpy:
            raise OSError(f"cannot open X display {display}")
        scr = x.XDefaultScreen(self.dpy)
        self.root = x.XDefaultRootWindow(self.dpy)
        self.w = width or x.XDisplayWidth(self.dpy, scr)
        self.h = height or x.XDisplayHeight(self.dpy, scr)
        self.shm = None
        try:
            self._init_shm(scr)
        except OSError:
            self.shm = None

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
        self._release_shm()
        self.w, self.h = int(width), int(height)
        try:
            self._init_shm(self.x11.XDefaultScreen(self.dpy))
        except OSError:
            self.shm = None

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
        if not self.xext.XShmGetImage(self.dpy, self.root, img, 0, 0, AllPlanes):
            raise OSError("XShmGetImage failed")
        return int(info.shmaddr), int(self.pitch)

    def grab(self) -> np.ndarray:
        """One frame as an (H, W, 4) uint8 BGRx array."""
        if self.shm is not None:
            info, img, size = self.shm
            if not self.xext.XShmGetImage(self.dpy, self.root, img, 0, 0, AllPlanes):
                raise OSError("XShmGetImage failed")
            return self.view.reshape(self.h, self.pitch)[:, : self.w * 4].reshape(self.h, self.w, 4)
        img = self.x11.XGetImage(self.dpy, self.root, 0, 0, self.w, self.h, AllPlanes, ZPixmap)
        if not img:
            raise OSError("XGetImage failed")
        bpl = img.contents.bytes_per_line
        buf = ctypes.string_at(img.contents.data, bpl * self.h)
        if self.x11.XDestroyImage is not None:
            pass  # XDestroyImage is a macro in Xlib; the image is leaked into Xlib's allocator
        return np.frombuffer(buf, np.uint8).reshape(self.h, bpl)[:, : self.w * 4].reshape(self.h, self.w, 4)
