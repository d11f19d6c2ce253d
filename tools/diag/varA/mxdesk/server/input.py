"""Remote input, clipboard and resize handling.

Accepts both mxdesk JSON messages (``{"type": "mouse", ...}``) and the selkies data-channel
text protocol [UP] (``m,x,y,mask,scroll`` / ``m2,dx,dy,mask,scroll`` / ``kd,keysym`` /
``ku,keysym`` / ``kr`` / ``cw,<base64>`` / ``r,WxH`` / ``vb,kbps`` / ``_f,fps`` /
``js,c|d|b|a,...`` gamepads) and turns them into injector / gamepad-server calls.

Injectors:
  * ``SyntheticInjector`` drives the synthetic desktop (remote cursor position; keys and
    clipboard are recorded) -- used on the GPU box, which has no X server;
  * ``XTestInjector`` injects into a real X server through libXtst/libX11 loaded with
    ctypes (the reference uses xdotool/XTest, Dockerfile:428-430); only constructed when
    ``DISPLAY`` has a server.
"""
from __future__ import annotations

import base64
import ctypes
import ctypes.util
import json
import logging
from dataclasses import dataclass, field
from typing import Any

log = logging.getLogger("mxdesk.input")


@dataclass
class InputEvent:
    kind: str                  # mouse | key | keyreset | clipboard | resize | bitrate | fps | pli | ack | stats
    x: int = 0
    y: int = 0
    buttons: int = 0
    scroll: int = 0
    relative: bool = False
    keysym: int = 0
    down: bool = False
    text: str = ""
    width: int = 0
    height: int = 0
    value: float = 0.0
    extra: dict = field(default_factory=dict)


def parse_message(msg: str) -> InputEvent | None:
    msg = msg.strip()
    if not msg:
        return None
    if msg.startswith("{"):
        d = json.loads(msg)
        t = d.get("type")
        if t == "mouse":
            return InputEvent("mouse", int(d.get("x", 0)), int(d.get("y", 0)), int(d.get("buttons", 0)),
                              int(d.get("scroll", 0)), bool(d.get("relative", False)))
        if t == "key":
            return InputEvent("key", keysym=int(d["keysym"]), down=bool(d.get("down", True)))
        if t == "clipboard":
            return InputEvent("clipboard", text=str(d.get("text", "")))
        if t == "resize":
            return InputEvent("resize", width=int(d["width"]), height=int(d["height"]))
        if t == "bitrate":
            return InputEvent("bitrate", value=float(d["kbps"]))
        if t in ("pli", "keyframe"):
            return InputEvent("pli")
        if t == "ack":
            return InputEvent("ack", extra=d)
        if t == "stats":
            return InputEvent("stats", extra=d)
        return InputEvent(str(t), extra=d)
    parts = msg.split(",")
    op = parts[0]
    try:
        if op in ("m", "m2"):
            return InputEvent("mouse", int(float(parts[1])), int(float(parts[2])), int(parts[3]) if len(parts) > 3 else 0,
                              int(parts[4]) if len(parts) > 4 else 0, relative=(op == "m2"))
        if op in ("kd", "ku"):
            return InputEvent("key", keysym=int(parts[1]), down=(op == "kd"))
        if op == "kr":
            return InputEvent("keyreset")
        if op == "cw":
            return InputEvent("clipboard", text=base64.b64decode(parts[1]).decode("utf-8", "replace"))
        if op == "r":
            w, h = parts[1].lower().split("x")
            return InputEvent("resize", width=int(w), height=int(h))
        if op == "vb":
            return InputEvent("bitrate", value=float(parts[1]))
        if op == "_f":
            return InputEvent("fps", value=float(parts[1]))
        if op == "pli":
            return InputEvent("pli")
        if op == "js":
            sub, idx = parts[1], int(parts[2])
            if sub == "c":
                name = base64.b64decode(parts[3]).decode("utf-8", "replace") if len(parts) > 3 else ""
                return InputEvent("gamepad", extra={"op": "c", "idx": idx, "name": name,
                                                    "axes": int(parts[4]) if len(parts) > 4 else 4,
                                                    "buttons": int(parts[5]) if len(parts) > 5 else 17})
            if sub == "d":
                return InputEvent("gamepad", extra={"op": "d", "idx": idx})
            if sub in ("b", "a"):
                return InputEvent("gamepad", extra={"op": sub, "idx": idx, "num": int(parts[3]),
                                                    "value": float(parts[4])})
            return None
    except (IndexError, ValueError) as e:
        log.debug("bad input message %r: %s", msg, e)
        return None
    return None


class SyntheticInjector:
    """Input sink for the synthetic desktop: moves the rendered remote cursor."""

    def __init__(self, pipeline: Any, width: int, height: int):
        self.pipeline = pipeline
        self.w, self.h = width, height
        self.x, self.y = width // 2, height // 2
        self.buttons = 0
        self.keys_down: set[int] = set()
        self.clipboard = ""
        self.events = 0

    def apply(self, ev: InputEvent) -> None:
        self.events += 1
        if ev.kind == "mouse":
            if ev.relative:
                self.x, self.y = self.x + ev.x, self.y + ev.y
            else:
                self.x, self.y = ev.x, ev.y
            self.x = max(0, min(self.w - 1, self.x))
            self.y = max(0, min(self.h - 1, self.y))
            self.buttons = ev.buttons
            self.pipeline.set_cursor(self.x, self.y)
        elif ev.kind == "key":
            (self.keys_down.add if ev.down else self.keys_down.discard)(ev.keysym)
        elif ev.kind == "keyreset":
            self.keys_down.clear()
        elif ev.kind == "clipboard":
            self.clipboard = ev.text


class XTestInjector:
    """XTest injection into a real X server via ctypes (libX11 + libXtst)."""

    def __init__(self, display: str = ":0"):
        x11 = ctypes.util.find_library("X11")
        xtst = ctypes.util.find_library("Xtst")
        if not x11 or not xtst:
            raise OSError("libX11/libXtst not found")
        self.x11 = ctypes.CDLL(x11)
        self.xtst = ctypes.CDLL(xtst)
        self.x11.XOpenDisplay.restype = ctypes.c_void_p
        self.x11.XOpenDisplay.argtypes = [ctypes.c_char_p]
        self.dpy = self.x11.XOpenDisplay(display.encode())
        if not self.dpy:
            raise OSError(f"cannot open X display {display}")
        self.x11.XKeysymToKeycode.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
        self.x11.XFlush.argtypes = [ctypes.c_void_p]
        vp, i, u, ul = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_ulong
        self.xtst.XTestFakeMotionEvent.argtypes = [vp, i, i, i, ul]
        self.xtst.XTestFakeRelativeMotionEvent.argtypes = [vp, i, i, ul]
        self.xtst.XTestFakeButtonEvent.argtypes = [vp, u, i, ul]
        self.xtst.XTestFakeKeyEvent.argtypes = [vp, u, i, ul]
        self.buttons = 0

    def apply(self, ev: InputEvent) -> None:
        if ev.kind == "mouse":
            if ev.relative:
                self.xtst.XTestFakeRelativeMotionEvent(self.dpy, ev.x, ev.y, 0)
            else:
                self.xtst.XTestFakeMotionEvent(self.dpy, -1, ev.x, ev.y, 0)
            changed = self.buttons ^ ev.buttons
            for b in range(5):
                if changed & (1 << b):
                    self.xtst.XTestFakeButtonEvent(self.dpy, b + 1, 1 if ev.buttons & (1 << b) else 0, 0)
            self.buttons = ev.buttons
            if ev.scroll:
                btn = 4 if ev.scroll > 0 else 5
                for _ in range(min(abs(ev.scroll), 10)):
                    self.xtst.XTestFakeButtonEvent(self.dpy, btn, 1, 0)
                    self.xtst.XTestFakeButtonEvent(self.dpy, btn, 0, 0)
        elif ev.kind == "key":
            kc = self.x11.XKeysymToKeycode(self.dpy, ev.keysym)
            if kc:
                self.xtst.XTestFakeKeyEvent(self.dpy, kc, 1 if ev.down else 0, 0)
        self.x11.XFlush(self.dpy)
