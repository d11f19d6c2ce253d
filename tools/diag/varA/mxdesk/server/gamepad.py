"""Browser gamepads -> Linux joystick API for apps in the desktop.

The reference preloads selkies' ``joystick_interposer.so`` (Dockerfile:473-476,
``SDL_JOYSTICK_DEVICE=/dev/input/js0``) and feeds it from the WebRTC data channel.  Here
``csrc/interposer/js_interposer.c`` (built as ``mxdesk/libmxjs_interposer.so``) redirects
``open("/dev/input/jsN")`` to the unix socket ``$MXDESK_JS_DIR/mxdesk_jsN.sock`` served by
this module: one config record, then ``struct js_event`` records (``<IhBB``: time ms, value,
type, number) built from the browser's Gamepad API messages.

Browser protocol (text, over /mxws):
  ``js,c,<idx>,<base64 name>,<num_axes>,<num_buttons>``  gamepad connected
  ``js,d,<idx>``                                         disconnected
  ``js,b,<idx>,<button>,<value 0..1>``                   button
  ``js,a,<idx>,<axis>,<value -1..1>``                    axis
"""
from __future__ import annotations

import asyncio
import logging
import os
import struct
import time
from pathlib import Path

log = logging.getLogger("mxdesk.gamepad")

MAX_PADS = 4
NAME_LEN = 128
KEY_MAX, BTN_MISC, ABS_CNT = 0x2FF, 0x100, 64
JS_EVENT_BUTTON, JS_EVENT_AXIS, JS_EVENT_INIT = 0x01, 0x02, 0x80
# W3C "standard" gamepad mapping -> Linux input codes
STD_BUTTONS = [0x130, 0x131, 0x133, 0x134, 0x136, 0x137, 0x138, 0x139, 0x13A, 0x13B, 0x13D, 0x13E,
               0x220, 0x221, 0x222, 0x223, 0x13C]
STD_AXES = [0x00, 0x01, 0x03, 0x04, 0x02, 0x05, 0x10, 0x11]


def config_record(name: str, num_axes: int, num_buttons: int) -> bytes:
    """Packed ``struct mx_js_config`` (js_interposer.c)."""
    nb = name.encode("utf-8", "replace")[:NAME_LEN - 1]
    btn = [STD_BUTTONS[i] if i < len(STD_BUTTONS) else 0x120 + i for i in range(num_buttons)]
    btn += [0] * (KEY_MAX - BTN_MISC + 1 - len(btn))
    axes = [STD_AXES[i] if i < len(STD_AXES) else 0x06 + i for i in range(num_axes)]
    axes += [0] * (ABS_CNT - len(axes))
    return (nb.ljust(NAME_LEN, b"\0") + struct.pack("<HBB", num_buttons, num_axes, 0)
            + struct.pack(f"<{len(btn)}H", *btn) + bytes(axes))


def js_event(etype: int, number: int, value: int, t_ms: int | None = None) -> bytes:
    t = int(time.monotonic() * 1000) if t_ms is None else t_ms
    return struct.pack("<IhBB", t & 0xFFFFFFFF, max(-32767, min(32767, value)), etype, number)


class _Pad:
    def __init__(self, idx: int):
        self.idx = idx
        self.name = "mxdesk virtual gamepad"
        self.axes = [0] * 8
        self.buttons = [0] * 17
        self.connected = False
        self.writers: set[asyncio.StreamWriter] = set()


class GamepadServer:
    def __init__(self, sock_dir: str | os.PathLike | None = None, max_pads: int = MAX_PADS):
        self.dir = Path(sock_dir or os.environ.get("MXDESK_JS_DIR", "/tmp"))
        self.pads = [_Pad(i) for i in range(max_pads)]
        self.servers: list[asyncio.AbstractServer] = []

    def sock_path(self, idx: int) -> Path:
        return self.dir / f"mxdesk_js{idx}.sock"

    async def start(self) -> None:
        self.dir.mkdir(parents=True, exist_ok=True)
        for pad in self.pads:
            p = self.sock_path(pad.idx)
            p.unlink(missing_ok=True)
            srv = await asyncio.start_unix_server(lambda r, w, pad=pad: self._client(pad, r, w), path=str(p))
            self.servers.append(srv)

    async def stop(self) -> None:
        for s in self.servers:
            s.close()
        for pad in self.pads:
            for w in list(pad.writers):
                w.close()
            self.sock_path(pad.idx).unlink(missing_ok=True)
        self.servers.clear()

    async def _client(self, pad: _Pad, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        writer.write(config_record(pad.name, len(pad.axes), len(pad.buttons)))
        # initial state, like the kernel joydev driver (JS_EVENT_INIT)
        for i, v in enumerate(pad.buttons):
            writer.write(js_event(JS_EVENT_BUTTON | JS_EVENT_INIT, i, v))
        for i, v in enumerate(pad.axes):
            writer.write(js_event(JS_EVENT_AXIS | JS_EVENT_INIT, i, v))
        pad.writers.add(writer)
        try:
            await writer.drain()
            await reader.read()  # apps never write; returns at EOF (app closed the device)
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:
            pad.writers.discard(writer)
            writer.close()

    def _send(self, pad: _Pad, data: bytes) -> None:
        for w in list(pad.writers):
            try:
                w.write(data)
            except (ConnectionError, RuntimeError):
                pad.writers.discard(w)

    def apply(self, ev) -> None:
        """Apply a parsed ``gamepad`` InputEvent (see input.parse_message)."""
        d = ev.extra
        if not 0 <= d.get("idx", -1) < len(self.pads):
            return
        pad = self.pads[d["idx"]]
        op = d["op"]
        if op == "c":
            pad.name = d.get("name") or pad.name
            pad.axes = [0] * max(0, min(ABS_CNT, d.get("axes", 4)))
            pad.buttons = [0] * max(0, min(KEY_MAX - BTN_MISC + 1, d.get("buttons", 17)))
            pad.connected = True
        elif op == "d":
            pad.connected = False
            for i, v in enumerate(pad.buttons):
                if v:
                    pad.buttons[i] = 0
                    self._send(pad, js_event(JS_EVENT_BUTTON, i, 0))
            for i, v in enumerate(pad.axes):
                if v:
                    pad.axes[i] = 0
                    self._send(pad, js_event(JS_EVENT_AXIS, i, 0))
        elif op == "b" and 0 <= d["num"] < len(pad.buttons):
            v = 1 if d["value"] >= 0.5 else 0
            if pad.buttons[d["num"]] != v:
                pad.buttons[d["num"]] = v
                self._send(pad, js_event(JS_EVENT_BUTTON, d["num"], v))
        elif op == "a" and 0 <= d["num"] < len(pad.axes):
            v = int(round(max(-1.0, min(1.0, d["value"])) * 32767))
            if pad.axes[d["num"]] != v:
                pad.axes[d["num"]] = v
                self._send(pad, js_event(JS_EVENT_AXIS, d["num"], v))


def interposer_path() -> Path:
    """The built interposer library (``python -c "from mxdesk import _build; _build.build()"``)."""
    return Path(__file__).resolve().parents[1] / "libmxjs_interposer.so"
