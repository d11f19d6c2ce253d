"""Remote -> client desktop state: clipboard and cursor image (selkies
``--enable_clipboard`` / ``--enable_cursors`` [UP], xclip and XFixes in the reference image,
Dockerfile:428-430).

* ``ClipboardSync`` keeps the remote clipboard and the browser's in step.  With a real X
  server it reads / writes the CLIPBOARD selection through ``xclip`` (what selkies uses);
  on the synthetic desktop the clipboard is the injector's text.  The remote side is polled
  and every change is pushed to the clients; text the client itself just sent is not echoed.
* ``CursorSync`` polls XFixesGetCursorImage through the capture object and turns every new
  cursor (by serial) into a PNG message, so the browser draws the cursor locally (no
  round-trip latency on pointer motion).

Both produce the selkies data-channel JSON shapes: ``{"type": "clipboard", "data":
{"content": <base64 utf-8>}}`` and ``{"type": "cursor", "data": {"curdata": <base64 png>,
"handle": serial, "hotspot": {"x", "y"}}}``; the same text goes on the ``/mxws`` control
WebSocket.
"""
from __future__ import annotations

import base64
import json
import logging
import os
import shutil
import subprocess
from typing import Any, Callable

from ..utils.png import encode_rgba

log = logging.getLogger("mxdesk.sync")


def clipboard_message(text: str) -> str:
    return json.dumps({"type": "clipboard", "data": {"content": base64.b64encode(text.encode()).decode()}})


def cursor_message(serial: int, xhot: int, yhot: int, rgba) -> str:
    png = base64.b64encode(encode_rgba(rgba)).decode()
    return json.dumps({"type": "cursor", "data": {"curdata": png, "handle": int(serial),
                                                  "hotspot": {"x": int(xhot), "y": int(yhot)}}})


class ClipboardSync:
    MAX_BYTES = 1 << 20

    def __init__(self, injector: Any, display: str | None = None, run: Callable = subprocess.run):
        self.injector = injector
        self.run = run
        self.display = display
        self.xclip = shutil.which("xclip") if display else None
        self.last: str | None = None  # last text known to both sides

    @property
    def mode(self) -> str:
        return "xclip" if self.xclip else "synthetic"

    def read(self) -> str | None:
        if self.xclip:
            try:
                r = self.run([self.xclip, "-selection", "clipboard", "-o"], capture_output=True, timeout=2,
                             env={**os.environ, "DISPLAY": self.display})
            except (OSError, subprocess.TimeoutExpired):
                return None
            if r.returncode != 0:
                return None  # empty selection / no owner
            return r.stdout[: self.MAX_BYTES].decode("utf-8", "replace")
        return getattr(self.injector, "clipboard", None)

    def write(self, text: str) -> None:
        """Client -> remote."""
        text = text[: self.MAX_BYTES]
        self.last = text
        if self.xclip:
            try:
                self.run([self.xclip, "-selection", "clipboard", "-i"], input=text.encode(), timeout=2,
                         env={**os.environ, "DISPLAY": self.display})
            except (OSError, subprocess.TimeoutExpired) as e:
                log.warning("xclip write failed: %s", e)
        elif hasattr(self.injector, "clipboard"):
            self.injector.clipboard = text

    def poll(self) -> str | None:
        """Remote -> client: the new clipboard text if it changed since the last poll."""
        cur = self.read()
        if self.last is None and cur is not None:  # first poll: baseline, nothing to push
            self.last = cur
            return None
        if cur is None or cur == self.last:
            return None
        self.last = cur
        return cur


class CursorSync:
    def __init__(self, capture: Any):
        self.capture = capture
        self.serial: int | None = None
        self.last_message: str | None = None

    def poll(self) -> str | None:
        img = self.capture.cursor_image() if hasattr(self.capture, "cursor_image") else None
        if img is None:
            return None
        serial, xhot, yhot, rgba = img
        if serial == self.serial or rgba.size == 0:
            return None
        self.serial = serial
        self.last_message = cursor_message(serial, xhot, yhot, rgba)
        return self.last_message
