"""Client-driven display resize through RandR (the reference enables it
with ``WEBRTC_ENABLE_RESIZE``, Dockerfile:211, and selkies resizes the X screen with
``xcvt`` + ``xrandr`` [UP], Dockerfile:464).

``plan_resize`` is a pure function from ``xrandr --query`` output to the command list, so
the mode selection is unit-tested without an X server; ``resize_display`` runs it.  New
modes come from our own CVT reduced-blanking generator (``cvt.py``), the same one that
writes the initial ``xorg.conf`` modeline.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
from dataclasses import dataclass

from .cvt import cvt

MIN_W, MIN_H = 320, 240
MAX_W, MAX_H = 7680, 4320


def clamp_size(width: int, height: int) -> tuple[int, int]:
    """Sanitise a client-requested size: inside [320x240, 7680x4320] and a multiple of 8 in
    both directions (CVT cell granularity; even sizes keep 4:2:0 chroma whole)."""
    w = max(MIN_W, min(MAX_W, int(width))) // 8 * 8
    h = max(MIN_H, min(MAX_H, int(height))) // 8 * 8
    return w, h


@dataclass
class RandrOutput:
    name: str
    connected: bool
    modes: list[str]
    current: str | None


def parse_query(text: str) -> list[RandrOutput]:
    """Outputs and their mode names from ``xrandr --query``."""
    outs: list[RandrOutput] = []
    for line in text.splitlines():
        m = re.match(r"^(\S+) (connected|disconnected)\b", line)
        if m:
            outs.append(RandrOutput(m.group(1), m.group(2) == "connected", [], None))
            continue
        m = re.match(r"^\s+(\S+)\s+(.*)$", line)
        if m and outs and re.match(r"^\d+x\d+", m.group(1)):
            outs[-1].modes.append(m.group(1))
            if "*" in m.group(2):
                outs[-1].current = m.group(1)
    return outs


def plan_resize(query: str, width: int, height: int, refresh: float = 60.0) -> list[list[str]]:
    """xrandr argument lists that switch the first connected output to ``width x height``.
    An existing mode of that size is reused; otherwise a CVT-RB mode is created and added."""
    outs = parse_query(query)
    out = next((o for o in outs if o.connected), outs[0] if outs else None)
    if out is None:
        raise RuntimeError("xrandr reports no outputs")
    size = f"{width}x{height}"
    existing = next((m for m in out.modes if m == size or re.match(rf"^{size}(R|_|$)", m)), None)
    if existing is not None:
        if existing == out.current:
            return []
        return [["--output", out.name, "--mode", existing]]
    ml = cvt(width, height, refresh, reduced=True)
    name = ml.name
    timings = [f"{ml.clock_mhz:.2f}", *map(str, (ml.hdisplay, ml.hsync_start, ml.hsync_end, ml.htotal,
                                                  ml.vdisplay, ml.vsync_start, ml.vsync_end, ml.vtotal)),
               "+hsync" if ml.hsync_pos else "-hsync", "+vsync" if ml.vsync_pos else "-vsync"]
    return [["--newmode", name, *timings], ["--addmode", out.name, name], ["--output", out.name, "--mode", name]]


def resize_display(display: str, width: int, height: int, refresh: float = 60.0, run=subprocess.run) -> list[list[str]]:
    """Resize the X screen on ``display``; returns the xrandr commands that were run."""
    xrandr = shutil.which("xrandr")
    if xrandr is None:
        raise RuntimeError("xrandr not installed")
    env = {**os.environ, "DISPLAY": display}
    q = run([xrandr, "--query"], capture_output=True, text=True, env=env, timeout=10)
    if q.returncode != 0:
        raise RuntimeError(f"xrandr --query failed: {q.stderr.strip()}")
    cmds = plan_resize(q.stdout, width, height, refresh)
    for c in cmds:
        r = run([xrandr, *c], capture_output=True, text=True, env=env, timeout=10)
        if r.returncode != 0 and c[0] != "--newmode":  # the mode may already exist from an earlier resize
            raise RuntimeError(f"xrandr {' '.join(c)} failed: {r.stderr.strip()}")
    return cmds
