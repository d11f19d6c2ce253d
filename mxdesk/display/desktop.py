"""Display-session bring-up: the MI355X replacement of the reference's ``entrypoint.sh``
(call stack §3.1).

Reference behaviour and what changes:

* pre-flight (entrypoint.sh:9-29): XDG runtime dir 0700, stale X locks removed.  The
  reference runs ``rm -rf /tmp/.X*`` unconditionally, which deletes the lock of a LIVE
  server when the program is restarted; here a lock is removed only when its
  PID is dead.
* NVIDIA userspace driver download (entrypoint.sh:31-55): not needed -- ROCm userspace is in
  the image and talks to the host amdgpu/KFD driver directly.
* GPU selection + BusID (entrypoint.sh:70-98): ``utils.devices`` (sysfs/KFD).
* xorg.conf + Xwrapper (entrypoint.sh:57-108): ``display.xorg``.
* ``Xorg ... &`` then poll the socket (entrypoint.sh:113-118): same, but the X server is
  *waited on*: if it dies this process exits non-zero so the supervisor restarts the whole
  display session (the reference backgrounds Xorg and never notices a crash, §5.2).
* desktop + IME (entrypoint.sh:128-131): ``MXDESK_DESKTOP_CMD`` (default KDE Plasma when
  installed), ``fcitx`` when installed; both in the session's process group.
"""
from __future__ import annotations

import logging
import os
import shlex
import shutil
import signal
import subprocess
import sys
import time
from pathlib import Path

from . import xorg as X

log = logging.getLogger("mxdesk.desktop")


def pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


def clean_stale_locks(display: str, tmp: str = "/tmp") -> list[str]:
    """Remove ``/tmp/.X<n>-lock`` and the socket of display ``n`` only if the owning PID is
    gone.  Returns the removed paths."""
    n = display.lstrip(":").split(".")[0]
    lock = Path(tmp) / f".X{n}-lock"
    sock = Path(tmp) / ".X11-unix" / f"X{n}"
    removed: list[str] = []
    if lock.exists():
        try:
            pid = int(lock.read_text().strip() or "0")
        except (ValueError, OSError):
            pid = 0
        if pid > 0 and pid_alive(pid):
            return removed  # live server: leave everything alone
        lock.unlink(missing_ok=True)
        removed.append(str(lock))
    if sock.exists():
        sock.unlink(missing_ok=True)
        removed.append(str(sock))
    return removed


def preflight(runtime_dir: str | None = None) -> str:
    rd = runtime_dir or os.environ.get("XDG_RUNTIME_DIR") or f"/tmp/runtime-{os.getuid()}"
    Path(rd).mkdir(parents=True, exist_ok=True)
    os.chmod(rd, 0o700)
    os.environ["XDG_RUNTIME_DIR"] = rd
    return rd


def joystick_placeholders(dev_input: str = "/dev/input", n: int = 4) -> list[str]:
    """Create empty /dev/input/js0..3 so apps that scan the directory find joysticks; the
    interposer redirects the actual open() (reference selkies-gstreamer-entrypoint.sh:15).
    Best effort: needs write access to /dev/input (root or a 1777 dir)."""
    made = []
    try:
        Path(dev_input).mkdir(parents=True, exist_ok=True)
        for i in range(n):
            p = Path(dev_input) / f"js{i}"
            if not p.exists():
                p.touch()
                made.append(str(p))
    except OSError as e:
        log.info("joystick placeholders not created (%s)", e)
    return made


# GL userspace hygiene for the desktop's clients (reference Dockerfile:196 sets NVIDIA's
# __GL_SYNC_TO_VBLANK=0): Mesa's equivalent is vblank_mode=0 -- a virtual display has no
# vblank to wait for, and a synced swap would cap every GL client at the dummy refresh.
GL_ENV = {"vblank_mode": "0", "__GL_SYNC_TO_VBLANK": "0", "KWIN_X11_NO_SYNC_TO_VBLANK": "1"}


def desktop_env(env: dict | None = None) -> dict:
    """Environment for the desktop session: GL_ENV unless already set by the user."""
    out = dict(os.environ if env is None else env)
    for k, v in GL_ENV.items():
        out.setdefault(k, v)
    return out


def icd_report(opencl_dirs=("/etc/OpenCL/vendors",),
               vulkan_dirs=("/usr/share/vulkan/icd.d", "/etc/vulkan/icd.d")) -> dict:
    """Registered OpenCL / Vulkan ICDs (reference Dockerfile:170-187 provisions NVIDIA's):
    {"opencl": [(file, library)], "vulkan": [(file, library_path)]}.  On MI355X the ROCm
    OpenCL ICD (libamdocl64.so) is the expected OpenCL entry; Vulkan has no CDNA driver, so
    only software ICDs (lavapipe) can appear."""
    import json

    rep: dict = {"opencl": [], "vulkan": []}
    for d in opencl_dirs:
        for f in sorted(Path(d).glob("*.icd")) if Path(d).is_dir() else []:
            try:
                rep["opencl"].append((str(f), f.read_text().strip()))
            except OSError:
                continue
    for d in vulkan_dirs:
        for f in sorted(Path(d).glob("*.json")) if Path(d).is_dir() else []:
            try:
                lib = json.loads(f.read_text()).get("ICD", {}).get("library_path", "")
            except (OSError, ValueError):
                continue
            rep["vulkan"].append((str(f), lib))
    return rep


def desktop_command(env: dict | None = None) -> list[str]:
    env = os.environ if env is None else env
    cmd = env.get("MXDESK_DESKTOP_CMD")
    if cmd:
        return shlex.split(cmd)
    if shutil.which("startplasma-x11"):
        return (["dbus-launch"] if shutil.which("dbus-launch") else []) + ["startplasma-x11"]
    for fallback in ("xfce4-session", "openbox-session", "xterm"):
        if shutil.which(fallback):
            return [fallback]
    return []


def run_display_session(cfg, conf_dir: str = "/tmp/mxdesk-x") -> int:
    """Bring up X + desktop and block until the X server exits; returns its exit code."""
    from ..utils import devices as D

    preflight()
    joystick_placeholders()
    removed = clean_stale_locks(cfg.display)
    if removed:
        log.info("removed stale X files: %s", removed)
    busid, driver = "", "dummy"
    gpus = D.visible_gpus(D.enumerate_gpus())
    if gpus:
        g = D.select_gpu(gpus, cfg.gpu)
        busid = g.xorg_busid
        # CDNA parts have no display engine: virtual framebuffer via the dummy driver
        driver = "amdgpu" if g.card and X.has_display_engine(f"/sys/class/drm/{g.card}") else "dummy"
    else:
        log.warning("no AMD GPU visible: X runs on the dummy driver, encoding needs a GPU")
    s = X.DisplaySettings(cfg.sizew, cfg.sizeh, cfg.refresh, cfg.cdepth, cfg.dpi, cfg.video_port, busid, driver,
                          cfg.display)
    xproc = X.start_x(s, conf_dir)
    if not X.wait_for_x(cfg.display, timeout=60.0):
        log.error("X server did not create its socket in 60 s")
        _terminate(xproc)
        return 1
    os.environ["DISPLAY"] = cfg.display
    icds = icd_report()
    log.info("ICDs: OpenCL %s, Vulkan %s", [lib for _, lib in icds["opencl"]] or "none",
             [lib for _, lib in icds["vulkan"]] or "none")
    env = desktop_env()
    children = []
    cmd = desktop_command(env)
    if cmd:
        children.append(subprocess.Popen(cmd, start_new_session=True, env=env))
    if shutil.which("fcitx"):
        children.append(subprocess.Popen(["fcitx"], start_new_session=True, env=env))
    print(f"mxdesk: display {cfg.display} ready ({cfg.sizew}x{cfg.sizeh}@{cfg.refresh}, driver {driver})", flush=True)

    def _stop(signum, frame):
        for c in children:
            _terminate(c)
        _terminate(xproc)
        sys.exit(0)

    signal.signal(signal.SIGTERM, _stop)
    signal.signal(signal.SIGINT, _stop)
    rc = xproc.wait()
    log.error("X server exited with %s; stopping the display session", rc)
    for c in children:
        _terminate(c)
    return rc or 1


def _terminate(p: subprocess.Popen, timeout: float = 5.0) -> None:
    if p.poll() is not None:
        return
    try:
        os.killpg(p.pid, signal.SIGTERM)
    except (ProcessLookupError, PermissionError):
        p.terminate()
    deadline = time.monotonic() + timeout
    while p.poll() is None and time.monotonic() < deadline:
        time.sleep(0.05)
    if p.poll() is None:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            p.kill()
