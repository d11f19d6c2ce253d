"""Display bring-up helpers: Xwrapper patch, Xorg command line,
X-socket readiness probe, X11 capture failure mode without a server, session-per-GPU programs."""
import os
import threading
import time
from pathlib import Path

import pytest

from mxdesk.display import xorg as X
from mxdesk.parallel.launcher import session_programs


def test_patch_xwrapper():
    out = X.patch_xwrapper("# Xwrapper.config\nallowed_users=console\n")
    assert "allowed_users=anybody" in out and "needs_root_rights=yes" in out
    assert X.patch_xwrapper("allowed_users=anybody\nneeds_root_rights=no\n").count("needs_root_rights") == 1


def test_xorg_command_extensions_and_randr_off():
    s = X.DisplaySettings(video_port="DFP", dpi=120, display=":3")
    cmd = X.xorg_command(s, "/tmp/x.conf")
    assert cmd[:6] == ["Xorg", "vt7", "-noreset", "-novtswitch", "-sharevts", "-dpi"] and cmd[-1] == ":3"
    assert ["+extension", "MIT-SHM"] == cmd[cmd.index("MIT-SHM") - 1:cmd.index("MIT-SHM") + 1]
    assert "RANDR" in cmd and "-config" in cmd
    assert "RANDR" not in X.xorg_command(X.DisplaySettings(video_port="none"))  # README.md:226,234


def test_wait_for_x_sees_socket():
    disp = ":%d" % (900 + os.getpid() % 90)
    path = Path(X.x_socket(disp))
    path.parent.mkdir(parents=True, exist_ok=True)
    path.unlink(missing_ok=True)
    try:
        assert not X.wait_for_x(disp, timeout=0.2, poll=0.05)
        threading.Timer(0.2, path.touch).start()
        t0 = time.monotonic()
        assert X.wait_for_x(disp, timeout=5, poll=0.05)
        assert time.monotonic() - t0 < 4
    finally:
        path.unlink(missing_ok=True)


def test_x11_capture_without_server_fails_cleanly():
    from mxdesk.models.x11 import X11Capture

    with pytest.raises(OSError, match="cannot open X display"):
        X11Capture(":987")


def test_session_programs_pin_one_gpu_each():
    # K sessions per GPU live in ONE process per GPU (serve --sessions K), ports base + K*gpu ..
    progs = session_programs(4, base_port=9000, sessions_per_gpu=2)
    assert len(progs) == 4
    assert [p.environment["HIP_VISIBLE_DEVICES"] for p in progs] == ["0", "1", "2", "3"]
    assert [p.environment["SELKIES_PORT"] for p in progs] == ["9000", "9002", "9004", "9006"]
    assert all(p.ready.kind == "tcp" and p.command[1:4] == ["-m", "mxdesk", "serve"] for p in progs)
    assert all(p.command[-2:] == ["--sessions", "2"] for p in progs)
    single = session_programs(2, base_port=9000)
    assert [p.environment["SELKIES_PORT"] for p in single] == ["9000", "9001"]
    assert all("--sessions" not in p.command for p in single)
    # more sessions than one event loop serves: split over processes of the same GPU
    many = session_programs(2, base_port=9000, sessions_per_gpu=40, sessions_per_process=16)
    assert len(many) == 6 and [p.environment["HIP_VISIBLE_DEVICES"] for p in many] == ["0"] * 3 + ["1"] * 3
    assert [p.environment["SELKIES_PORT"] for p in many] == ["9000", "9014", "9027", "9040", "9054", "9067"]
    assert [int(p.command[-1]) for p in many] == [14, 13, 13, 14, 13, 13]


def test_serve_sessions_streams_k_sessions_from_one_process(native, monkeypatch):
    """`mxdesk serve --sessions 3` (CPU plumbing backend here): three MediaServers on consecutive
    ports in one event loop, each streaming its own desktop over /mxws."""
    import asyncio
    import threading

    from mxdesk import cli
    from mxdesk.server import app as A
    from mxdesk.utils import config as C

    from .test_server import free_port, view

    base = free_port()
    cfg = C.load(env={"WEBRTC_ENCODER": "x264enc", "SIZEW": "160", "SIZEH": "96", "REFRESH": "30",
                      "ENABLE_BASIC_AUTH": "false", "SELKIES_ENABLE_AUDIO": "false", "MXDESK_GAMEPAD": "false",
                      "MXDESK_SOURCE": "synthetic"}, argv=["--port", str(base), "--sessions", "3"])
    assert cfg.sessions == 3
    started = {}

    def fake_run(servers, host, ports, ssl_ctx=None):
        started["servers"], started["ports"] = servers, ports

        async def main():
            runners = [await A.serve(s, "127.0.0.1", p) for s, p in zip(servers, ports)]
            try:
                return [await view(f"http://127.0.0.1:{p}/mxws", 3) for p in ports]
            finally:
                for r in runners:
                    await r.cleanup()
        started["results"] = asyncio.run(main())

    monkeypatch.setattr(A, "run_forever_multi", fake_run)
    cli.cmd_serve(cfg, None)
    assert started["ports"] == [base, base + 1, base + 2]
    assert len({id(s.pipeline) for s in started["servers"]}) == 3
    assert [len(r.frames) for r in started["results"]] == [3, 3, 3]
    assert all(r.frames[0]["key"] for r in started["results"])
    assert threading.active_count() < 50


def test_desktop_env_gl_hygiene_and_icd_report(tmp_path):
    from mxdesk.display.desktop import GL_ENV, desktop_env, icd_report

    env = desktop_env({"PATH": "/bin", "vblank_mode": "1"})
    assert env["vblank_mode"] == "1"  # a user's explicit choice wins
    assert env["__GL_SYNC_TO_VBLANK"] == "0" and env["PATH"] == "/bin"
    assert desktop_env({})["vblank_mode"] == GL_ENV["vblank_mode"] == "0"
    ocl = tmp_path / "ocl"
    vk = tmp_path / "vk"
    ocl.mkdir()
    vk.mkdir()
    (ocl / "amdocl64.icd").write_text("libamdocl64.so\n")
    (vk / "lvp_icd.x86_64.json").write_text('{"ICD": {"library_path": "libvulkan_lvp.so"}}')
    (vk / "broken.json").write_text("{not json")
    rep = icd_report((str(ocl),), (str(vk), str(tmp_path / "missing")))
    assert rep["opencl"] == [(str(ocl / "amdocl64.icd"), "libamdocl64.so")]
    assert rep["vulkan"] == [(str(vk / "lvp_icd.x86_64.json"), "libvulkan_lvp.so")]
