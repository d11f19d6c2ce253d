"""CPU tests of the control plane: config schema (reference env contract), CVT-RB
modelines (vs known `cvt` output), xorg.conf rendering, PCI bus-id conversion, device
discovery on a fake sysfs tree, and the supervisor (restart/backoff/readiness/killpg)."""
import os
import signal
import sys
import time
from pathlib import Path

import pytest

from mxdesk.display import xorg
from mxdesk.display.cvt import cvt
from mxdesk.utils import config as C
from mxdesk.utils import devices as D
from mxdesk.utils.supervisor import Program, Ready, State, Supervisor, load_ini

REF = Path("/root/reference")


# ------------------------------------------------------------------ config
def test_reference_defaults():
    cfg = C.load(env={}, argv=[])
    assert (cfg.sizew, cfg.sizeh, cfg.refresh, cfg.dpi, cfg.cdepth) == (1920, 1080, 60, 96, 24)
    assert cfg.video_port == "DFP" and cfg.passwd == "mypasswd" and cfg.tz == "UTC"
    assert cfg.novnc_enable is False and cfg.enable_basic_auth is True and cfg.enable_resize is False
    assert cfg.encoder == "nvh264enc" and cfg.encoder_backend == "mxh264enc"
    assert cfg.port == 8080 and cfg.display == ":0"
    assert cfg.effective_basic_auth_password == "mypasswd"  # selkies-gstreamer-entrypoint.sh:20


def test_env_and_cli_override_and_bool_case():
    env = {"SIZEW": "1280", "SIZEH": "720", "NOVNC_ENABLE": "TRUE", "ENABLE_BASIC_AUTH": "False",
           "WEBRTC_ENCODER": "x264enc", "BASIC_AUTH_PASSWORD": "s3cret", "TURN_PORT": "5349"}
    cfg = C.load(env=env, argv=["--refresh", "30"])
    assert (cfg.sizew, cfg.sizeh, cfg.refresh) == (1280, 720, 30)
    assert cfg.novnc_enable is True and cfg.enable_basic_auth is False
    assert cfg.encoder_backend == "cpuh264enc"
    assert cfg.effective_basic_auth_password == "s3cret"
    assert cfg.sources["refresh"] == "cli" and cfg.sources["sizew"] == "env:SIZEW"
    red = cfg.redacted()
    assert red["BASIC_AUTH_PASSWORD"] == "******" and red["PASSWD"] == "******"


@pytest.mark.parametrize("env", [{"SIZEW": "1281"}, {"CDEPTH": "17"}, {"WEBRTC_ENCODER": "bogusenc"},
                                 {"TURN_PROTOCOL": "sctp"}, {"NOVNC_ENABLE": "maybe"}])
def test_invalid_config_rejected(env):
    with pytest.raises(ValueError):
        C.load(env=env, argv=[])


def test_every_reference_env_var_is_in_schema():
    names = {n for v in C.SCHEMA for n in v.env}
    dockerfile_vars = ["TZ", "SIZEW", "SIZEH", "REFRESH", "DPI", "CDEPTH", "VIDEO_PORT", "PASSWD", "NOVNC_ENABLE",
                       "WEBRTC_ENCODER", "WEBRTC_ENABLE_RESIZE", "ENABLE_BASIC_AUTH", "DISPLAY", "XDG_RUNTIME_DIR",
                       "PULSE_SERVER"]
    k8s_vars = ["NOVNC_VIEWPASS", "ENABLE_HTTPS_WEB", "HTTPS_WEB_CERT", "HTTPS_WEB_KEY", "BASIC_AUTH_PASSWORD",
                "TURN_HOST", "TURN_PORT", "TURN_SHARED_SECRET", "TURN_USERNAME", "TURN_PASSWORD", "TURN_PROTOCOL",
                "TURN_TLS", "GST_DEBUG"]
    missing = [v for v in dockerfile_vars + k8s_vars if v not in names]
    assert not missing, missing
    if (REF / "xgl.yml").exists():  # every env name in the reference manifest is known
        import re
        for n in re.findall(r"name:\s+([A-Z_]+)\s*$", (REF / "xgl.yml").read_text(), re.M):
            assert n in names, n


def test_keyframe_distance_and_log_level():
    cfg = C.load(env={"SELKIES_KEYFRAME_DISTANCE": "2", "GST_DEBUG": "*:4"}, argv=[])
    assert cfg.keyint_frames == 120 and cfg.log_level_name == "INFO"
    assert C.load(env={}, argv=[]).keyint_frames == 0


# ------------------------------------------------------------------ CVT / xorg
@pytest.mark.parametrize("args,expect", [
    ((1920, 1080, 60, True), 'Modeline "1920x1080R"  138.50  1920 1968 2000 2080  1080 1083 1088 1111 +hsync -vsync'),
    ((1280, 720, 60, True), 'Modeline "1280x720R"  64.00  1280 1328 1360 1440  720 723 728 741 +hsync -vsync'),
    ((3840, 2160, 60, True), 'Modeline "3840x2160R"  533.25  3840 3888 3920 4000  2160 2163 2168 2222 +hsync -vsync'),
    ((1920, 1080, 60, False),
     'Modeline "1920x1080_60.00"  173.00  1920 2048 2248 2576  1080 1083 1088 1120 -hsync +vsync'),
    ((1024, 768, 60, False), 'Modeline "1024x768_60.00"  63.50  1024 1072 1176 1328  768 771 775 798 -hsync +vsync'),
])
def test_cvt_matches_cvt_tool(args, expect):
    w, h, r, rb = args
    m = cvt(w, h, r, reduced=rb)
    assert m.xorg() == expect
    assert abs(m.refresh_hz - r) < 0.6


def test_xorg_conf_rendering():
    s = xorg.DisplaySettings(width=2560, height=1440, refresh=60, depth=24, busid=D.pci_to_xorg_busid("0000:0a:00.0"))
    text = xorg.render_xorg_conf(s)
    assert 'BusID          "PCI:10:0:0"' in text
    assert '"AutoAddGPU" "false"' in text
    assert 'Modeline "2560x1440R"' in text and "Virtual     2560 1440" in text
    assert 'Driver         "dummy"' in text
    none = xorg.render_xorg_conf(xorg.DisplaySettings(video_port="none"))
    assert '"RANDR" "Disable"' in none
    cmd = xorg.xorg_command(xorg.DisplaySettings(dpi=120, video_port="none"))
    assert cmd[:2] == ["Xorg", "vt7"] and "-dpi" in cmd and "RANDR" not in cmd and cmd[-1] == ":0"
    assert xorg.patch_xwrapper("allowed_users=console\n") == "allowed_users=anybody\nneeds_root_rights=yes\n"
    assert xorg.x_socket(":0") == "/tmp/.X11-unix/X0"


@pytest.mark.parametrize("bdf,busid", [("0000:0a:00.0", "PCI:10:0:0"), ("00000000:C1:1F.7", "PCI:193:31:7"),
                                       ("1b:00.0", "PCI:27:0:0")])
def test_pci_busid(bdf, busid):
    assert D.pci_to_xorg_busid(bdf) == busid


# ------------------------------------------------------------------ devices (fake sysfs)
def _fake_sysfs(tmp: Path, gpus):
    sysfs, dev = tmp / "sys", tmp / "dev"
    (dev / "dri").mkdir(parents=True)
    for k, (bdf, uid, visible) in enumerate(gpus):
        pdev = sysfs / "devices/pci0000:00" / bdf
        pdev.mkdir(parents=True)
        (pdev / "vendor").write_text("0x1002\n")
        (pdev / "device").write_text("0x75a3\n")
        (pdev / "numa_node").write_text(f"{k % 2}\n")
        (pdev / "unique_id").write_text(uid + "\n")
        rn = sysfs / "class/drm" / f"renderD{128 + k}"
        rn.mkdir(parents=True)
        (rn / "device").symlink_to(pdev)
        card = sysfs / "class/drm" / f"card{k}"
        card.mkdir(parents=True)
        (card / "device").symlink_to(pdev)
        if visible:
            (dev / "dri" / f"renderD{128 + k}").write_text("")
        node = sysfs / "class/kfd/kfd/topology/nodes" / str(k + 1)
        (node / "io_links/0").mkdir(parents=True)
        b, d_, f = int(bdf[5:7], 16), int(bdf[8:10], 16), int(bdf[11], 16)
        (node / "properties").write_text(f"simd_count 1024\nlocation_id {(b << 8) | (d_ << 3) | f}\ndomain 0\n"
                                         f"gfx_target_version 90500\n")
        (node / "io_links/0/properties").write_text(f"type 11\nnode_to {((k + 1) % len(gpus)) + 1}\n")
    return sysfs, dev


def test_enumerate_and_select(tmp_path):
    sysfs, dev = _fake_sysfs(tmp_path, [("0000:75:00.0", "aaaa", True), ("0000:0a:00.0", "bbbb", True),
                                        ("0000:f5:00.0", "cccc", False)])
    gpus = D.enumerate_gpus(sysfs, dev)
    assert [g.pci_bdf for g in gpus] == ["0000:0a:00.0", "0000:75:00.0"]
    assert gpus[0].xorg_busid == "PCI:10:0:0" and gpus[0].unique_id == "bbbb"
    assert gpus[0].kfd_node == 2 and gpus[0].xgmi_peers and gpus[0].gfx_target == "90500"
    assert D.visible_gpus(gpus, {"HIP_VISIBLE_DEVICES": "1"})[0].pci_bdf == "0000:75:00.0"
    assert D.visible_gpus(gpus, {"ROCR_VISIBLE_DEVICES": "0000:75:00.0"})[0].unique_id == "aaaa"
    assert len(D.visible_gpus(gpus, {"HIP_VISIBLE_DEVICES": "all"})) == 2
    assert D.select_gpu(gpus, "aaaa").pci_bdf == "0000:75:00.0"
    assert D.select_gpu(gpus, "nonexistent").index == 0  # falls back to the first GPU
    with pytest.raises(D.NoGpuError):
        D.select_gpu([])


# ------------------------------------------------------------------ supervisor
def _py(code):
    return [sys.executable, "-c", code]


def test_supervisor_restart_backoff_and_fatal(tmp_path):
    flap = Program("flap", _py("import sys; sys.exit(3)"), priority=2, startsecs=0.5, startretries=2,
                   autorestart="true")
    ok = Program("ok", _py("import time; time.sleep(30)"), priority=1, startsecs=0.2)
    sup = Supervisor([flap, ok], log_dir=str(tmp_path), poll=0.02)
    sup.start()
    deadline = time.monotonic() + 10
    while time.monotonic() < deadline and sup.states["flap"].state != State.FATAL:
        sup.tick()
        time.sleep(0.02)
    st = sup.status()
    assert st["flap"]["state"] == "FATAL" and st["flap"]["restarts"] >= 2 and set(st["flap"]["exit_codes"]) == {3}
    assert st["ok"]["state"] in ("RUNNING", "STARTING")
    sup.stop()
    assert sup.states["ok"].proc.poll() is not None


def test_supervisor_readiness_orders_start_and_kills_group(tmp_path):
    sock = tmp_path / "X0"
    marker = tmp_path / "child.pid"
    # first program becomes "ready" after 0.3 s and forks a grandchild
    p1 = Program("x", _py(f"import os,time,subprocess; time.sleep(0.3); open({str(sock)!r},'w').close(); "
                          f"c=subprocess.Popen(['sleep','60']); open({str(marker)!r},'w').write(str(c.pid)); "
                          f"time.sleep(60)"),
                 priority=1, ready=Ready("file", str(sock), 5.0))
    p2 = Program("after", _py(f"import os,sys; sys.exit(0 if os.path.exists({str(sock)!r}) else 9)"), priority=2,
                 autorestart="false", startsecs=0)
    sup = Supervisor([p1, p2], log_dir=str(tmp_path), poll=0.02)
    sup.start()
    for _ in range(100):
        sup.tick()
        time.sleep(0.02)
        if sup.states["after"].exit_codes:
            break
    assert sup.states["after"].exit_codes == [0]
    for _ in range(100):
        if marker.exists() and marker.read_text():
            break
        time.sleep(0.02)
    child = int(marker.read_text())
    sup.stop()
    time.sleep(0.2)
    status = Path(f"/proc/{child}/status")
    alive = status.exists() and "State:\tZ" not in status.read_text()
    assert not alive  # the grandchild died with the process group (dead or zombie)


def test_load_reference_supervisord_conf(tmp_path):
    ref = REF / "supervisord.conf"
    text = ref.read_text() if ref.exists() else "[supervisord]\nlogfile=/tmp/s.log\n[program:a]\ncommand=true\n"
    p = tmp_path / "s.conf"
    p.write_text(text)
    progs, sup = load_ini(p, env={"NOVNC_ENABLE": "false", "DISPLAY": ":0"})
    if ref.exists():
        assert [x.name for x in sorted(progs, key=lambda x: x.priority)] == ["entrypoint", "pulseaudio",
                                                                            "selkies-gstreamer"]
        assert all(x.autorestart == "true" for x in progs) and progs[0].stopsignal == signal.SIGINT
        assert "false" in " ".join(progs[2].command)
        assert sup["logfile"] == "/tmp/supervisord.log"


def test_gpu_telemetry_from_fake_sysfs(tmp_path):
    from mxdesk.utils.devices import gpu_telemetry
    from mxdesk.utils.metrics import SessionMetrics

    dev = tmp_path / "bus/pci/devices/0000:05:00.0"
    (dev / "hwmon/hwmon3").mkdir(parents=True)
    (dev / "gpu_busy_percent").write_text("37\n")
    (dev / "mem_info_vram_used").write_text("1073741824\n")
    (dev / "mem_info_vram_total").write_text("309237645312\n")
    (dev / "hwmon/hwmon3/power1_average").write_text("512000000\n")
    (dev / "hwmon/hwmon3/temp1_input").write_text("45000\n")
    (dev / "hwmon/hwmon3/temp2_input").write_text("61000\n")
    t = gpu_telemetry("0000:05:00.0", tmp_path)
    assert t == {"busy_percent": 37.0, "vram_used_bytes": 1073741824.0, "vram_total_bytes": 309237645312.0,
                 "power_watts": 512.0, "temperature_c": 61.0}
    assert gpu_telemetry("0000:99:00.0", tmp_path) == {}
    m = SessionMetrics("s0")
    m.set_gpu_telemetry("0000:05:00.0", t)
    text = m.exposition().decode()
    assert 'mxdesk_gpu{gpu="0000:05:00.0",metric="power_watts",session="s0"} 512.0' in text


def test_json_log_format():
    import json
    import logging

    from mxdesk.cli import JsonFormatter

    rec = logging.LogRecord("mxdesk.test", logging.WARNING, __file__, 1, "hello %s", ("wörld",), None)
    d = json.loads(JsonFormatter().format(rec))
    assert d["msg"] == "hello wörld" and d["level"] == "WARNING" and d["logger"] == "mxdesk.test"
    assert C.load(env={"MXDESK_LOG_FORMAT": "json"}, argv=[]).log_format == "json"


def test_unimplemented_selkies_encoders_fall_back_to_h264():
    cfg = C.load(env={"WEBRTC_ENCODER": "vp9enc"}, argv=[])
    assert cfg.encoder_backend == "mxh264enc" and cfg.codec == "h264" and cfg.gpu_encoder
    assert "vp9enc" in cfg.encoder_fallback
    assert C.load(env={"WEBRTC_ENCODER": "nvh264enc"}, argv=[]).encoder_fallback is None
    with pytest.raises(ValueError):
        C.load(env={"WEBRTC_ENCODER": "bogusenc"}, argv=[]).encoder_backend


def test_vp8enc_selects_the_vp8_encoder():
    # the reference's libvpx choice (README.md:21,35) is implemented: no fallback
    for name in ("vp8enc", "vaapivp8enc", "mxvp8enc"):
        cfg = C.load(env={"WEBRTC_ENCODER": name}, argv=[])
        assert cfg.encoder_backend == "mxvp8enc" and cfg.codec == "vp8" and cfg.gpu_encoder
        assert cfg.encoder_fallback is None
    cfg = C.load(env={"WEBRTC_ENCODER": "cpuvp8enc"}, argv=[])
    assert cfg.codec == "vp8" and not cfg.gpu_encoder


def test_serve_wires_xtest_injector_for_x11_capture(monkeypatch):
    """with an X11 capture the WebRTC/VNC input must reach X through XTest, not the
    synthetic cursor; without a capture (synthetic desktop) no XTest is attempted."""
    import types

    from mxdesk import cli
    from mxdesk.server import input as I
    from mxdesk.utils import config as C

    made = []

    class FakeXTest:
        def __init__(self, display):
            made.append(display)

        def apply(self, ev):
            pass

    monkeypatch.setattr(I, "XTestInjector", FakeXTest)
    cfg = C.load(env={"DISPLAY": ":7"})
    inj = cli.make_injector(cfg, types.SimpleNamespace(capture=object()))
    assert isinstance(inj, FakeXTest) and made == [cfg.display]
    assert cli.make_injector(cfg, types.SimpleNamespace(capture=None)) is None

    class Broken:
        def __init__(self, display):
            raise OSError("no libXtst")

    monkeypatch.setattr(I, "XTestInjector", Broken)
    assert cli.make_injector(cfg, types.SimpleNamespace(capture=object())) is None
