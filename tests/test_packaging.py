"""Packaging contract: container defaults match the config schema (and
therefore the reference's Dockerfile:200-212), the supervisor config parses with the right
priorities/readiness gates, the k8s manifests request AMD GPUs, the display bring-up only
removes stale X locks; host ASan/UBSan run of the native code."""
import os
import re
import shutil
import subprocess
from pathlib import Path

import pytest
import yaml

from mxdesk.display.desktop import clean_stale_locks, desktop_command
from mxdesk.utils import config as C
from mxdesk.utils.supervisor import load_ini

ROOT = Path(__file__).resolve().parents[1]


def _dockerfile_env():
    text = (ROOT / "docker/Dockerfile").read_text().replace("\\\n", " ")
    env = {}
    for line in text.splitlines():
        if line.startswith("ENV "):
            for k, v in re.findall(r"(\w+)=(\S+)", line):
                env[k] = v
    return env


def test_dockerfile_defaults_match_schema():
    env = _dockerfile_env()
    cfg = C.load(env={}, argv=[])
    names = {"TZ": "tz", "SIZEW": "sizew", "SIZEH": "sizeh", "REFRESH": "refresh", "DPI": "dpi", "CDEPTH": "cdepth",
             "VIDEO_PORT": "video_port", "PASSWD": "passwd", "NOVNC_ENABLE": "novnc_enable",
             "WEBRTC_ENCODER": "encoder", "WEBRTC_ENABLE_RESIZE": "enable_resize", "ENABLE_BASIC_AUTH": "enable_basic_auth"}
    for k, attr in names.items():
        assert k in env, k
        assert getattr(C.load(env={k: env[k]}, argv=[]), attr) == getattr(cfg, attr), k
    assert env["DISPLAY"] == ":0" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert "EXPOSE 8080" in (ROOT / "docker/Dockerfile").read_text()


def test_supervisord_conf_parses():
    progs, sup = load_ini(ROOT / "docker/supervisord.conf", env={"NOVNC_ENABLE": "false"})
    by = {p.name: p for p in progs}
    assert [p.name for p in sorted(progs, key=lambda p: p.priority)] == ["desktop", "pulseaudio", "mxdesk"]
    assert by["desktop"].ready.kind == "socket" and by["desktop"].ready.target == "/tmp/.X11-unix/X0"
    assert by["mxdesk"].ready.kind == "tcp" and by["mxdesk"].command[:3] == ["python3", "-m", "mxdesk"]
    assert all(p.autorestart == "true" for p in progs)
    assert sup["logfile"] == "/tmp/supervisord.log"


def test_k8s_manifests_request_amd_gpus():
    docs = list(yaml.safe_load_all((ROOT / "docker/k8s/mxdesk.yml").read_text()))
    dep = docs[0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 1
    assert {m["mountPath"] for m in c["volumeMounts"]} == {"/dev/shm", "/home/user", "/cache"}
    envs = {e["name"] for e in c["env"]}
    assert {"SIZEW", "SIZEH", "REFRESH", "PASSWD", "WEBRTC_ENCODER"} <= envs
    node = yaml.safe_load((ROOT / "docker/k8s/mxdesk-node.yml").read_text())
    assert node["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == 8


def test_stale_lock_cleanup_keeps_live_server(tmp_path):
    (tmp_path / ".X11-unix").mkdir()
    (tmp_path / ".X5-lock").write_text(f"{os.getpid():>10}\n")
    (tmp_path / ".X11-unix" / "X5").write_text("")
    assert clean_stale_locks(":5", str(tmp_path)) == []  # our own PID is alive
    assert (tmp_path / ".X5-lock").exists()
    p = subprocess.Popen(["true"])
    p.wait()
    (tmp_path / ".X5-lock").write_text(f"{p.pid:>10}\n")
    removed = clean_stale_locks(":5", str(tmp_path))
    assert len(removed) == 2 and not (tmp_path / ".X5-lock").exists()


def test_desktop_command_override():
    assert desktop_command({"MXDESK_DESKTOP_CMD": "openbox --replace"}) == ["openbox", "--replace"]


@pytest.mark.skipif(shutil.which("hipcc") is None and not Path("/opt/rocm/bin/hipcc").exists(), reason="no hipcc")
def test_host_sanitizers_clean():
    r = subprocess.run(["bash", str(ROOT / "tools/sanitize.sh")], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "sanitize: ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_dockerfile_optional_app_bundle_and_wine():
    text = (ROOT / "docker/Dockerfile").read_text()
    for arg in ("ARG APPS=core", "ARG WINE=false", "ARG WINE_BRANCH=staging"):
        assert arg in text
    assert "winehq-${WINE_BRANCH}" in text and "winetricks" in text and "lutris" in text
    assert "firefox" in text and "libreoffice" in text and "kscreenlockerrc" in text
    import yaml

    ci = yaml.safe_load((ROOT / ".github/workflows/ci.yml").read_text())
    tags = [m["tag"] for m in ci["jobs"]["image"]["strategy"]["matrix"]["include"]]
    assert "kde-full" in tags
