"""bench.py's serving-configuration probe (serving_probe): a child process of the bench rank -- never
an exec -- with the serving path's 16 hardware queues, on the rank's own GPU, outside the process
group, whose one JSON line is parsed back (subprocess.run mocked: no GPU here)."""
import json
import subprocess
import sys
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_serving_probe_child_command_and_env(monkeypatch):
    seen = {}

    def fake_run(cmd, env, capture_output, text, timeout):
        seen["cmd"], seen["env"] = cmd, env
        out = {"density": {"sustained": 176}, "storm": {"sustained": 121}, "hw_queues": env["GPU_MAX_HW_QUEUES"]}
        return subprocess.CompletedProcess(cmd, 0, stdout="noise\n" + json.dumps(out) + "\n", stderr="")

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "5", "--codec", "h264"])
    for k, v in {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3", "MASTER_ADDR": "127.0.0.1"}.items():
        monkeypatch.setenv(k, v)
    r = bench.serving_probe(SimpleNamespace(), 3)
    assert r["density"]["sustained"] == 176 and r["storm"]["sustained"] == 121
    cmd, env = seen["cmd"], seen["env"]
    assert cmd[0] == sys.executable and cmd[1].endswith("bench.py")
    assert cmd[2:5] == ["--steps", "5", "--codec"]  # the rank's own flags, then the overrides (last wins)
    i = cmd.index("--density-only")
    assert cmd[i + 1] == "1" and cmd[cmd.index("--device-index") + 1] == "3" and cmd[cmd.index("--gpus") + 1] == "1"
    assert env["GPU_MAX_HW_QUEUES"] == "16"
    assert not any(k in env for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR"))


def test_serving_probe_failure_is_reported_not_raised(monkeypatch, capsys):
    monkeypatch.setattr(subprocess, "run",
                        lambda cmd, **kw: subprocess.CompletedProcess(cmd, 1, stdout="", stderr="boom"))
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert bench.serving_probe(SimpleNamespace(), 0) is None
    assert "serving probe failed" in capsys.readouterr().err
