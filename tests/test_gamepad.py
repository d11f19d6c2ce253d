"""Gamepad path: browser js,* messages -> GamepadServer -> LD_PRELOAD
interposer -> an unmodified C program reading /dev/input/js0 with the joystick ioctls."""
import asyncio
import os
import shutil
import subprocess
from pathlib import Path

import pytest

from mxdesk.server.gamepad import GamepadServer, interposer_path
from mxdesk.server.input import parse_message

HERE = Path(__file__).resolve().parent


def test_parse_gamepad_messages():
    ev = parse_message("js,c,0,WGJveCBQYWQ=,6,17")
    assert ev.kind == "gamepad" and ev.extra == {"op": "c", "idx": 0, "name": "Xbox Pad", "axes": 6, "buttons": 17}
    assert parse_message("js,a,1,3,-0.5").extra == {"op": "a", "idx": 1, "num": 3, "value": -0.5}
    assert parse_message("js,b,0,2,1").extra["op"] == "b"
    assert parse_message("js,d,2").extra == {"op": "d", "idx": 2}


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no C compiler")
def test_interposer_end_to_end(tmp_path):
    from mxdesk import _build

    lib = _build.build_interposer()
    assert lib == interposer_path() and lib.exists()
    exe = tmp_path / "js_reader"
    subprocess.run(["gcc", "-O1", "-o", str(exe), str(HERE / "native/js_reader.c")], check=True)

    async def go():
        srv = GamepadServer(tmp_path)
        await srv.start()
        srv.apply(parse_message("js,c,0,bXhkZXNrIHBhZA==,6,17"))
        env = dict(os.environ)
        env["MXDESK_JS_DIR"] = str(tmp_path)
        env["LD_PRELOAD"] = str(lib) + (":" + env["LD_PRELOAD"] if env.get("LD_PRELOAD") else "")
        proc = await asyncio.create_subprocess_exec(str(exe), "3", env=env, stdout=asyncio.subprocess.PIPE,
                                                    stderr=asyncio.subprocess.PIPE)
        for _ in range(200):  # wait until the app has connected
            if srv.pads[0].writers:
                break
            await asyncio.sleep(0.01)
        for m in ("js,b,0,0,1", "js,a,0,1,-1.0", "js,b,0,0,0", "js,b,0,0,0"):  # last one: no change, no event
            srv.apply(parse_message(m))
        for w in srv.pads[0].writers:
            await w.drain()
        out, err = await asyncio.wait_for(proc.communicate(), 20)
        await srv.stop()
        return proc.returncode, out.decode(), err.decode()

    rc, out, err = asyncio.run(go())
    assert rc == 0, (out, err)
    lines = out.strip().splitlines()
    assert lines[0] == "version=020100 axes=6 buttons=17 name=mxdesk pad btn0=0x130 ax2=3"
    assert lines[1:] == ["event type=1 number=0 value=1", "event type=2 number=1 value=-32767",
                         "event type=1 number=0 value=0"]


def test_interposer_absent_device_behaves_like_enoent(tmp_path):
    lib = interposer_path()
    if not lib.exists():
        pytest.skip("interposer not built")
    env = dict(os.environ, MXDESK_JS_DIR=str(tmp_path))
    env["LD_PRELOAD"] = str(lib) + (":" + env["LD_PRELOAD"] if env.get("LD_PRELOAD") else "")
    r = subprocess.run(["python3", "-c", "import os\ntry:\n os.open('/dev/input/js1', os.O_RDONLY)\nexcept OSError as e:\n print(e.errno)"],
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.stdout.strip() == "2"  # ENOENT: no server socket -> no joystick
