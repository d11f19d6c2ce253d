"""Integration tests of the web front end with the CPU plumbing backend (no GPU): media
WebSocket -> independent decoder -> barcode, basic auth, health/turn/metrics/status,
selkies signalling relay, input injection, keyframe resync, fault injection."""
import asyncio
import base64
import json
import socket

import aiohttp
import numpy as np
import pytest

from mxdesk.codec.h264_decoder import Decoder
from mxdesk.models.synthetic import read_barcode
from mxdesk.pipeline.stream import StreamPipeline
from mxdesk.server.app import MediaServer, serve
from mxdesk.server.client import view
from mxdesk.server.input import parse_message
from mxdesk.utils import config as C


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_server(env=None, **kw):
    cfg = C.load(env={"WEBRTC_ENCODER": "x264enc", "SIZEW": "320", "SIZEH": "96", "REFRESH": "30",
                      **(env or {})}, argv=[])
    if kw.get("codec", "h264") is None:
        kw["codec"] = cfg.codec
    pipe = StreamPipeline(cfg.sizew, cfg.sizeh, cfg.stream_fps, backend="cpu", bitrate_kbps=0, **kw)
    return cfg, pipe, MediaServer(pipe, cfg)


def run(coro):
    return asyncio.run(coro)


def test_stream_decodes_and_barcodes_match():
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await view(f"http://127.0.0.1:{port}/mxws", 6)
        finally:
            await runner.cleanup()

    res = run(go())
    assert res.config["codec"].startswith("avc1.42C0") and res.config["width"] == 320
    assert len(res.frames) == 6 and res.frames[0]["key"]
    frames = Decoder().decode(res.stream)
    assert len(frames) == 6
    for (y, _, _), meta in zip(frames, res.frames):
        fid, _ = read_barcode(y)
        assert fid == meta["frame_id"]
    assert all(0 <= ms < 5000 for ms in res.latency_ms)


def test_basic_auth_and_endpoints():
    cfg, pipe, srv = make_server({"PASSWD": "pw1", "TURN_HOST": "turn.example.com", "TURN_SHARED_SECRET": "sekret"})

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        base = f"http://127.0.0.1:{port}"
        try:
            async with aiohttp.ClientSession() as s:
                async with s.get(base + "/") as r:
                    assert r.status == 401 and "Basic" in r.headers["WWW-Authenticate"]
                async with s.get(base + "/health") as r:
                    assert r.status == 200
            auth = aiohttp.BasicAuth("user", "pw1")
            async with aiohttp.ClientSession(headers={"Authorization": auth.encode()} if auth else None) as s:
                async with s.get(base + "/") as r:
                    assert r.status == 200 and "client.js" in await r.text()
                async with s.get(base + "/client.js") as r:
                    assert r.status == 200
                async with s.get(base + "/turn") as r:
                    d = await r.json()
                    turn = [x for x in d["iceServers"] if x["urls"][0].startswith("turn")][0]
                    assert turn["urls"] == ["turn:turn.example.com:3478?transport=udp"]
                    assert ":" in turn["username"] and len(base64.b64decode(turn["credential"])) == 20
                async with s.get(base + "/manifest.json") as r:
                    assert json.loads(await r.text())["short_name"] == "mxdesk"
            res = await view(base.replace("http", "http") + "/mxws", 3, user="user", password="pw1")
            async with aiohttp.ClientSession(headers={"Authorization": auth.encode()} if auth else None) as s:
                async with s.get(base + "/metrics") as r:
                    assert "mxdesk_encoded_frames_total" in await r.text()
                async with s.get(base + "/status") as r:
                    st = await r.json()
                    assert st["frames"] >= 3 and st["backend"] == "cpu"
            return res
        finally:
            await runner.cleanup()

    res = run(go())
    assert len(res.frames) == 3


def test_signalling_relay():
    # browser <-> browser relaying (the in-process streaming peer off: it would take uid 0)
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "MXDESK_SELKIES_PEER": "false"})

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        url = f"http://127.0.0.1:{port}/ws"
        try:
            async with aiohttp.ClientSession() as s:
                a = await s.ws_connect(url)
                b = await s.ws_connect(url)
                await a.send_str("HELLO 0")
                assert (await a.receive()).data == "HELLO"
                await b.send_str("HELLO 1 eyJ9")
                assert (await b.receive()).data == "HELLO"
                await b.send_str("SESSION 7")
                assert (await b.receive()).data.startswith("ERROR")
                await b.send_str("SESSION 0")
                assert (await b.receive()).data == "SESSION_OK"
                await b.send_str(json.dumps({"sdp": {"type": "offer", "sdp": "v=0"}}))
                assert json.loads((await a.receive()).data)["sdp"]["type"] == "offer"
                await a.send_str(json.dumps({"ice": {"candidate": "x", "sdpMLineIndex": 0}}))
                assert "ice" in json.loads((await b.receive()).data)
                await a.close()
                assert "disconnected" in (await b.receive()).data
                await b.close()
        finally:
            await runner.cleanup()

    run(go())


def test_input_moves_synthetic_cursor_and_pli():
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await view(f"http://127.0.0.1:{port}/mxws", 4, send=["m,40,30,1,0", "kd,65", "pli",
                                                                          json.dumps({"type": "bitrate", "kbps": 500})])
        finally:
            await runner.cleanup()

    res = run(go())
    inj = srv.injector
    assert (inj.x, inj.y, inj.buttons) == (40, 30, 1) and 65 in inj.keys_down
    assert pipe._cursor == (40, 30)


def test_parse_selkies_messages():
    assert parse_message("m2,-3,4,0,0").relative
    assert parse_message("cw," + base64.b64encode("héllo".encode()).decode()).text == "héllo"
    assert (parse_message("r,1280x720").width, parse_message("r,1280x720").height) == (1280, 720)
    assert parse_message("bogus,1") is None and parse_message("m,x") is None


def test_pipeline_fault_injection_restarts(monkeypatch):
    monkeypatch.setenv("MXDESK_FAULT", "crash:2")
    pipe = StreamPipeline(64, 48, 60, backend="cpu", bitrate_kbps=0, paced=False)
    pipe.start()
    import time
    deadline = time.time() + 10
    while pipe.frames_out < 5 and time.time() < deadline:
        time.sleep(0.01)
    pipe.stop()
    assert pipe.restarts == 1 and "injected" in pipe.last_error and pipe.frames_out >= 5


def test_slow_client_resync():
    """A viewer whose queue overflows loses its backlog and waits for an IDR -- which the overflow
    itself forces, so the viewer resumes at the next frame (without it the viewer stalled until
    the stream's next key frame)."""
    pipe = StreamPipeline(64, 48, 60, backend="cpu", bitrate_kbps=0, queue_frames=2, idr_min_interval_s=0.0)

    async def go():
        sub = pipe.subscribe(asyncio.get_running_loop())
        for _ in range(8):
            pipe.step()
        await asyncio.sleep(0.05)
        got = []
        while not sub.queue.empty():
            got.append(sub.queue.get_nowait())
        state = (sub.dropped, sub.need_idr)
        fr = pipe.step()
        await asyncio.sleep(0.05)
        after = []
        while not sub.queue.empty():
            after.append(sub.queue.get_nowait())
        return sub, state, fr, after

    sub, (dropped, waiting), fr, after = run(go())
    assert dropped > 0 and waiting  # backlog dropped, waiting for the next IDR
    assert pipe.metrics.dropped.labels("0")._value.get() > 0
    assert fr.idr and after and after[0].idr and not sub.need_idr  # the forced IDR resynchronised it


class _FakeClock:
    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def test_pli_burst_codes_one_idr():
    """50 PLIs within 100 ms (a burst of viewers on a lossy link) produce exactly one IDR: the
    first schedules it, the ones arriving while it is pending join it, the ones after it was
    coded are covered by it."""
    clk = _FakeClock()
    pipe = StreamPipeline(64, 48, 60, backend="cpu", bitrate_kbps=0)
    pipe.keyframes.clock = clk
    first = pipe.step()
    assert first.idr
    clk.t += 1.0  # well past the minimum interval
    idrs, pli = 0, 0
    for f in range(30):  # 0.5 s of frames at 60 fps, PLIs every 2 ms during the first 100 ms
        t_end = clk.t + 1 / 60
        while clk.t < t_end:
            if pli < 50:
                pipe.request_idr("pli")
                pli += 1
            clk.t += 0.002
        idrs += pipe.step().idr
    assert pli == 50 and idrs == 1
    snap = pipe.keyframes.snapshot()
    assert snap["requests"]["pli"] == 50 and snap["coalesced"] == 49 and snap["forced"] >= 1
    assert pipe.metrics.kf_coalesced.labels("0")._value.get() == 49
    assert b"mxdesk_keyframe_requests_total" in pipe.metrics.exposition()


def test_stalled_viewer_idr_rate_is_bounded():
    """A viewer that never drains overflows its queue again right after every resync: its IDR
    requests back off exponentially and the session's forced IDRs stay >= the minimum interval
    apart (ADVICE r5 stream.py:323)."""
    clk = _FakeClock()
    pipe = StreamPipeline(64, 48, 60, backend="cpu", bitrate_kbps=0, queue_frames=2)
    pipe.keyframes.clock = clk

    async def go():
        pipe.subscribe(asyncio.get_running_loop())  # never read
        times = []
        for _ in range(600):  # 10 s at 60 fps
            if pipe.step().idr:
                times.append(clk.t)
            await asyncio.sleep(0)
            clk.t += 1 / 60
        return times

    times = run(go())
    gaps = [b - a for a, b in zip(times, times[1:])]
    assert 3 <= len(times) <= 8, times  # resyncs happen, but backed off (0, 0.5, 1, 2, 4 s)
    assert min(gaps) >= 0.25 - 1e-9
    assert pipe.metrics.kf_requests.labels("0", "overflow_backoff")._value.get() > 0


def test_hevc_stream_over_websocket():
    from mxdesk.codec.hevc_decoder import Decoder as HevcDecoder

    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "WEBRTC_ENCODER": "x265enc"}, codec=None)

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await view(f"http://127.0.0.1:{port}/mxws", 4)
        finally:
            await runner.cleanup()

    assert cfg.codec == "hevc" and pipe.codec == "hevc"
    res = run(go())
    assert res.config["codec"].startswith("hvc1.1.6.L") and res.config["codec"].endswith(".B0")
    assert all(f["codec"] == 2 for f in res.frames)
    frames = HevcDecoder().decode(res.stream)
    assert len(frames) == 4
    for (y, _, _), meta in zip(frames, res.frames):
        assert read_barcode(y)[0] == meta["frame_id"]


def test_webrtc_statistics_csv(tmp_path):
    import csv

    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "SELKIES_ENABLE_WEBRTC_STATISTICS": "true",
                                  "SELKIES_WEBRTC_STATISTICS_DIR": str(tmp_path)})
    srv._on_client_message('{"type": "stats", "fps": 59.9, "packets_lost": 2, "nested": {"x": 1}}')
    srv._on_client_message('{"type": "stats", "fps": 60.0, "jitter": 0.001}')
    rows = list(csv.reader(open(srv.stats_log.path)))
    assert rows[0] == ["server_time", "fps", "packets_lost"]
    assert rows[1][1:] == ["59.9", "2"] and rows[2][1:] == ["60.0", ""]
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false"})
    assert srv.stats_log is None
