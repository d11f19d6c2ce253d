#!/usr/bin/env python3
"""Concurrent sessions per GPU through the whole serving stack (BASELINE metric "concurrent
sessions/node"; config "8 concurrent 1080p60 WebRTC sessions").

K session processes share one GPU, as K desktops would: each runs the paced 1080p60 HIP
pipeline, the aiohttp server and one headless viewer (WebRTC: WHEP + ICE-lite + DTLS-SRTP
over UDP loopback, or the WebSocket transport).  Each child reports the frame rate its
viewer received and the render-start -> access-unit-at-client latency; the parent prints one
JSON line with the aggregate (every session within 1 fps of the target = sustained).

    python tools/bench_density.py --sessions 8 --frames 600 [--transport webrtc|ws]

Processes that touch the GPU are capped at 16 on the test boxes: keep --sessions <= 12.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def child(a) -> None:
    os.environ["MXDESK_WEBRTC_HOST"] = "127.0.0.1"
    from mxdesk.pipeline.stream import StreamPipeline
    from mxdesk.server.app import MediaServer, serve
    from mxdesk.server.client import view
    from mxdesk.server.whep_client import whep_view
    from mxdesk.utils import config as C

    cfg = C.load(env={"ENABLE_BASIC_AUTH": "false", "SIZEW": str(a.width), "SIZEH": str(a.height),
                      "REFRESH": str(a.fps), "MXDESK_AUDIO_SOURCE": "none", "MXDESK_GAMEPAD": "false"}, argv=[])
    pipe = StreamPipeline(a.width, a.height, a.fps, backend=a.backend, device=0, bitrate_kbps=a.bitrate_kbps,
                          session_name=str(a.index))
    srv = MediaServer(pipe, cfg)

    loss: dict = {}

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            await asyncio.sleep(a.start_at - time.time())  # all sessions start their viewers together
            t0 = time.monotonic()
            if a.transport == "webrtc":
                r = await whep_view(f"http://127.0.0.1:{port}/whep", a.frames, timeout=a.frames / a.fps + 60)
                lat = [(t - tc) / 1000.0 for t, tc in zip(r.arrival_us, _capture_times(r))]
                n = len(r.aus)
                loss.update(nacked=r.nacked, recovered=r.recovered, gave_up=r.gave_up)
                if n > 1:  # frame rate over the received stream (excludes ICE/DTLS setup)
                    return n, (r.arrival_us[-1] - r.arrival_us[0]) / 1e6 * n / (n - 1), lat
            else:
                r = await view(f"http://127.0.0.1:{port}/mxws", a.frames, ack=False, timeout=a.frames / a.fps + 60)
                lat = list(r.latency_ms)
                n = len(r.frames)
            elapsed = time.monotonic() - t0
            return n, elapsed, lat
        finally:
            await runner.cleanup()

    def _capture_times(r):
        # RTP timestamp = (t_capture - ts0) * 90 kHz, ts0 = capture time of the first frame sent
        first = srv.whep.last_peer.ts0
        return [first + ts * 100 // 9 for ts in r.rtp_ts]

    n, elapsed, lat = asyncio.run(go())
    # the first frames include connection setup / IDR; report the steady state
    steady = lat[a.fps:] if len(lat) > 2 * a.fps else lat
    print(json.dumps({"index": a.index, "frames": n, "fps": n / elapsed,
                      "p50_ms": statistics.median(steady), "p95_ms": sorted(steady)[int(0.95 * (len(steady) - 1))],
                      "gpu_ms_p50": pipe.metrics.summary().get("encode_ms_p50"), **loss}), flush=True)


def parent(a) -> None:
    start_at = time.time() + 25.0 + 1.5 * a.sessions  # time for every child to import torch, build and serve
    procs = []
    for i in range(a.sessions):
        cmd = [sys.executable, __file__, "--child", "--index", str(i), "--start-at", str(start_at),
               "--frames", str(a.frames), "--width", str(a.width), "--height", str(a.height), "--fps", str(a.fps),
               "--bitrate-kbps", str(a.bitrate_kbps), "--transport", a.transport, "--backend", a.backend]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res, errs = [], []
    for p in procs:
        out, err = p.communicate(timeout=a.frames / a.fps + 240)
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            errs.append(err[-2000:])
            continue
        res.append(json.loads(lines[-1]))
    if errs:
        print(json.dumps({"error": "session failed", "failed": len(errs), "stderr": errs[0]}))
        sys.exit(1)
    fps = [r["fps"] for r in res]
    print(json.dumps({
        "metric": "concurrent 1080p60 sessions per GPU through the serving stack",
        "transport": a.transport, "sessions": a.sessions, "frames_per_session": a.frames,
        "min_session_fps": round(min(fps), 2), "mean_session_fps": round(statistics.mean(fps), 2),
        "sustained_target_fps": all(f >= a.fps - 1.0 for f in fps),
        "p50_e2e_latency_ms": round(statistics.median([r["p50_ms"] for r in res]), 3),
        "p95_e2e_latency_ms_worst": round(max(r["p95_ms"] for r in res), 3),
        "resolution": f"{a.width}x{a.height}@{a.fps}", "bitrate_kbps": a.bitrate_kbps,
        "data": "synthetic HIP-rendered desktop", "per_session": res}))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=8)
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fps", type=int, default=60)
    ap.add_argument("--bitrate-kbps", type=int, default=8000)
    ap.add_argument("--transport", default="webrtc", choices=["webrtc", "ws"])
    ap.add_argument("--backend", default="gpu", help="gpu (HIP encoder) | cpu (plumbing check without a GPU)")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--index", type=int, default=0)
    ap.add_argument("--start-at", type=float, default=0.0)
    a = ap.parse_args()
    if a.sessions > 12 and not a.child:
        ap.error("at most 12 GPU processes per box")
    (child if a.child else parent)(a)


if __name__ == "__main__":
    main()
