#!/usr/bin/env python3
"""End-to-end latency through the whole serving stack on one GPU (BASELINE metric "p50
end-to-end latency"): the paced 1080p60 GPU pipeline -> aiohttp server -> WebSocket (MXV1)
-> headless client on the same host (shared CLOCK_MONOTONIC), and the same session over
WebRTC (WHEP + DTLS-SRTP + RTP over UDP loopback).  Latency = frame render start -> complete
access unit received by the client.  Prints one JSON line."""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fps", type=int, default=60)
    ap.add_argument("--bitrate-kbps", type=int, default=8000)
    ap.add_argument("--backend", default="gpu")
    a = ap.parse_args()
    os.environ["MXDESK_WEBRTC_HOST"] = "127.0.0.1"

    from mxdesk.pipeline.stream import StreamPipeline
    from mxdesk.server.app import MediaServer, serve
    from mxdesk.server.client import view
    from mxdesk.server.whep_client import whep_view
    from mxdesk.utils import config as C

    cfg = C.load(env={"ENABLE_BASIC_AUTH": "false", "SIZEW": str(a.width), "SIZEH": str(a.height),
                      "REFRESH": str(a.fps), "MXDESK_AUDIO_SOURCE": "none"}, argv=[])
    pipe = StreamPipeline(a.width, a.height, a.fps, backend=a.backend, bitrate_kbps=a.bitrate_kbps)
    srv = MediaServer(pipe, cfg)

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            await asyncio.sleep(0.5)
            t0 = time.monotonic()
            ws = await view(f"http://127.0.0.1:{port}/mxws", a.frames, ack=False, timeout=a.frames / a.fps + 60)
            ws_elapsed = time.monotonic() - t0
            rtc = await whep_view(f"http://127.0.0.1:{port}/whep", min(a.frames, 300), timeout=a.frames / a.fps + 60)
            return ws, ws_elapsed, rtc
        finally:
            await runner.cleanup()

    ws, ws_elapsed, rtc = asyncio.run(go())
    lat = ws.latency_ms[10:]
    out = {
        "metric": "end-to-end latency through the serving stack (render start -> AU at client), paced",
        "config": f"{a.width}x{a.height}@{a.fps} H.264 CBR {a.bitrate_kbps} kbps, {a.backend} encoder",
        "websocket": {"frames": len(ws.frames), "fps": round(len(ws.frames) / ws_elapsed, 2),
                      "p50_ms": round(statistics.median(lat), 3), "p95_ms": round(sorted(lat)[int(0.95 * (len(lat) - 1))], 3),
                      "max_ms": round(max(lat), 3)},
    }
    peer = srv.whep.last_peer
    if rtc.arrival_us and peer is not None and peer.ts0 is not None:
        # RTP timestamp = (t_capture - ts0) * 90 kHz with ts0 = capture time of the first frame sent
        rl = [(arr - (peer.ts0 + ts * 100 // 9)) / 1000.0 for ts, arr in zip(rtc.rtp_ts, rtc.arrival_us)][10:]
        out["webrtc"] = {"frames": len(rtc.aus), "p50_ms": round(statistics.median(rl), 3),
                         "p95_ms": round(sorted(rl)[int(0.95 * (len(rl) - 1))], 3),
                         "connect_ms": round(rtc.connect_ms, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
