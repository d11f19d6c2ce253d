"""Headless viewer (test + benchmark harness, SURVEY.md §4.2 integration tier).

Connects to ``/mxws``, receives N access units, optionally decodes them with the
reference decoder and checks the embedded frame-id barcode, and reports end-to-end
latency (capture timestamp -> receipt; valid when client and server share the host
clock, as in loopback tests and benches).
"""
from __future__ import annotations

import asyncio
import base64
import json
import statistics
import time
from dataclasses import dataclass, field

import aiohttp

from ..audio.pipeline import parse_audio_message
from ..pipeline.stream import parse_frame


@dataclass
class ViewerResult:
    config: dict = field(default_factory=dict)
    frames: list[dict] = field(default_factory=list)
    latency_ms: list[float] = field(default_factory=list)
    stream: bytes = b""
    audio: list[dict] = field(default_factory=list)  # parsed MXA1 chunks (PCM)

    @property
    def p50_ms(self) -> float:
        return statistics.median(self.latency_ms) if self.latency_ms else float("nan")


async def view(url: str, nframes: int, user: str | None = None, password: str | None = None,
               send: list[str] | None = None, timeout: float = 60.0, ack: bool = True) -> ViewerResult:
    headers = {}
    if user is not None:
        headers["Authorization"] = "Basic " + base64.b64encode(f"{user}:{password}".encode()).decode()
    res = ViewerResult()
    async with aiohttp.ClientSession(headers=headers) as s:
        async with s.ws_connect(url, max_msg_size=64 * 1024 * 1024, timeout=aiohttp.ClientWSTimeout(ws_close=timeout)) as ws:
            deadline = time.monotonic() + timeout
            for m in send or []:
                await ws.send_str(m)
            while len(res.frames) < nframes and time.monotonic() < deadline:
                msg = await ws.receive(timeout=max(0.1, deadline - time.monotonic()))
                if msg.type == aiohttp.WSMsgType.TEXT:
                    d = json.loads(msg.data)
                    if d.get("type") == "config":
                        res.config = d
                elif msg.type == aiohttp.WSMsgType.BINARY:
                    t_recv = time.monotonic() * 1e6
                    if msg.data[:4] == b"MXA1":
                        res.audio.append(parse_audio_message(msg.data))
                        continue
                    fr = parse_frame(msg.data)
                    lat = (t_recv - fr["t_capture_us"]) / 1000.0
                    res.latency_ms.append(lat)
                    res.frames.append({k: v for k, v in fr.items() if k != "au"})
                    res.stream += fr["au"]
                    if ack:
                        await ws.send_str(json.dumps({"type": "ack", "frame_id": fr["frame_id"], "latency_ms": lat}))
                elif msg.type in (aiohttp.WSMsgType.CLOSED, aiohttp.WSMsgType.ERROR):
                    break
    return res


def view_sync(url: str, nframes: int, **kw) -> ViewerResult:
    return asyncio.run(view(url, nframes, **kw))
