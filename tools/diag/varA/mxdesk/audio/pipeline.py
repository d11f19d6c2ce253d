"""Audio capture thread + subscriber fan-out (same drop policy as the video pipeline)."""
from __future__ import annotations

import asyncio
import logging
import math
import os
import shutil
import struct
import subprocess
import threading
import time
from dataclasses import dataclass

import numpy as np

log = logging.getLogger("mxdesk.audio")

RATE = 48000
CHANNELS = 2
CHUNK_MS = 10
CHUNK_FRAMES = RATE * CHUNK_MS // 1000


@dataclass
class AudioChunk:
    seq: int
    t_capture_us: int
    pcm: np.ndarray  # int16 [frames * channels] interleaved


class SyntheticTone:
    """Deterministic test signal: a 440 Hz tone whose amplitude steps every second, plus a
    1 kHz 'tick' during the first 10 ms of every second (A/V-sync checks against the video
    barcode timestamps)."""

    def __init__(self, rate: int = RATE, channels: int = CHANNELS):
        self.rate, self.channels, self.n = rate, channels, 0

    def read(self, frames: int) -> np.ndarray:
        t = (self.n + np.arange(frames)) / self.rate
        sec = np.floor(t)
        amp = 4000 + 2000 * (sec % 4)
        x = amp * np.sin(2 * math.pi * 440 * t)
        tick = (t - sec) < 0.010
        x = np.where(tick, 12000 * np.sin(2 * math.pi * 1000 * t), x)
        self.n += frames
        return np.repeat(x.astype(np.int16), self.channels)

    def close(self) -> None:
        pass


class PipeSource:
    """Raw s16le interleaved PCM from a subprocess (``parec``) or a FIFO/file."""

    def __init__(self, cmd: list[str] | None = None, path: str | None = None, channels: int = CHANNELS):
        self.channels = channels
        self.proc = None
        if cmd:
            self.proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
            self.f = self.proc.stdout
        else:
            self.f = open(path, "rb")

    def read(self, frames: int) -> np.ndarray:
        need = frames * self.channels * 2
        buf = b""
        while len(buf) < need:
            b = self.f.read(need - len(buf))
            if not b:
                raise EOFError("audio source ended")
            buf += b
        return np.frombuffer(buf, dtype="<i2").copy()

    def close(self) -> None:
        if self.proc is not None:
            self.proc.terminate()
        self.f.close()


def make_source(spec: str = "auto"):
    """``auto`` (PulseAudio via parec if available, else none), ``pulse``, ``synthetic``,
    ``fifo:/path``, ``none``."""
    spec = (spec or "auto").strip()
    if spec == "none":
        return None
    if spec == "synthetic":
        return SyntheticTone()
    if spec.startswith("fifo:") or spec.startswith("file:"):
        return PipeSource(path=spec.split(":", 1)[1])
    if spec in ("auto", "pulse"):
        parec = shutil.which("parec")
        if parec:
            dev = os.environ.get("MXDESK_PULSE_DEVICE")
            cmd = [parec, "--raw", "--format=s16le", f"--rate={RATE}", f"--channels={CHANNELS}", "--latency-msec=10"]
            if dev:
                cmd.append(f"--device={dev}")
            return PipeSource(cmd=cmd)
        if spec == "pulse":
            raise FileNotFoundError("parec (pulseaudio-utils) not installed")
        return None
    raise ValueError(f"unknown audio source {spec!r}")


class _Sub:
    def __init__(self, loop: asyncio.AbstractEventLoop, maxsize: int = 50):
        self.loop = loop
        self.queue: asyncio.Queue = asyncio.Queue(maxsize=maxsize)
        self.dropped = 0

    def push(self, ch: AudioChunk) -> None:
        def put():
            if self.queue.full():  # late consumer: drop the oldest 10 ms
                self.queue.get_nowait()
                self.dropped += 1
            self.queue.put_nowait(ch)

        try:
            self.loop.call_soon_threadsafe(put)
        except RuntimeError:
            pass


class AudioPipeline:
    """Reads CHUNK_MS chunks from the source on a thread (paced for sources that are not
    clocked themselves) and fans them out to asyncio subscribers."""

    def __init__(self, source, paced: bool | None = None):
        self.source = source
        self.paced = isinstance(source, SyntheticTone) if paced is None else paced
        self._subs: list[_Sub] = []
        self._lock = threading.Lock()
        self._thread: threading.Thread | None = None
        self._stop = threading.Event()
        self.chunks = 0

    @staticmethod
    def now_us() -> int:
        return time.monotonic_ns() // 1000

    def subscribe(self, loop: asyncio.AbstractEventLoop) -> _Sub:
        s = _Sub(loop)
        with self._lock:
            self._subs.append(s)
        return s

    def unsubscribe(self, s: _Sub) -> None:
        with self._lock:
            if s in self._subs:
                self._subs.remove(s)

    def start(self) -> None:
        if self._thread is None and self.source is not None:
            self._stop.clear()
            self._thread = threading.Thread(target=self._run, name="mxdesk-audio", daemon=True)
            self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2)
            self._thread = None
        if self.source is not None:
            self.source.close()

    def _run(self) -> None:
        t0 = time.monotonic()
        while not self._stop.is_set():
            try:
                pcm = self.source.read(CHUNK_FRAMES)
            except (EOFError, OSError) as e:
                log.warning("audio source stopped: %s", e)
                return
            ch = AudioChunk(self.chunks, self.now_us(), pcm)
            self.chunks += 1
            with self._lock:
                subs = list(self._subs)
            for s in subs:
                s.push(ch)
            if self.paced:
                delay = t0 + self.chunks * CHUNK_MS / 1000.0 - time.monotonic()
                if delay > 0:
                    time.sleep(delay)


# WebSocket audio message: "MXA1" | u8 codec (1 = s16le PCM) | u8 channels | u16 rate/100 |
# u32 seq | u64 t_capture_us | u32 payload bytes | payload
AUDIO_HDR = struct.Struct("<4sBBHIQI")


def audio_message(ch: AudioChunk) -> bytes:
    payload = ch.pcm.astype("<i2").tobytes()
    return AUDIO_HDR.pack(b"MXA1", 1, CHANNELS, RATE // 100, ch.seq & 0xFFFFFFFF, ch.t_capture_us, len(payload)) + payload


def parse_audio_message(msg: bytes) -> dict:
    magic, codec, chans, rate100, seq, tcap, n = AUDIO_HDR.unpack_from(msg)
    if magic != b"MXA1":
        raise ValueError("not an audio message")
    pcm = np.frombuffer(msg[AUDIO_HDR.size:AUDIO_HDR.size + n], dtype="<i2")
    return {"codec": codec, "channels": chans, "rate": rate100 * 100, "seq": seq, "t_capture_us": tcap, "pcm": pcm}
