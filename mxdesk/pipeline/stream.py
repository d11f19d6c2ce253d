"""Streaming pipeline: paced frame production + fan-out to viewers.

A ``StreamPipeline`` owns one encoder session (GPU: the native HIP session; CPU: numpy
desktop + CPU H.264 encoder for the plumbing configuration), produces frames at the stream
rate on a dedicated thread and pushes each encoded access unit to every subscriber queue
(asyncio-safe).  Policies:
  * a new viewer or a PLI/keyframe request forces an IDR on the next frame -- through the
    session's ``KeyframeCoalescer``: requests arriving while an IDR is pending or just sent join
    it, and forced IDRs are at least ``MXDESK_IDR_MIN_INTERVAL`` (0.25 s) apart;
  * a viewer whose queue overflows is resynchronised: its backlog is dropped, it waits for the
    next IDR and the pipeline requests one (counted in ``mxdesk_dropped_frames``; without the
    request such a viewer received nothing more -- no gap to NACK, no PLI -- until the
    stream's next key frame: the stalls of the 96-viewer density runs, profiles/r05_density);
    a viewer that overflows again before draining asks with an exponential backoff;
  * a watchdog restarts the encoder session if no frame was produced for ``stall_s``;
  * ``MXDESK_FAULT`` (tests only) injects failures: ``drop:N`` drops every Nth frame,
    ``stall:S`` stalls the producer once for S seconds, ``crash:N`` raises at frame N.
"""
from __future__ import annotations

import asyncio
import logging
import math
import os
import threading
import time
from dataclasses import dataclass
from typing import Any, Callable

import numpy as np

from ..models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12
from ..utils.metrics import SessionMetrics

log = logging.getLogger("mxdesk.pipeline")


@dataclass
class EncodedFrame:
    frame_id: int
    t_capture_us: int   # CLOCK_MONOTONIC us
    t_encoded_us: int
    idr: bool
    qp: int
    au: bytes
    width: int
    height: int
    gpu_ms: float = 0.0
    codec_id: int = 1  # media header codec byte: 1 = H.264, 2 = HEVC, 3 = VP8


def hevc_codec_string(width: int, height: int, fps: int) -> str:
    """WebCodecs/RFC 6381 codec id of our Main-profile HEVC stream (hvc1.1.6.L<level>.B0)."""
    from .. import native

    return f"hvc1.1.6.L{native().hevc_level(width, height, fps)}.B0"


CODEC_IDS = {"h264": 1, "hevc": 2, "vp8": 3}


def codec_string(codec: str, width: int, height: int, fps: int) -> str:
    if codec == "vp8":
        return "vp8"  # WebCodecs codec string of VP8
    return hevc_codec_string(width, height, fps) if codec == "hevc" else h264_codec_string(width, height, fps)


def cpu_encoder_class(N, codec: str):
    """The serial CPU encoder of a codec (no-GPU plumbing backend, CPU wall tiles)."""
    return {"h264": N.CpuH264Encoder, "hevc": N.CpuHevcEncoder, "vp8": N.CpuVp8Encoder}[codec]


def h264_codec_string(width: int, height: int, fps: int) -> str:
    """WebCodecs/RFC 6381 codec id of our Constrained Baseline stream (avc1.42C0LL)."""
    from .. import native

    mbs = ((width + 15) // 16) * ((height + 15) // 16)
    level = native().h264.level_for(mbs, fps)
    return f"avc1.42C0{level:02X}"


class KeyframeCoalescer:
    """Per-session keyframe-request coalescer (ADVICE r5 stream.py:323).

    Every source of a forced IDR -- RTCP PLI / FIR, the WebSocket client's ``pli``, a new viewer,
    a viewer whose queue overflowed, an encoder restart -- goes through :meth:`request`.  An IDR
    costs about five frame-times of link time at CBR (the IDR budget, h264_encoder.h), and a
    burst of PLIs (every viewer of a lossy link, a browser repeating its request until a key frame
    arrives) used to code one IDR per request.  The rules:

      * a request while an IDR is already pending (requested, not yet coded) joins it;
      * a PLI / FIR / client request within ``cover`` (0.1 s: about a round trip plus a frame) of
        the last IDR is covered by that IDR (it was sent before the viewer received it) and is
        dropped; a later one reports a loss after the IDR and schedules a new one;
      * a request that needs a *new* key frame (a new viewer, a resynchronising viewer) is kept
        but not coded before ``last IDR + min_interval``, so the IDR rate of a session is bounded
        by 1 / min_interval whatever the viewers do;
      * any IDR the encoder codes (periodic, first frame, forced) satisfies what is pending.

    ``min_interval`` defaults to ``MXDESK_IDR_MIN_INTERVAL`` seconds (0.25: four IDRs per second at
    most), ``cover`` to ``MXDESK_IDR_COVER`` seconds (at most ``min_interval``).  Counts per reason, coalesced requests and forced IDRs are exported on ``/metrics``.
    The reference has no equivalent: ``nvh264enc`` codes an IDR per upstream force-key-unit event
    (reference Dockerfile:210, selkies-gstreamer [UP])."""

    COVERED_BY_RECENT = ("pli", "fir", "client")

    def __init__(self, min_interval_s: float | None = None, clock: Callable[[], float] = time.monotonic,
                 metrics: SessionMetrics | None = None, cover_s: float | None = None):
        if min_interval_s is None:
            min_interval_s = float(os.environ.get("MXDESK_IDR_MIN_INTERVAL", "") or 0.25)
        self.min_interval = max(0.0, float(min_interval_s))
        if cover_s is None:
            cover_s = float(os.environ.get("MXDESK_IDR_COVER", "") or 0.1)
        self.cover = min(max(0.0, float(cover_s)), self.min_interval)
        self.clock = clock
        self.metrics = metrics
        self._lock = threading.Lock()
        self.pending = False
        self.not_before = 0.0
        self.last_idr_t = -math.inf
        self.requests: dict[str, int] = {}
        self.coalesced = 0
        self.forced = 0

    def request(self, reason: str = "api") -> bool:
        """Ask for a key frame; returns True if this request scheduled one (False: it joined a
        pending IDR or was covered by the one just coded)."""
        now = self.clock()
        with self._lock:
            self.requests[reason] = self.requests.get(reason, 0) + 1
            joined = self.pending or (reason in self.COVERED_BY_RECENT and now - self.last_idr_t < self.cover)
            if joined:
                self.coalesced += 1
            else:
                self.pending = True
                self.not_before = self.last_idr_t + self.min_interval
        if self.metrics is not None:
            self.metrics.on_keyframe_request(reason, joined)
        return not joined

    def take(self) -> bool:
        """Producer, once per frame: True if this frame must be coded as an IDR."""
        with self._lock:
            if self.pending and self.clock() >= self.not_before:
                self.pending = False
                self.forced += 1
                return True
            return False

    def on_idr(self) -> None:
        """An IDR was coded (forced or not): it satisfies every pending request."""
        with self._lock:
            self.last_idr_t = self.clock()
            self.pending = False

    def snapshot(self) -> dict:
        with self._lock:
            return {"requests": dict(self.requests), "coalesced": self.coalesced, "forced": self.forced,
                    "pending": self.pending, "min_interval_s": self.min_interval, "cover_s": self.cover}


class _Subscriber:
    # a viewer that keeps overflowing (a stalled socket) asks for its resynchronising IDR with an
    # exponential backoff: 0, 0.5, 1, 2, 4 s after its previous one; reset once it drains
    BACKOFF_S = (0.0, 0.5, 1.0, 2.0, 4.0)

    def __init__(self, loop: asyncio.AbstractEventLoop, maxsize: int):
        self.loop = loop
        self.queue: asyncio.Queue = asyncio.Queue(maxsize=maxsize)
        self.need_idr = True
        self.dropped = 0
        self.overflows = 0        # consecutive overflows without the viewer reading in between
        self.last_resync_t = -math.inf
        self._queued = 0          # frames put since the queue was last cleared
        self.resync_at: float | None = None  # backed-off resynchronising IDR request, due then

    def offer(self, fr: EncodedFrame, on_drop: Callable[["_Subscriber", int], None]) -> None:
        def put():
            if self.need_idr and not fr.idr:
                return
            if self.queue.full():
                n = self.queue.qsize()
                while not self.queue.empty():
                    self.queue.get_nowait()
                self.dropped += n
                self.need_idr = True
                self._queued = 0
                on_drop(self, n)
                return
            self.need_idr = False
            if self.queue.qsize() < self._queued:
                self.overflows = 0  # the viewer reads its queue again
            self._queued = self.queue.qsize() + 1
            self.queue.put_nowait(fr)

        try:
            self.loop.call_soon_threadsafe(put)
        except RuntimeError:
            pass  # loop closed


class StreamPipeline:
    def __init__(self, width: int, height: int, fps: int, *, backend: str = "gpu", device: int = 0,
                 bitrate_kbps: int = 8000, keyint: int = 0, search_range: int = 16, subpel: bool = True,
                 noise: bool = True, out_width: int = 0, out_height: int = 0, session_name: str = "0",
                 capture: Any = None, metrics: SessionMetrics | None = None, queue_frames: int | None = None,
                 stall_s: float = 2.0, paced: bool = True, codec: str = "h264",
                 idr_min_interval_s: float | None = None):
        if codec not in CODEC_IDS:
            raise ValueError(f"unknown codec {codec!r} (h264 | hevc | vp8)")
        self.codec = codec
        self.codec_id = CODEC_IDS[codec]
        self.width, self.height, self.fps = width, height, fps
        self.out_w = out_width or width
        self.out_h = out_height or height
        self.backend = backend
        self.device = device
        self.capture = capture
        self.metrics = metrics or SessionMetrics(session_name)
        # frames a viewer may fall behind before it is resynchronised (MXDESK_VIEWER_QUEUE; 16 =
        # 267 ms at 60 fps: 8 resynchronised viewers of busy serve processes, profiles/r05_density)
        self.queue_frames = int(queue_frames or os.environ.get("MXDESK_VIEWER_QUEUE", "") or 16)
        self.stall_s = stall_s
        self.paced = paced
        self.bitrate_kbps = bitrate_kbps  # configured CBR target (congestion control upper bound)
        self._enc_args = dict(bitrate_kbps=bitrate_kbps, keyint=keyint, search_range=search_range, subpel=subpel,
                              noise=noise)
        self._subs: list[_Subscriber] = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.keyframes = KeyframeCoalescer(idr_min_interval_s, metrics=self.metrics)
        self.keyframes.request("viewer")  # the first frame is an IDR anyway
        self._pending_bitrate: int | None = None
        self._cursor = (-1, -1)
        self._pending_resize: tuple[int, int] | None = None
        self.resizes = 0
        self.frames_out = 0
        self.last_frame_t = 0.0
        self.restarts = 0
        self.last_error: str | None = None
        self._fault = self._parse_fault(os.environ.get("MXDESK_FAULT", ""))
        # damage-driven frame rate (captures with XDamage only): frames without damage after which
        # production pauses (0: never), and the longest pause (MXDESK_IDLE_AFTER / _HEARTBEAT_S)
        self.idle_after = int(os.environ.get("MXDESK_IDLE_AFTER", "") or 30)
        self.idle_heartbeat_s = float(os.environ.get("MXDESK_IDLE_HEARTBEAT_S", "") or 1.0)
        self.frames_idle = 0
        self._static_frames = 0
        self._idle_cursor = self._cursor
        self._last_produced_t = 0.0
        self._make_session()

    # ------------------------------------------------------------------ session backends
    @staticmethod
    def _parse_fault(spec: str) -> dict[str, float]:
        out = {}
        for part in spec.split(","):
            if ":" in part:
                k, v = part.split(":", 1)
                out[k.strip()] = float(v)
        return out

    def _make_session(self) -> None:
        a = self._enc_args
        if self.backend == "gpu":
            from .. import native

            N = native()
            N.set_device(self.device)
            cfg = N.SessionConfig()
            cfg.width, cfg.height, cfg.fps = self.width, self.height, self.fps
            cfg.out_width, cfg.out_height = self.out_w, self.out_h
            cfg.noise = 1 if a["noise"] else 0
            cfg.enc.bitrate_kbps = a["bitrate_kbps"]
            cfg.enc.keyint = a["keyint"]
            cfg.enc.search_range = a["search_range"]
            cfg.enc.subpel = 1 if a["subpel"] else 0
            cfg.codec = self.codec
            self._sess = N.Session(cfg)
            self._cpu = None
        elif self.backend == "cpu":
            from .. import native

            N = native()
            if (self.out_w, self.out_h) != (self.width, self.height):
                raise ValueError("the CPU plumbing backend does not scale")
            ec = N.EncoderConfig()
            ec.width, ec.height, ec.fps = self.width, self.height, self.fps
            ec.bitrate_kbps = a["bitrate_kbps"]
            ec.keyint = a["keyint"]
            ec.search_range = min(a["search_range"], 4)  # keep the serial encoder real-time
            ec.subpel = 0
            self._cpu = cpu_encoder_class(N, self.codec)(ec)
            self._desk = CpuSyntheticDesktop(self.width, self.height, a["noise"])
            self._sess = None
            self._cpu_frame = 0
        else:
            raise ValueError(f"unknown backend {self.backend}")

    def _idle_skip(self, bands, force_idr: bool) -> bool:
        """Damage-driven frame rate: after ``idle_after`` consecutive frames without damage
        (the encoder has refined the still picture by then) no frame is produced until the
        screen or the cursor changes, a key frame is asked for, or ``idle_heartbeat_s`` passed
        since the last frame (receivers keep statistics and liveness).  An idle desktop then
        costs no GPU work and no link bandwidth; receivers keep showing the last picture."""
        cursor = self._cursor
        if bands or force_idr or cursor != self._idle_cursor:
            self._static_frames = 0
            self._idle_cursor = cursor
            return False
        self._static_frames += 1
        now = time.monotonic()
        if (self.idle_after > 0 and self._static_frames > self.idle_after
                and now - self._last_produced_t < self.idle_heartbeat_s):
            self.frames_idle += 1
            self.metrics.on_idle()
            return True
        return False

    def _produce(self, force_idr: bool) -> EncodedFrame | None:
        from .. import native

        if self._pending_bitrate is not None:
            (self._sess or self._cpu).set_bitrate(self._pending_bitrate)
            self._pending_bitrate = None
        if self._sess is not None:
            s = self._sess
            s.set_cursor(*self._cursor)
            if self.capture is not None:
                # zero-copy when the capture lands in a registered MIT-SHM segment: the GPU DMAs
                # the frame straight out of it (no CPU copy into the staging buffer)
                shm = getattr(self.capture, "shm_buffer", lambda: None)()
                if shm is not None and (getattr(self.capture, "w", self.width), getattr(self.capture, "h", self.height)) \
                        != (self.width, self.height):
                    shm = None  # capture resized but the session not yet: copy path (size-checked)
                if shm is not None and getattr(self, "_shm_reg", None) != shm:
                    try:
                        s.register_host_buffer(*shm)
                        self._shm_reg = shm
                    except RuntimeError as e:  # page-locking refused: keep the staging copy path
                        log.warning("register_host_buffer failed (%s); using the staging copy", e)
                        shm = None
                        self.capture_zero_copy = False
                dmg = getattr(self.capture, "damage", None) if shm is not None else None
                if dmg is not None:
                    # damage-driven: the X server copies and the GPU DMAs only the changed bands
                    # (into the session's device-resident screen; its first frame is whole)
                    if getattr(self, "_damage_sess", None) is not s:
                        self._damage_sess = s  # new session (resize / restart): whole frame
                        dmg.invalidate()
                        s.invalidate_screen()
                    addr, pitch, bands = self.capture.grab_shm_damage()
                    self.metrics.on_capture_rows(sum(y1 - y0 for y0, y1 in bands))
                    if self._idle_skip(bands, force_idr):
                        return None
                    s.submit_bgrx_damage(addr, pitch, shm[1] - (addr - shm[0]), bands, force_idr)
                elif shm is not None and getattr(self, "capture_zero_copy", True):
                    addr, pitch = self.capture.grab_shm()
                    s.submit_bgrx_ptr(addr, pitch, shm[1] - (addr - shm[0]), force_idr)
                else:
                    s.submit_bgrx(self.capture.grab(), force_idr)
                r = s.collect()
            else:
                r = s.step(force_idr)
            return EncodedFrame(r.frame_id, r.t_capture_us, r.t_encoded_us, bool(r.idr), r.qp, r.au, self.out_w,
                                self.out_h, r.gpu_ms, self.codec_id)
        t_cap = native().now_us()
        fid = self._cpu_frame
        self._cpu_frame += 1
        self._desk.cursor = self._cursor
        img = self.capture.grab() if self.capture is not None else self._desk.render(fid, fid / self.fps,
                                                                                     t_cap & 0xFFFFFFFF)
        y, uv = bgrx_to_nv12(img)
        au = self._cpu.encode(y, uv, force_idr)
        st = self._cpu.stats
        return EncodedFrame(fid, t_cap, native().now_us(), bool(st.idr), st.qp, au, self.width, self.height,
                            codec_id=self.codec_id)

    # ------------------------------------------------------------------ control
    def request_idr(self, reason: str = "api") -> bool:
        """Ask for a key frame (PLI / FIR / a client request / a new viewer ...); requests are
        coalesced and rate-limited per session (KeyframeCoalescer)."""
        return self.keyframes.request(reason)

    def set_bitrate(self, kbps: int) -> None:
        self._pending_bitrate = int(max(100, min(kbps, 200_000)))

    def set_fps(self, fps: float) -> None:
        """Client frame-rate request (selkies ``_f,fps``): changes the pacing only; the
        stream's VUI timing stays at the session rate."""
        self.pace_fps = float(max(1.0, min(float(fps), 240.0)))

    def resize(self, width: int, height: int) -> tuple[int, int]:
        """Client-driven resize (``WEBRTC_ENABLE_RESIZE``): the next frame is produced by a new
        session at the (sanitised) size, starting with an IDR; returns that size.  The
        desktop and the encoded stream both take the new size (the X screen is resized by
        the caller through RandR)."""
        from ..display.randr import clamp_size

        w, h = clamp_size(width, height)
        self._pending_resize = (w, h)
        return w, h

    def _apply_resize(self, w: int, h: int) -> None:
        if (w, h) == (self.width, self.height) and (self.out_w, self.out_h) == (w, h):
            return
        if self.capture is not None and hasattr(self.capture, "resize"):
            self.capture.resize(w, h)
        self.width, self.height = w, h
        self.out_w, self.out_h = w, h
        self._make_session()
        self.keyframes.request("resize")
        self.resizes += 1
        log.info("session resized to %dx%d", w, h)

    def set_cursor(self, x: int, y: int) -> None:
        self._cursor = (int(x), int(y))

    def subscribe(self, loop: asyncio.AbstractEventLoop | None = None) -> _Subscriber:
        sub = _Subscriber(loop or asyncio.get_event_loop(), self.queue_frames)
        with self._lock:
            self._subs.append(sub)
            self.metrics.set_clients(len(self._subs))
        self.request_idr("viewer")
        return sub

    def unsubscribe(self, sub: _Subscriber) -> None:
        with self._lock:
            if sub in self._subs:
                self._subs.remove(sub)
            self.metrics.set_clients(len(self._subs))

    @property
    def subscribers(self) -> int:
        with self._lock:
            return len(self._subs)

    # ------------------------------------------------------------------ loop
    def step(self) -> EncodedFrame | None:
        """Produce one frame synchronously (no pacing); publishes to subscribers.  None when the
        damage-driven capture reports an idle screen (``_idle_skip``)."""
        pending, self._pending_resize = self._pending_resize, None
        if pending is not None:
            self._apply_resize(*pending)
        self._due_resyncs()
        force = self.keyframes.take()
        n = self.frames_out
        if "crash" in self._fault and n == int(self._fault["crash"]):
            raise RuntimeError("injected encoder crash")
        if "stall" in self._fault and n == 3:
            time.sleep(self._fault.pop("stall"))
        fr = self._produce(force)
        self.last_frame_t = time.monotonic()  # the loop is alive (also while idle)
        if fr is None:  # idle: nothing changed on screen (damage-driven frame rate)
            return None
        self._last_produced_t = self.last_frame_t
        if fr.idr:
            self.keyframes.on_idr()
        self.frames_out += 1
        self.metrics.on_frame(len(fr.au), (fr.t_encoded_us - fr.t_capture_us) / 1000.0, fr.gpu_ms, fr.qp, fr.idr)
        if "drop" in self._fault and self.frames_out % int(self._fault["drop"]) == 0:
            self.metrics.on_drop()
            return fr
        with self._lock:
            subs = list(self._subs)
        for s in subs:
            s.offer(fr, self._on_sub_overflow)
        return fr

    def _on_sub_overflow(self, sub: _Subscriber, n: int) -> None:
        """A viewer's queue overflowed (event-loop thread): count the dropped frames and ask for an
        IDR so that viewer resynchronises at the next key frame.  The request goes through the
        session's coalescer (rate-bounded), and a viewer that overflows again before it drained
        asks with an exponential backoff (a stalled socket does not drive the session's IDR rate)."""
        self.metrics.on_drop(n)
        now = self.keyframes.clock()
        wait = sub.BACKOFF_S[min(sub.overflows, len(sub.BACKOFF_S) - 1)]
        sub.overflows += 1
        if now - sub.last_resync_t >= wait:
            sub.last_resync_t = now
            sub.resync_at = None
            self.request_idr("overflow")
        else:  # asked again when its backoff has passed (step() checks)
            sub.resync_at = sub.last_resync_t + wait
            self.metrics.on_keyframe_request("overflow_backoff", True)

    def _due_resyncs(self) -> None:
        now = self.keyframes.clock()
        with self._lock:
            due = [s for s in self._subs if s.resync_at is not None and now >= s.resync_at]
        for s in due:
            s.resync_at = None
            s.last_resync_t = now
            self.request_idr("overflow")

    def _run(self) -> None:
        # pacing phase (seconds into the frame period): sessions of one process start staggered
        # so their frames do not all reach the GPU in the same instant of every period
        next_t = time.monotonic() + float(getattr(self, "pace_phase", 0.0))
        if self.paced and next_t > time.monotonic():
            self._stop.wait(next_t - time.monotonic())
        while not self._stop.is_set():
            try:
                self.step()
            except Exception as e:  # encoder failure -> restart the session, force IDR
                self.last_error = repr(e)
                log.exception("frame production failed; restarting session")
                self.restarts += 1
                self._fault.pop("crash", None)
                try:
                    self._make_session()
                except Exception:
                    log.exception("session restart failed")
                self.request_idr("restart")
                self._stop.wait(min(2.0, 0.1 * self.restarts))  # back off on repeated failures
            if self.paced:
                next_t += 1.0 / (getattr(self, "pace_fps", None) or self.fps)
                delay = next_t - time.monotonic()
                if delay > 0:
                    self._stop.wait(delay)
                else:
                    next_t = time.monotonic()  # fell behind: do not burst

    def start(self) -> None:
        if self._thread is None:
            self._stop.clear()
            self._thread = threading.Thread(target=self._run, name="mxdesk-pipeline", daemon=True)
            self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    def healthy(self) -> bool:
        return self._thread is not None and (time.monotonic() - self.last_frame_t) < self.stall_s

    def status(self) -> dict:
        return {"backend": self.backend, "device": self.device, "width": self.out_w, "height": self.out_h,
                "fps": self.fps, "frames": self.frames_out, "clients": self.subscribers, "restarts": self.restarts,
                "last_error": self.last_error, "resizes": self.resizes, "keyframes": self.keyframes.snapshot(),
                "frames_idle": self.frames_idle,
                **self.metrics.summary()}


def frame_header(fr: EncodedFrame, t_send_us: int) -> bytes:
    """Binary media header of the WebSocket transport (36 bytes, little endian)."""
    import struct

    return struct.pack("<4sBBHIQQHHI", b"MXV1", 1 if fr.idr else 0, fr.codec_id, 0, fr.frame_id & 0xFFFFFFFF,
                       fr.t_capture_us, t_send_us, fr.width, fr.height, len(fr.au))


def parse_frame(msg: bytes) -> dict:
    import struct

    magic, flags, codec, _, fid, tcap, tsend, w, h, n = struct.unpack_from("<4sBBHIQQHHI", msg)
    if magic != b"MXV1":
        raise ValueError("bad media frame")
    return {"key": bool(flags & 1), "codec": codec, "frame_id": fid, "t_capture_us": tcap, "t_send_us": tsend,
            "width": w, "height": h, "au": msg[36:36 + n]}


def nv12_planes_equal(a: tuple[np.ndarray, np.ndarray], b: tuple[np.ndarray, np.ndarray]) -> bool:
    return all(np.array_equal(x, y) for x, y in zip(a, b))
