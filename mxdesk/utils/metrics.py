"""Metrics / observability.

The reference only has GStreamer debug logs (selkies-gstreamer-entrypoint.sh:18); selkies
can expose a metrics HTTP port [UP].  Here every session exports Prometheus series
(encoded FPS, per-stage latencies, bitrate, QP, clients, drops) on ``/metrics`` and keeps
rolling quantiles for the JSON status endpoint and the bench harness.
"""
from __future__ import annotations

import collections
import threading
import time

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

LAT_BUCKETS_MS = (0.1, 0.25, 0.5, 1, 2, 4, 8, 16, 33, 66, 133, 266, 533, 1000)


class Rolling:
    """Fixed-size window of samples with quantiles."""

    def __init__(self, n: int = 600):
        self.buf = collections.deque(maxlen=n)
        self.lock = threading.Lock()

    def add(self, v: float) -> None:
        with self.lock:
            self.buf.append(v)

    def quantile(self, q: float) -> float | None:
        with self.lock:
            if not self.buf:
                return None
            s = sorted(self.buf)
        return s[min(len(s) - 1, int(q * (len(s) - 1) + 0.5))]

    def __len__(self) -> int:
        return len(self.buf)


class SessionMetrics:
    def __init__(self, session: str = "0", registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        lab = ["session"]
        self.session = session
        self.frames = Counter("mxdesk_encoded_frames", "Encoded frames", lab, registry=self.registry)
        self.idr = Counter("mxdesk_idr_frames", "IDR frames", lab, registry=self.registry)
        self.bytes = Counter("mxdesk_encoded_bytes", "Encoded bytes", lab, registry=self.registry)
        self.dropped = Counter("mxdesk_dropped_frames", "Frames dropped for slow clients", lab,
                               registry=self.registry)
        self.encode_ms = Histogram("mxdesk_encode_latency_ms", "Capture -> access unit (ms)", lab,
                                   buckets=LAT_BUCKETS_MS, registry=self.registry)
        self.e2e_ms = Histogram("mxdesk_e2e_latency_ms", "Capture -> client receipt (ms)", lab,
                                buckets=LAT_BUCKETS_MS, registry=self.registry)
        self.gpu_ms = Histogram("mxdesk_gpu_encode_ms", "GPU encode time (ms)", lab, buckets=LAT_BUCKETS_MS,
                                registry=self.registry)
        self.kf_requests = Counter("mxdesk_keyframe_requests", "Keyframe requests by reason (pli, fir, client, viewer, "
                                   "overflow, overflow_backoff, restart, resize)", ["session", "reason"],
                                   registry=self.registry)
        self.kf_coalesced = Counter("mxdesk_keyframe_requests_coalesced", "Keyframe requests that joined a pending "
                                    "or just-coded IDR (or waited out a viewer's backoff)", lab,
                                    registry=self.registry)
        self.idle = Counter("mxdesk_idle_frames", "Frame ticks not encoded because the screen did not change "
                            "(damage-driven capture)", lab, registry=self.registry)
        self.capture_rows = Counter("mxdesk_capture_rows", "Screen rows grabbed and uploaded by the damage-driven "
                                    "capture", lab, registry=self.registry)
        self.qp = Gauge("mxdesk_qp", "Current QP", lab, registry=self.registry)
        self.bitrate = Gauge("mxdesk_bitrate_kbps", "Measured bitrate (kbps, 1 s window)", lab,
                             registry=self.registry)
        self.fps = Gauge("mxdesk_encoded_fps", "Encoded frames per second (1 s window)", lab, registry=self.registry)
        self.clients = Gauge("mxdesk_clients", "Connected viewers", lab, registry=self.registry)
        self.gpu = Gauge("mxdesk_gpu", "GPU telemetry from amdgpu sysfs (busy_percent, vram_used_bytes, "
                         "vram_total_bytes, power_watts, temperature_c)", ["session", "gpu", "metric"],
                         registry=self.registry)
        self.roll_encode = Rolling()
        self.roll_e2e = Rolling()
        self._win = collections.deque()
        self._lock = threading.Lock()

    def on_frame(self, nbytes: int, encode_ms: float, gpu_ms: float, qp: int, idr: bool) -> None:
        s = self.session
        self.frames.labels(s).inc()
        self.bytes.labels(s).inc(nbytes)
        if idr:
            self.idr.labels(s).inc()
        self.encode_ms.labels(s).observe(encode_ms)
        self.gpu_ms.labels(s).observe(gpu_ms)
        self.qp.labels(s).set(qp)
        self.roll_encode.add(encode_ms)
        now = time.monotonic()
        with self._lock:
            self._win.append((now, nbytes))
            while self._win and now - self._win[0][0] > 1.0:
                self._win.popleft()
            n = len(self._win)
            tot = sum(b for _, b in self._win)
        self.fps.labels(s).set(n)
        self.bitrate.labels(s).set(tot * 8 / 1000.0)

    def on_client_latency(self, ms: float) -> None:
        self.e2e_ms.labels(self.session).observe(ms)
        self.roll_e2e.add(ms)

    def on_keyframe_request(self, reason: str, coalesced: bool) -> None:
        self.kf_requests.labels(self.session, reason).inc()
        if coalesced:
            self.kf_coalesced.labels(self.session).inc()

    def on_idle(self) -> None:
        self.idle.labels(self.session).inc()

    def on_capture_rows(self, n: int) -> None:
        self.capture_rows.labels(self.session).inc(n)

    def on_drop(self, n: int = 1) -> None:
        self.dropped.labels(self.session).inc(n)

    def set_clients(self, n: int) -> None:
        self.clients.labels(self.session).set(n)

    def summary(self) -> dict:
        return {
            "encoded_fps_1s": self.fps.labels(self.session)._value.get(),
            "bitrate_kbps_1s": self.bitrate.labels(self.session)._value.get(),
            "qp": self.qp.labels(self.session)._value.get(),
            "encode_ms_p50": self.roll_encode.quantile(0.5),
            "encode_ms_p99": self.roll_encode.quantile(0.99),
            "e2e_ms_p50": self.roll_e2e.quantile(0.5),
            "e2e_ms_p95": self.roll_e2e.quantile(0.95),
        }

    def set_gpu_telemetry(self, gpu: str, values: dict) -> None:
        for k, v in values.items():
            self.gpu.labels(self.session, gpu, k).set(float(v))

    def exposition(self) -> bytes:
        return generate_latest(self.registry)


class ClientStatsLog:
    """``SELKIES_ENABLE_WEBRTC_STATISTICS``: client-reported statistics (``{"type": "stats",
    ...}`` on the data channel or the control WebSocket) appended to
    ``<dir>/mxdesk-webrtc-stats-<pid>.csv``; the header row is the first report's keys,
    later reports are written in that column order (missing values left empty)."""

    FIELDS_MAX = 64

    def __init__(self, directory: str):
        import os

        os.makedirs(directory, exist_ok=True)
        self.path = os.path.join(directory, f"mxdesk-webrtc-stats-{os.getpid()}.csv")
        self.cols: list[str] | None = None
        self._lock = threading.Lock()

    def write(self, report: dict) -> None:
        import csv

        row = {k: v for k, v in report.items() if k != "type" and isinstance(v, (int, float, str, bool))}
        with self._lock, open(self.path, "a", newline="") as f:
            w = csv.writer(f)
            if self.cols is None:
                self.cols = ["server_time"] + sorted(row)[: self.FIELDS_MAX]
                w.writerow(self.cols)
            w.writerow([round(time.time(), 3)] + [row.get(c, "") for c in self.cols[1:]])
