"""Typed configuration schema.

One schema for every environment variable of the reference image, with the reference's
names and defaults (reference Dockerfile:14-17,200-212; xgl.yml:25-109;
selkies-gstreamer-entrypoint.sh:18-20; entrypoint.sh:121-123), the selkies-gstreamer
pass-through options it forwards as ``"$@"`` (selkies-gstreamer-entrypoint.sh:44-47;
README.md:38) under both their ``SELKIES_*`` and legacy env names, plus mxdesk's own
options.  Booleans are compared case-insensitively like ``${VAR,,}`` in the reference
scripts.  ``--flag`` CLI overrides win over the environment.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Mapping, Sequence

TRUE = {"true", "1", "yes", "on"}
FALSE = {"false", "0", "no", "off", ""}


def parse_bool(v: Any, default: bool = False) -> bool:
    if isinstance(v, bool):
        return v
    if v is None:
        return default
    s = str(v).strip().lower()
    if s in TRUE:
        return True
    if s in FALSE:
        return False
    raise ValueError(f"not a boolean: {v!r}")


# Encoder names accepted by WEBRTC_ENCODER.  The reference's nvh264enc (NVENC) and the
# VA-API names map to the HIP encoders; x264enc / x265enc (CPU) map to the CPU encoders.
ENCODER_ALIASES = {
    "nvh264enc": "mxh264enc",
    "vah264enc": "mxh264enc",
    "vaapih264enc": "mxh264enc",
    "mxh264enc": "mxh264enc",
    "x264enc": "cpuh264enc",
    "openh264enc": "cpuh264enc",
    "cpuh264enc": "cpuh264enc",
    "nvh265enc": "mxh265enc",
    "vah265enc": "mxh265enc",
    "vaapih265enc": "mxh265enc",
    "mxh265enc": "mxh265enc",
    "x265enc": "cpuh265enc",
    "cpuh265enc": "cpuh265enc",
    # the reference's libvpx choice (README.md:21,35) -> the HIP VP8 encoder
    "vp8enc": "mxvp8enc",
    "vaapivp8enc": "mxvp8enc",
    "mxvp8enc": "mxvp8enc",
    "cpuvp8enc": "cpuvp8enc",
}
GPU_ENCODERS = {"mxh264enc", "mxh265enc", "mxvp8enc"}
# selkies encoders without an mxdesk implementation: the session falls back to the GPU H.264
# encoder (every WebRTC browser decodes H.264) with a startup warning instead of failing
FALLBACK_ENCODERS = {"vp9enc": "mxh264enc", "av1enc": "mxh264enc", "vaapivp9enc": "mxh264enc",
                     "vaapiav1enc": "mxh264enc"}


@dataclass
class Var:
    """Declaration of one configuration variable."""

    attr: str
    env: Sequence[str]  # accepted env names, first = canonical
    default: Any
    kind: type = str
    help: str = ""
    secret: bool = False
    ref: str = ""  # reference file:line


SCHEMA: list[Var] = [
    # ---- reference image defaults (Dockerfile:200-212, xgl.yml)
    Var("tz", ["TZ"], "UTC", str, "timezone", ref="Dockerfile:201"),
    Var("sizew", ["SIZEW"], 1920, int, "desktop width", ref="Dockerfile:202"),
    Var("sizeh", ["SIZEH"], 1080, int, "desktop height", ref="Dockerfile:203"),
    Var("refresh", ["REFRESH"], 60, int, "refresh rate / capture frame rate", ref="Dockerfile:204"),
    Var("dpi", ["DPI"], 96, int, "X server DPI", ref="Dockerfile:205"),
    Var("cdepth", ["CDEPTH"], 24, int, "colour depth", ref="Dockerfile:206"),
    Var("video_port", ["VIDEO_PORT"], "DFP", str, "virtual connector; 'none' disables RANDR", ref="Dockerfile:207"),
    Var("passwd", ["PASSWD"], "mypasswd", str, "user password; default web/VNC password", True, "Dockerfile:208"),
    Var("novnc_enable", ["NOVNC_ENABLE"], False, bool, "serve the RFB/noVNC front end instead of WebRTC",
        ref="Dockerfile:209"),
    Var("novnc_viewpass", ["NOVNC_VIEWPASS"], None, str, "view-only VNC password", True, "entrypoint.sh:122"),
    Var("encoder", ["WEBRTC_ENCODER", "SELKIES_ENCODER"], "nvh264enc", str, "video encoder", ref="Dockerfile:210"),
    Var("enable_resize", ["WEBRTC_ENABLE_RESIZE", "SELKIES_ENABLE_RESIZE"], False, bool,
        "let the client resize the remote display", ref="Dockerfile:211"),
    Var("enable_basic_auth", ["ENABLE_BASIC_AUTH", "SELKIES_ENABLE_BASIC_AUTH"], True, bool, "HTTP basic auth",
        ref="Dockerfile:212"),
    Var("basic_auth_user", ["BASIC_AUTH_USER", "SELKIES_BASIC_AUTH_USER"], "user", str, "basic auth user name",
        ref="README.md:23"),
    Var("basic_auth_password", ["BASIC_AUTH_PASSWORD", "SELKIES_BASIC_AUTH_PASSWORD"], None, str,
        "basic auth password (defaults to PASSWD)", True, "selkies-gstreamer-entrypoint.sh:20"),
    Var("enable_https", ["ENABLE_HTTPS_WEB", "SELKIES_ENABLE_HTTPS"], False, bool, "serve HTTPS", ref="xgl.yml:68"),
    Var("https_cert", ["HTTPS_WEB_CERT", "SELKIES_HTTPS_CERT"], "/etc/ssl/certs/ssl-cert-snakeoil.pem", str,
        "HTTPS certificate", ref="xgl.yml:71"),
    Var("https_key", ["HTTPS_WEB_KEY", "SELKIES_HTTPS_KEY"], "/etc/ssl/private/ssl-cert-snakeoil.key", str,
        "HTTPS key", ref="xgl.yml:73"),
    Var("turn_host", ["TURN_HOST", "SELKIES_TURN_HOST"], None, str, "TURN server host", ref="xgl.yml:85"),
    Var("turn_port", ["TURN_PORT", "SELKIES_TURN_PORT"], 3478, int, "TURN server port", ref="xgl.yml:87"),
    Var("turn_shared_secret", ["TURN_SHARED_SECRET", "SELKIES_TURN_SHARED_SECRET"], None, str,
        "time-limited TURN credentials (HMAC shared secret)", True, "xgl.yml:90"),
    Var("turn_username", ["TURN_USERNAME", "SELKIES_TURN_USERNAME"], None, str, "legacy TURN user",
        ref="xgl.yml:95"),
    Var("turn_password", ["TURN_PASSWORD", "SELKIES_TURN_PASSWORD"], None, str, "legacy TURN password", True,
        "xgl.yml:98"),
    Var("turn_protocol", ["TURN_PROTOCOL", "SELKIES_TURN_PROTOCOL"], "udp", str, "udp or tcp", ref="xgl.yml:105"),
    Var("turn_tls", ["TURN_TLS", "SELKIES_TURN_TLS"], False, bool, "TURN over TLS", ref="xgl.yml:108"),
    Var("turn_rest_uri", ["TURN_REST_URI", "SELKIES_TURN_REST_URI"], None, str, "TURN REST credential service",
        ref="README.md:38"),
    Var("stun_host", ["STUN_HOST", "SELKIES_STUN_HOST"], "stun.l.google.com", str, "STUN server",
        ref="README.md:38"),
    Var("stun_port", ["STUN_PORT", "SELKIES_STUN_PORT"], 19302, int, "STUN port", ref="README.md:38"),
    Var("log_level", ["LOG_LEVEL", "GST_DEBUG"], "*:2", str, "log level (GST_DEBUG style '*:N' or a name)",
        ref="selkies-gstreamer-entrypoint.sh:18"),
    # ---- fixed environment (Dockerfile:14-17)
    Var("display", ["DISPLAY"], ":0", str, "X display", ref="Dockerfile:15"),
    Var("xdg_runtime_dir", ["XDG_RUNTIME_DIR"], "/tmp/runtime-user", str, "runtime dir", ref="Dockerfile:16"),
    Var("pulse_server", ["PULSE_SERVER"], "unix:/run/pulse/native", str, "audio server", ref="Dockerfile:17"),
    # ---- selkies pass-through flags (README.md:38)
    Var("addr", ["SELKIES_ADDR"], "0.0.0.0", str, "listen address", ref="selkies-gstreamer-entrypoint.sh:45"),
    Var("port", ["SELKIES_PORT", "MXDESK_PORT"], 8080, int, "listen port", ref="selkies-gstreamer-entrypoint.sh:46"),
    Var("framerate", ["SELKIES_FRAMERATE", "WEBRTC_FRAMERATE"], 0, int, "stream frame rate (0 = REFRESH)"),
    Var("video_bitrate", ["SELKIES_VIDEO_BITRATE", "WEBRTC_VIDEO_BITRATE"], 8000, int, "video bitrate (kbps)"),
    Var("keyframe_distance", ["SELKIES_KEYFRAME_DISTANCE"], -1.0, float, "seconds between IDRs (-1 = on demand)"),
    Var("congestion_control", ["SELKIES_CONGESTION_CONTROL"], False, bool, "adapt bitrate to the client"),
    Var("enable_audio", ["SELKIES_ENABLE_AUDIO"], True, bool, "desktop audio (PCM over WebSocket, PCMU over WebRTC)"),
    Var("audio_source", ["MXDESK_AUDIO_SOURCE"], "auto", str, "audio capture: auto | pulse | synthetic | fifo:PATH | none"),
    Var("audio_bitrate", ["SELKIES_AUDIO_BITRATE"], 128000, int, "audio bitrate (bps)"),
    Var("enable_clipboard", ["SELKIES_ENABLE_CLIPBOARD"], "true", str,
        "clipboard sync: true | false | in (browser -> desktop only) | out (desktop -> browser only)"),
    Var("enable_cursors", ["SELKIES_ENABLE_CURSORS"], True, bool, "remote cursor forwarding"),
    Var("enable_metrics_http", ["SELKIES_ENABLE_METRICS_HTTP"], False, bool, "Prometheus /metrics on its own port"),
    Var("enable_webrtc_statistics", ["SELKIES_ENABLE_WEBRTC_STATISTICS"], False, bool,
        "append client-reported WebRTC statistics to CSV files"),
    Var("webrtc_statistics_dir", ["SELKIES_WEBRTC_STATISTICS_DIR"], "/tmp", str, "directory of those CSV files"),
    Var("metrics_http_port", ["SELKIES_METRICS_HTTP_PORT"], 8000, int, "metrics port"),
    Var("web_root", ["SELKIES_WEB_ROOT"], "", str, "static web client directory ('' = bundled)"),
    # ---- mxdesk options
    Var("gpu", ["MXDESK_GPU", "GPU_SELECT"], None, str, "GPU index / PCI bus id / unique id to use"),
    Var("source", ["MXDESK_SOURCE"], "auto", str, "frame source: synthetic | x11 | auto"),
    Var("capture_damage", ["MXDESK_CAPTURE_DAMAGE"], True, bool,
        "X11 capture driven by XDamage: grab and upload only the changed row bands"),
    Var("out_width", ["MXDESK_OUT_WIDTH"], 0, int, "encoded width (0 = SIZEW; else Lanczos scale)"),
    Var("out_height", ["MXDESK_OUT_HEIGHT"], 0, int, "encoded height (0 = SIZEH)"),
    Var("search_range", ["MXDESK_SEARCH_RANGE"], 16, int, "motion search radius (integer pels, <= 32)"),
    Var("subpel", ["MXDESK_SUBPEL"], True, bool, "quarter-pel motion refinement"),
    Var("noise", ["MXDESK_NOISE"], True, bool, "synthetic desktop: animated-noise panel"),
    Var("wall", ["MXDESK_WALL"], "", str, "tiled wall layout, e.g. '2x2' (one tile per GPU)"),
    Var("sessions", ["MXDESK_SESSIONS"], 1, int,
        "sessions per process: `serve` streams K independent desktops from one process on one GPU "
        "(ports port .. port+K-1, one HIP stream and native encode thread each); `launch` starts one such "
        "process per visible GPU"),
    Var("enable_gamepad", ["MXDESK_GAMEPAD", "SELKIES_ENABLE_GAMEPAD"], True, bool,
        "browser gamepads -> /dev/input/jsN via the LD_PRELOAD interposer", ref="Dockerfile:473-476"),
    Var("js_dir", ["MXDESK_JS_DIR"], "/tmp", str, "directory of the joystick interposer sockets"),
    Var("webrtc_host", ["MXDESK_WEBRTC_HOST"], "", str, "address advertised in the WebRTC host candidate"),
    Var("webrtc_udp_port", ["MXDESK_WEBRTC_UDP_PORT"], 0, int, "UDP port for WebRTC media (0 = ephemeral)"),
    Var("selkies_peer", ["MXDESK_SELKIES_PEER"], True, bool,
        "the streaming peer on /ws offers a stream to every registering selkies client"),
    Var("turn_relay", ["MXDESK_TURN_RELAY"], True, bool,
        "allocate a server-side TURN relay candidate when TURN_HOST + credentials are set"),
    Var("log_dir", ["MXDESK_LOG_DIR"], "/tmp", str, "log directory", ref="supervisord.conf:9"),
    Var("log_format", ["MXDESK_LOG_FORMAT"], "text", str, "log line format: text | json"),
]
_BY_ATTR = {v.attr: v for v in SCHEMA}


def _convert(var: Var, raw: Any) -> Any:
    if raw is None:
        return None
    if var.kind is bool:
        return parse_bool(raw)
    if var.kind is int:
        return int(str(raw).strip())
    if var.kind is float:
        return float(str(raw).strip())
    return str(raw)


@dataclass
class Config:
    values: dict[str, Any] = field(default_factory=dict)
    sources: dict[str, str] = field(default_factory=dict)

    def __getattr__(self, name: str) -> Any:
        try:
            return self.__dict__["values"][name]
        except KeyError:
            raise AttributeError(name) from None

    # ---- derived values
    @property
    def effective_basic_auth_password(self) -> str:
        """selkies-gstreamer-entrypoint.sh:20 / entrypoint.sh:123: BASIC_AUTH_PASSWORD or PASSWD."""
        return self.values["basic_auth_password"] or self.values["passwd"]

    @property
    def encoder_backend(self) -> str:
        name = str(self.values["encoder"]).strip().lower()
        if name in FALLBACK_ENCODERS:
            return FALLBACK_ENCODERS[name]
        if name not in ENCODER_ALIASES:
            raise ValueError(f"unknown WEBRTC_ENCODER={name}")
        return ENCODER_ALIASES[name]

    @property
    def encoder_fallback(self) -> str | None:
        """Why the requested WEBRTC_ENCODER is not the one running, or None."""
        name = str(self.values["encoder"]).strip().lower()
        if name in FALLBACK_ENCODERS:
            return (f"WEBRTC_ENCODER={name} is not implemented; streaming H.264 with "
                    f"{FALLBACK_ENCODERS[name]} instead (all WebRTC browsers decode it)")
        return None

    @property
    def codec(self) -> str:
        """Bitstream format of the selected encoder: "h264", "hevc" or "vp8"."""
        b = self.encoder_backend
        return "hevc" if "265" in b else ("vp8" if "vp8" in b else "h264")

    @property
    def gpu_encoder(self) -> bool:
        return self.encoder_backend in GPU_ENCODERS

    @property
    def stream_fps(self) -> int:
        return self.values["framerate"] or self.values["refresh"]

    @property
    def keyint_frames(self) -> int:
        kd = self.values["keyframe_distance"]
        return 0 if kd is None or kd < 0 else max(1, int(round(kd * self.stream_fps)))

    @property
    def log_level_name(self) -> str:
        lv = str(self.values["log_level"]).strip()
        if lv.startswith("*:"):
            n = int(lv[2:] or 2)
            return {0: "CRITICAL", 1: "ERROR", 2: "WARNING", 3: "INFO", 4: "INFO"}.get(n, "DEBUG")
        return lv.upper()

    def validate(self) -> None:
        v = self.values
        if v["sizew"] <= 0 or v["sizeh"] <= 0 or v["sizew"] % 2 or v["sizeh"] % 2:
            raise ValueError("SIZEW/SIZEH must be positive and even")
        if v["refresh"] <= 0 or v["refresh"] > 480:
            raise ValueError("REFRESH out of range")
        if v["cdepth"] not in (8, 15, 16, 24, 30):
            raise ValueError("CDEPTH must be one of 8, 15, 16, 24, 30")
        if str(v["turn_protocol"]).lower() not in ("udp", "tcp"):
            raise ValueError("TURN_PROTOCOL must be udp or tcp")
        if not 1 <= v["search_range"] <= 32:
            raise ValueError("MXDESK_SEARCH_RANGE must be in [1, 32]")
        if v["source"] not in ("auto", "synthetic", "x11"):
            raise ValueError("MXDESK_SOURCE must be auto, synthetic or x11")
        self.encoder_backend  # noqa: B018  (raises on unknown encoders)

    def redacted(self) -> dict[str, Any]:
        out = {}
        for var in SCHEMA:
            val = self.values[var.attr]
            out[var.env[0]] = "******" if (var.secret and val) else val
        return out

    def dump(self) -> str:
        return json.dumps(self.redacted(), indent=1, sort_keys=True, default=str)


def add_cli_flags(ap: argparse.ArgumentParser) -> None:
    for var in SCHEMA:
        flag = "--" + var.attr
        if var.kind is bool:
            ap.add_argument(flag, type=str, default=None, metavar="true|false", help=var.help)
        else:
            ap.add_argument(flag, type=str, default=None, help=var.help)


def load(env: Mapping[str, str] | None = None, argv: Sequence[str] | None = None,
         cli: argparse.Namespace | None = None) -> Config:
    """Build the config: defaults < environment (first matching name) < CLI flags."""
    env = os.environ if env is None else env
    if argv is not None and cli is None:
        ap = argparse.ArgumentParser(add_help=False)
        add_cli_flags(ap)
        cli, _ = ap.parse_known_args(list(argv))
    cfg = Config()
    for var in SCHEMA:
        val, src = var.default, "default"
        for name in var.env:
            if name in env:
                val, src = _convert(var, env[name]), f"env:{name}"
                break
        if cli is not None and getattr(cli, var.attr, None) is not None:
            val, src = _convert(var, getattr(cli, var.attr)), "cli"
        cfg.values[var.attr] = val
        cfg.sources[var.attr] = src
    cfg.validate()
    return cfg


def schema_table() -> list[dict[str, Any]]:
    return [dataclasses.asdict(v) | {"kind": v.kind.__name__} for v in SCHEMA]


def clipboard_directions(value: Any) -> tuple[bool, bool]:
    """(browser -> desktop, desktop -> browser) for SELKIES_ENABLE_CLIPBOARD's selkies values."""
    v = str(value if value is not None else "true").strip().lower()
    if v == "in":
        return True, False
    if v == "out":
        return False, True
    on = parse_bool(v, True)
    return on, on
