"""mxdesk command line (``python -m mxdesk <command>``).

Commands
  desktop    X server + desktop session, blocks while X runs (reference entrypoint.sh)
  serve      one streaming session on :8080 (the reference's selkies-gstreamer entrypoint,
             selkies-gstreamer-entrypoint.sh:44-47, or noVNC when NOVNC_ENABLE=true)
  launch     one session per visible GPU on ports 8080+i
  wall       tiled video wall: one tile per GPU, RCCL all-gather, single stream (C58)
  supervise  run a supervisord-style config (C56)
  config     print the resolved configuration (secrets redacted)
  devices    list AMD GPUs (sysfs/KFD) and the selected one
  cvt        print a CVT / CVT-RB modeline (``cvt [-r] W H [R]``)
  xorg-conf  print the generated xorg.conf for the current config
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys

from .utils import config as C


class JsonFormatter(logging.Formatter):
    """One JSON object per line (``MXDESK_LOG_FORMAT=json``; SURVEY.md §5.5 structured logs)."""

    def format(self, record: logging.LogRecord) -> str:
        import json

        d = {"ts": round(record.created, 6), "level": record.levelname, "logger": record.name,
             "msg": record.getMessage(), "pid": record.process}
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d, ensure_ascii=False)


def _setup_logging(cfg: C.Config) -> None:
    level = getattr(logging, cfg.log_level_name, logging.WARNING)
    if str(getattr(cfg, "log_format", "text")).lower() == "json":
        h = logging.StreamHandler()
        h.setFormatter(JsonFormatter())
        logging.basicConfig(level=level, handlers=[h])
    else:
        logging.basicConfig(level=level, format="%(asctime)s %(name)s %(levelname)s %(message)s")


def build_pipeline(cfg: C.Config, device: int = 0, session_name: str = "0", capture_allowed: bool = True):
    from .pipeline.stream import StreamPipeline

    backend = "gpu" if cfg.gpu_encoder else "cpu"
    capture = None
    if capture_allowed and (cfg.source == "x11" or (cfg.source == "auto" and _x_available(cfg.display))):
        from .models.x11 import X11Capture

        capture = X11Capture(cfg.display, cfg.sizew, cfg.sizeh)
        if cfg.capture_damage and not capture.enable_damage():
            logging.getLogger("mxdesk").info("XDamage unavailable: full-frame capture")
    return StreamPipeline(cfg.sizew, cfg.sizeh, cfg.stream_fps, backend=backend, device=device,
                          bitrate_kbps=cfg.video_bitrate, keyint=cfg.keyint_frames, search_range=cfg.search_range,
                          subpel=cfg.subpel, noise=cfg.noise, out_width=cfg.out_width, out_height=cfg.out_height,
                          session_name=session_name, capture=capture, codec=cfg.codec)


def _x_available(display: str) -> bool:
    from .display.xorg import x_socket

    return os.path.exists(x_socket(display))


def _gpu_index(cfg: C.Config) -> int:
    """HIP ordinal of the selected GPU: HIP enumerates only the visible devices, in PCI
    order, so the ordinal is the position inside the visible list."""
    from .utils import devices as D

    gpus = D.visible_gpus(D.enumerate_gpus())
    if not gpus:
        return 0
    return gpus.index(D.select_gpu(gpus, cfg.gpu))


def make_injector(cfg: C.Config, pipe):
    """Input sink for a pipeline: XTest into the X server the pipeline captures (the reference
    injects through XTest/xdotool, Dockerfile:428-430); the synthetic desktop's cursor only when
    there is no X capture, or when libXtst / the display cannot be opened."""
    if getattr(pipe, "capture", None) is None:
        return None  # MediaServer / RfbServer build their SyntheticInjector
    from .server.input import XTestInjector

    try:
        return XTestInjector(cfg.display)
    except OSError as e:
        logging.getLogger("mxdesk").warning("XTest injection unavailable (%s): input drives the synthetic cursor", e)
        return None


def _clipboard_in(cfg: C.Config) -> bool:
    return C.clipboard_directions(getattr(cfg, "enable_clipboard", "true"))[0]


def session_config(cfg: C.Config, i: int) -> C.Config:
    """Session i of a multi-session process: its own HTTP port and (if fixed) WebRTC UDP port;
    the process-wide singletons -- gamepad sockets, desktop audio capture -- stay with session 0."""
    c = C.Config(values=dict(cfg.values), sources=dict(cfg.sources))
    c.values["port"] = cfg.port + i
    if cfg.webrtc_udp_port:
        c.values["webrtc_udp_port"] = cfg.webrtc_udp_port + i
    if i > 0:
        c.values["enable_gamepad"] = False
        c.values["enable_audio"] = False
    return c


def cmd_serve_sessions(cfg: C.Config, k: int) -> None:
    """`mxdesk serve --sessions K`: K independent sessions from one process on one GPU (VERDICT r2
    #6) -- each a StreamPipeline with its own HIP stream and encode thread and its own
    MediaServer on port + i, all on one event loop.  Synthetic desktops: an X display is one
    desktop, so only K == 1 captures it."""
    from .server.app import MediaServer, run_forever_multi, ssl_context
    from .utils.sampler import install_from_env

    install_from_env()  # MXDESK_PYPROFILE: per-thread stack samples of this serve process
    if cfg.source == "x11":
        raise SystemExit("serve --sessions K > 1 streams synthetic desktops; MXDESK_SOURCE=x11 serves one")
    if cfg.novnc_enable:
        # the RFB fallback front end exists per single session (cmd_serve); K WebRTC sessions
        # with NOVNC_ENABLE set would silently serve the wrong front end
        raise SystemExit("serve --sessions K > 1 serves WebRTC sessions; NOVNC_ENABLE=true needs a single session")
    # every session drives two HIP streams; with HIP's default of 4 hardware queues per process,
    # K sessions' streams share 4 queues and serialise behind each other.  Must be set before
    # the HIP runtime initialises (the first pipeline below); an explicit setting wins.
    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(max(4, min(16, 2 * k))))
    # K frame threads waiting for their frames: poll-and-sleep instead of hipEventSynchronize, whose
    # waiting kept the host CPUs busy at 32 sessions per process (profiles/r06_density/NOTES.md)
    os.environ.setdefault("MXDESK_WAIT", "sleep")
    # K frame threads and the event loop trade the GIL every frame; with the default 5 ms switch
    # interval a thread that wants it can wait a whole interval behind a busy one
    sys.setswitchinterval(float(os.environ.get("MXDESK_SWITCH_INTERVAL", "0.0005")))
    device = _gpu_index(cfg) if cfg.gpu_encoder else 0
    servers = []
    for i in range(k):
        ci = session_config(cfg, i)
        pipe = build_pipeline(ci, device, session_name=str(i), capture_allowed=False)
        pipe.pace_phase = i / (k * max(1.0, float(ci.stream_fps)))  # spread the K sessions over the period
        # input of a synthetic session drives its own cursor (make_injector -> MediaServer's
        # SyntheticInjector), as in single-session serve
        servers.append(MediaServer(pipe, ci, injector=make_injector(ci, pipe)))
    print(f"mxdesk: serving {k} sessions {cfg.sizew}x{cfg.sizeh}@{cfg.stream_fps} ({cfg.encoder_backend}) on "
          f"{cfg.addr}:{cfg.port}..{cfg.port + k - 1}", flush=True)
    run_forever_multi(servers, cfg.addr, [cfg.port + i for i in range(k)], ssl_context(cfg))


def cmd_serve(cfg: C.Config, args) -> None:
    from .server.app import MediaServer, run_forever, ssl_context


    if cfg.sessions > 1:
        cmd_serve_sessions(cfg, cfg.sessions)
        return
    device = _gpu_index(cfg) if cfg.gpu_encoder else 0
    pipe = build_pipeline(cfg, device)
    injector = make_injector(cfg, pipe)
    rfb = None
    if cfg.novnc_enable:
        from .server.rfb import RfbServer

        rfb = RfbServer(pipe, cfg.effective_basic_auth_password, cfg.novnc_viewpass, fps=min(cfg.stream_fps, 30),
                        injector=injector, clipboard_in=_clipboard_in(cfg))
    # NOVNC_ENABLE=true: the RFB front end replaces WebRTC (supervisord.conf:36 puts selkies
    # to sleep), so the H.264 pipeline is not started.
    srv = MediaServer(pipe, cfg, injector=injector, rfb=rfb, start_pipeline=not cfg.novnc_enable)
    print(f"mxdesk: serving {cfg.sizew}x{cfg.sizeh}@{cfg.stream_fps} ({cfg.encoder_backend}) on "
          f"{cfg.addr}:{cfg.port}", flush=True)
    run_forever(srv, cfg.addr, cfg.port, ssl_context(cfg))


def main(argv: list[str] | None = None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return
    cmd, rest = argv[0], argv[1:]
    if cmd == "cvt":
        from .display.cvt import main as cvt_main

        cvt_main(rest)
        return
    if cmd == "supervise":
        from .utils.supervisor import main as sup_main

        sup_main(rest)
        return
    ap = argparse.ArgumentParser(prog=f"mxdesk {cmd}")
    C.add_cli_flags(ap)
    if cmd == "launch":
        ap.add_argument("--base-port", type=int, default=None)
    if cmd == "wall":
        ap.add_argument("--layout", default=None)
    args, _ = ap.parse_known_args(rest)
    cfg = C.load(cli=args)
    _setup_logging(cfg)
    if cfg.encoder_fallback:
        logging.getLogger("mxdesk").warning(cfg.encoder_fallback)
    if cmd == "config":
        print(cfg.dump())
    elif cmd == "devices":
        from dataclasses import asdict

        from .utils import devices as D

        from .display.desktop import icd_report

        gpus = D.visible_gpus(D.enumerate_gpus())
        print(json.dumps({"gpus": [asdict(g) | {"xorg_busid": g.xorg_busid} for g in gpus], "icds": icd_report()},
                         indent=1))
    elif cmd == "xorg-conf":
        from .display.xorg import DisplaySettings, render_xorg_conf
        from .utils import devices as D

        gpus = D.visible_gpus(D.enumerate_gpus())
        busid = D.select_gpu(gpus, cfg.gpu).xorg_busid if gpus else ""
        print(render_xorg_conf(DisplaySettings(cfg.sizew, cfg.sizeh, cfg.refresh, cfg.cdepth, cfg.dpi,
                                               cfg.video_port, busid, "dummy", cfg.display)), end="")
    elif cmd == "serve":
        cmd_serve(cfg, args)
    elif cmd == "desktop":
        from .display.desktop import run_display_session

        sys.exit(run_display_session(cfg))
    elif cmd == "launch":
        from .parallel.launcher import launch_sessions

        launch_sessions(cfg, base_port=args.base_port or cfg.port, sessions_per_gpu=max(1, cfg.sessions))
    elif cmd == "wall":
        from .parallel.wall import wall_main

        sys.exit(wall_main(cfg, layout=args.layout or cfg.wall or "2x2", argv=rest))
    else:
        print(f"unknown command {cmd}\n{__doc__}")
        sys.exit(2)


if __name__ == "__main__":
    main()
