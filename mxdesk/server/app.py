"""HTTP(S) + WebSocket front end on :8080.

Replaces the selkies-gstreamer web/signalling server started by
selkies-gstreamer-entrypoint.sh:44-47 (``--addr=0.0.0.0 --port=8080``) and, when
``NOVNC_ENABLE=true``, the noVNC/websockify front end (entrypoint.sh:121-125):

  GET  /                 web client (WebCodecs H.264 player + input capture), PWA manifest;
                         with NOVNC_ENABLE=true the VNC viewer (web/vnc.html + vnc.js)
  GET  /health           liveness/readiness (200 when frames flow)
  GET  /turn             RTCConfiguration JSON (STUN/TURN; HMAC or legacy credentials)
  GET  /metrics          Prometheus exposition
  GET  /status           JSON session status (fps, bitrate, QP, latency quantiles)
  WS   /ws               selkies signalling: streaming peer (offers to each client) + relay
  WS   /mxws             media transport: binary Annex-B access units + JSON control/input
  WS   /websockify       RFB (noVNC) over WebSocket when NOVNC_ENABLE=true

Basic auth (ENABLE_BASIC_AUTH, user ``user``, password BASIC_AUTH_PASSWORD or PASSWD) and
HTTPS (ENABLE_HTTPS_WEB + HTTPS_WEB_CERT/KEY) follow the reference contract.

Remote -> client state (``desktop_sync``): clipboard changes (SELKIES_ENABLE_CLIPBOARD) and
cursor images (SELKIES_ENABLE_CURSORS, X capture only) are pushed to every /mxws client and
every WebRTC data channel.  With WEBRTC_ENABLE_RESIZE a client ``r,WxH`` / ``{"type":
"resize"}`` message resizes the X screen (RandR) and restarts the session at that size; the
WebSocket clients get a new ``config`` message before the first frame of the new size.
"""
from __future__ import annotations

import asyncio
import json
import logging
import ssl
import time
from pathlib import Path
from typing import Any

from aiohttp import WSMsgType, web

from ..pipeline.stream import StreamPipeline, codec_string, frame_header
from . import turn
from .auth import basic_auth_middleware
from .input import SyntheticInjector, parse_message
from .signalling import SignallingRelay

log = logging.getLogger("mxdesk.server")
WEB_ROOT = Path(__file__).resolve().parent.parent.parent / "web"


def render_manifest(app_name: str = "mxdesk", short: str = "mxdesk", start_url: str = "/index.html") -> str:
    """PWA manifest (reference templating: selkies-gstreamer-entrypoint.sh:27-38)."""
    return json.dumps({
        "name": app_name, "short_name": short, "start_url": start_url, "display": "fullscreen",
        "background_color": "#000000", "theme_color": "#000000",
        "icons": [{"src": "icon.svg", "sizes": "any", "type": "image/svg+xml"}],
    }, indent=1)


class MediaServer:
    def __init__(self, pipeline: StreamPipeline, cfg: Any = None, injector: Any = None,
                 web_root: Path | None = None, rfb: Any = None, start_pipeline: bool = True):
        self.pipeline = pipeline
        self.cfg = cfg
        self.injector = injector or SyntheticInjector(pipeline, pipeline.out_w, pipeline.out_h)
        self.web_root = Path(web_root) if web_root else WEB_ROOT
        self.signalling = SignallingRelay()
        self.rfb = rfb
        self.start_pipeline = start_pipeline
        self.clients: set[web.WebSocketResponse] = set()
        self.resize_enabled = bool(getattr(cfg, "enable_resize", False))
        from .desktop_sync import ClipboardSync, CursorSync

        x_display = getattr(cfg, "display", None) if pipeline.capture is not None else None
        self.x_display = x_display
        from ..utils.config import clipboard_directions

        self.clipboard_in, self.clipboard_out = clipboard_directions(getattr(cfg, "enable_clipboard", "true"))
        self.clipboard = ClipboardSync(self.injector, x_display) if (self.clipboard_in or self.clipboard_out) \
            else None
        self.cursors = CursorSync(pipeline.capture) if (pipeline.capture is not None and
                                                         bool(getattr(cfg, "enable_cursors", True))) else None
        self._sync_task: asyncio.Task | None = None
        self.stats_log = None
        if bool(getattr(cfg, "enable_webrtc_statistics", False)):
            from ..utils.metrics import ClientStatsLog

            self.stats_log = ClientStatsLog(getattr(cfg, "webrtc_statistics_dir", "/tmp") or "/tmp")
        from .gamepad import GamepadServer
        from .webrtc import WhepEndpoint, turn_relay_settings

        self.gamepad = GamepadServer(getattr(cfg, "js_dir", None)) if bool(getattr(cfg, "enable_gamepad", True)) else None

        self.audio = None
        if bool(getattr(cfg, "enable_audio", False)):
            from ..audio import AudioPipeline, make_source

            try:
                src = make_source(getattr(cfg, "audio_source", "auto"))
            except (OSError, ValueError) as e:
                log.warning("audio disabled: %s", e)
                src = None
            self.audio = AudioPipeline(src) if src is not None else None
        self.whep = WhepEndpoint(pipeline, audio=self.audio,
                                 congestion_control=bool(getattr(cfg, "congestion_control", False)), host=getattr(cfg, "webrtc_host", None) or None,
                                 udp_port=int(getattr(cfg, "webrtc_udp_port", 0) or 0),
                                 on_input=self._on_client_message, turn=turn_relay_settings(cfg))
        self.selkies = None
        if bool(getattr(cfg, "selkies_peer", True)):
            from .selkies_peer import SelkiesServerPeer
            from .webrtc import WebRtcPeer

            w = self.whep
            self.selkies = SelkiesServerPeer(self.signalling, lambda: WebRtcPeer(
                pipeline, None, w.host, w.udp_port, w.level_idc, audio=w.audio,
                congestion_control=w.congestion_control, on_input=w.on_input, turn=w.turn,
                server_channels=("input",)))
            self.signalling.attach_server(self.selkies)

    # ------------------------------------------------------------------ app
    def make_app(self) -> web.Application:
        mws = []
        if self.cfg is not None and getattr(self.cfg, "enable_basic_auth", False):
            mws.append(basic_auth_middleware(getattr(self.cfg, "basic_auth_user", "user"),
                                             self.cfg.effective_basic_auth_password))
        app = web.Application(middlewares=mws)
        app.router.add_get("/", self.index)
        app.router.add_get("/index.html", self.index)
        app.router.add_get("/health", self.health)
        app.router.add_get("/turn", self.turn)
        app.router.add_get("/turn/", self.turn)
        app.router.add_get("/metrics", self.metrics)
        app.router.add_get("/status", self.status)
        app.router.add_get("/manifest.json", self.manifest)
        app.router.add_get("/ws", self.signalling.handler)
        app.router.add_get("/webrtc/signalling/", self.signalling.handler)  # selkies >= 1.5 web app path
        app.router.add_get("/mxws", self.media_ws)
        self.whep.routes(app)
        if self.rfb is not None:
            app.router.add_get("/websockify", self.rfb.ws_handler)
        if self.web_root.is_dir():
            app.router.add_static("/static/", self.web_root, show_index=False)
            app.router.add_get("/{name:[A-Za-z0-9_.-]+\\.(?:js|css|svg|json|html)}", self.static_file)
        app.on_startup.append(self._on_startup)
        app.on_cleanup.append(self._on_cleanup)
        return app

    async def _on_startup(self, app):
        if self.gamepad is not None:
            try:
                await self.gamepad.start()
            except OSError as e:  # e.g. read-only /tmp: gamepads are optional
                log.warning("gamepad sockets unavailable: %s", e)
                self.gamepad = None
        if self.start_pipeline:
            self.pipeline.start()
        if self.audio is not None:
            self.audio.start()
        if self.clipboard is not None or self.cursors is not None:
            self._sync_task = asyncio.create_task(self._sync_loop())

    async def _on_cleanup(self, app):
        if self._sync_task is not None:
            self._sync_task.cancel()
        self.whep.close_all()
        if self.selkies is not None:
            self.selkies.close_all()
        if self.audio is not None:
            self.audio.stop()
        if self.gamepad is not None:
            await self.gamepad.stop()
        self.pipeline.stop()
        for ws in list(self.clients):
            await ws.close()

    # ------------------------------------------------------------------ http handlers
    async def index(self, request: web.Request) -> web.StreamResponse:
        # NOVNC_ENABLE=true: the VNC viewer (RFB over /websockify) is the front page, as noVNC's
        # vnc.html is in the reference (entrypoint.sh:124)
        f = self.web_root / ("vnc.html" if self.rfb is not None else "index.html")
        if f.exists():
            return web.FileResponse(f)
        return web.Response(text="<html><body>mxdesk</body></html>", content_type="text/html")

    async def static_file(self, request: web.Request) -> web.StreamResponse:
        name = request.match_info["name"]
        if name == "manifest.json":
            return await self.manifest(request)
        f = (self.web_root / name).resolve()
        if self.web_root.resolve() not in f.parents or not f.is_file():
            raise web.HTTPNotFound()
        return web.FileResponse(f)

    async def manifest(self, request: web.Request) -> web.Response:
        return web.Response(text=render_manifest(), content_type="application/manifest+json")

    async def health(self, request: web.Request) -> web.Response:
        ok = not self.start_pipeline or self.pipeline.healthy() or self.pipeline.frames_out == 0
        return web.Response(status=200 if ok else 503, text="OK" if ok else "STALLED")

    async def turn(self, request: web.Request) -> web.Response:
        cfg = self.cfg
        if cfg is not None and getattr(cfg, "turn_rest_uri", None):
            data = await turn.fetch_rest_credentials(cfg.turn_rest_uri, protocol=cfg.turn_protocol,
                                                     tls=cfg.turn_tls)
        else:
            data = turn.rtc_config(cfg) if cfg is not None else {"iceServers": []}
        return web.json_response(data)

    async def metrics(self, request: web.Request) -> web.Response:
        self._refresh_gpu_telemetry()
        return web.Response(body=self.pipeline.metrics.exposition(), content_type="text/plain")

    def _refresh_gpu_telemetry(self) -> None:
        """GPU busy %, VRAM, power, temperature of the session's GPU (amdgpu sysfs)."""
        if getattr(self.pipeline, "backend", "cpu") != "gpu":
            return
        try:
            from ..utils import devices as D

            if not hasattr(self, "_gpu_bdf"):
                vis = D.visible_gpus(D.enumerate_gpus())
                dev = int(getattr(self.pipeline, "device", 0))
                self._gpu_bdf = vis[dev].pci_bdf if dev < len(vis) else None
            if self._gpu_bdf:
                self.pipeline.metrics.set_gpu_telemetry(self._gpu_bdf, D.gpu_telemetry(self._gpu_bdf))
        except (OSError, ValueError, IndexError) as e:
            log.debug("GPU telemetry unavailable: %s", e)
            self._gpu_bdf = None

    async def status(self, request: web.Request) -> web.Response:
        st = self.pipeline.status()
        fb = getattr(self.cfg, "encoder_fallback", None) if self.cfg is not None else None
        if fb:
            st["encoder_fallback"] = fb
        return web.json_response(st)

    # ------------------------------------------------------------------ media websocket
    async def media_ws(self, request: web.Request) -> web.WebSocketResponse:
        ws = web.WebSocketResponse(heartbeat=10, max_msg_size=64 * 1024 * 1024)
        await ws.prepare(request)
        p = self.pipeline
        # ?media=0: control/input channel only (the WebRTC client receives media over SRTP)
        media = request.query.get("media", "1") != "0"
        want_audio = media and self.audio is not None and request.query.get("audio", "1") != "0"
        from ..audio.pipeline import CHANNELS, RATE

        await ws.send_str(json.dumps({
            "type": "config", "codec": codec_string(getattr(p, "codec", "h264"), p.out_w, p.out_h, p.fps), "width": p.out_w,
            "height": p.out_h, "fps": p.fps, "resize": self.resize_enabled,
            "audio": {"codec": "pcm_s16le", "rate": RATE, "channels": CHANNELS} if want_audio else None,
        }))
        if self.cursors is not None and self.cursors.last_message:
            await ws.send_str(self.cursors.last_message)
        sub = p.subscribe(asyncio.get_running_loop()) if media else None
        self.clients.add(ws)
        sender = asyncio.create_task(self._send_loop(ws, sub)) if media else None
        asub = self.audio.subscribe(asyncio.get_running_loop()) if want_audio else None
        asender = asyncio.create_task(self._audio_loop(ws, asub)) if want_audio else None
        try:
            async for msg in ws:
                if msg.type == WSMsgType.TEXT:
                    self._on_client_message(msg.data)
                elif msg.type == WSMsgType.ERROR:
                    break
        finally:
            if sender is not None:
                sender.cancel()
                p.unsubscribe(sub)
            if asender is not None:
                asender.cancel()
                self.audio.unsubscribe(asub)
            self.clients.discard(ws)
        return ws

    def _config_message(self, width: int, height: int) -> str:
        p = self.pipeline
        return json.dumps({"type": "config", "codec": codec_string(getattr(p, "codec", "h264"), width, height, p.fps),
                           "width": width, "height": height, "fps": p.fps, "resize": self.resize_enabled,
                           "audio": None, "reconfigure": True})

    async def _send_loop(self, ws: web.WebSocketResponse, sub) -> None:
        from .. import native

        dims = (self.pipeline.out_w, self.pipeline.out_h)
        while not ws.closed:
            fr = await sub.queue.get()
            try:
                if (fr.width, fr.height) != dims:  # resized session: new decoder config first
                    dims = (fr.width, fr.height)
                    await ws.send_str(self._config_message(*dims))
                await ws.send_bytes(frame_header(fr, native().now_us()) + fr.au)
            except (ConnectionResetError, RuntimeError):
                return

    async def _audio_loop(self, ws: web.WebSocketResponse, sub) -> None:
        from ..audio.pipeline import audio_message

        while not ws.closed:
            ch = await sub.queue.get()
            try:
                await ws.send_bytes(audio_message(ch))
            except (ConnectionResetError, RuntimeError):
                return

    def _on_client_message(self, text: str) -> None:
        ev = parse_message(text)
        if ev is None:
            return
        p = self.pipeline
        if ev.kind == "pli":
            p.request_idr("client")
        elif ev.kind == "bitrate":
            p.set_bitrate(int(ev.value))
        elif ev.kind == "ack":
            # client-measured latency (same-clock clients) or RTT-based estimate
            lat = ev.extra.get("latency_ms")
            if lat is not None:
                p.metrics.on_client_latency(float(lat))
        elif ev.kind == "fps":
            p.set_fps(ev.value)
        elif ev.kind == "stats":
            if self.stats_log is not None:
                self.stats_log.write(ev.extra)
        elif ev.kind == "gamepad":
            if self.gamepad is not None:
                self.gamepad.apply(ev)
        elif ev.kind == "resize":
            if self.resize_enabled:
                self.request_resize(ev.width, ev.height)
            else:
                log.info("client resize %dx%d ignored (WEBRTC_ENABLE_RESIZE=false)", ev.width, ev.height)
        elif ev.kind == "clipboard":
            if self.clipboard_in:
                self.injector.apply(ev)
                if self.clipboard is not None:
                    self.clipboard.write(ev.text)
        else:
            self.injector.apply(ev)

    # ------------------------------------------------------------------ resize / sync
    def request_resize(self, width: int, height: int) -> None:
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            loop = None
        if loop is not None:  # RandR runs subprocesses: keep them off the event loop
            loop.run_in_executor(None, self._resize_blocking, width, height)
        else:
            self._resize_blocking(width, height)

    def _resize_blocking(self, width: int, height: int) -> None:
        from ..display.randr import clamp_size, resize_display

        w, h = clamp_size(width, height)
        if (w, h) == (self.pipeline.out_w, self.pipeline.out_h):
            return
        if self.x_display:
            try:
                resize_display(self.x_display, w, h, float(getattr(self.cfg, "refresh", 60) or 60))
            except Exception as e:
                log.warning("RandR resize to %dx%d failed: %s", w, h, e)
                return
        self.pipeline.resize(w, h)
        if hasattr(self.injector, "w"):
            self.injector.w, self.injector.h = w, h
        log.info("client resize -> %dx%d", w, h)

    def broadcast(self, text: str) -> None:
        """One control message to every /mxws client and every WebRTC data channel."""
        for ws in list(self.clients):
            if not ws.closed:
                asyncio.ensure_future(ws.send_str(text))
        for peer in list(self.whep.peers.values()):
            peer.dc_send(text)

    async def _sync_loop(self, period: float = 0.1, clipboard_every: int = 10) -> None:
        loop = asyncio.get_running_loop()
        n = 0
        while True:
            try:
                if self.cursors is not None:
                    msg = await loop.run_in_executor(None, self.cursors.poll)
                    if msg:
                        self.broadcast(msg)
                if self.clipboard is not None and self.clipboard_out and n % clipboard_every == 0:
                    text = await loop.run_in_executor(None, self.clipboard.poll)
                    if text is not None:
                        from .desktop_sync import clipboard_message

                        self.broadcast(clipboard_message(text))
            except asyncio.CancelledError:
                raise
            except Exception:
                log.exception("desktop sync")
            n += 1
            await asyncio.sleep(period)


def ssl_context(cfg: Any) -> ssl.SSLContext | None:
    if not getattr(cfg, "enable_https", False):
        return None
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(cfg.https_cert, cfg.https_key)
    return ctx


async def serve(server: MediaServer, host: str, port: int, ssl_ctx: ssl.SSLContext | None = None) -> web.AppRunner:
    runner = web.AppRunner(server.make_app())
    await runner.setup()
    site = web.TCPSite(runner, host, port, ssl_context=ssl_ctx)
    await site.start()
    log.info("serving on %s://%s:%d", "https" if ssl_ctx else "http", host, port)
    return runner


def run_forever(server: MediaServer, host: str, port: int, ssl_ctx: ssl.SSLContext | None = None) -> None:
    async def main():
        runner = await serve(server, host, port, ssl_ctx)
        try:
            while True:
                await asyncio.sleep(3600)
        finally:
            await runner.cleanup()

    try:
        asyncio.run(main())
    except KeyboardInterrupt:
        pass


def run_forever_multi(servers: list[MediaServer], host: str, ports: list[int],
                      ssl_ctx: ssl.SSLContext | None = None) -> None:
    """Several MediaServers (one per session) on one event loop, each on its own port."""
    async def main():
        runners = [await serve(s, host, p, ssl_ctx) for s, p in zip(servers, ports)]
        try:
            while True:
                await asyncio.sleep(3600)
        finally:
            for r in runners:
                await r.cleanup()

    try:
        asyncio.run(main())
    except KeyboardInterrupt:
        pass


def now_ms() -> float:
    return time.monotonic() * 1000.0
