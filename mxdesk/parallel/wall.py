"""Tiled video wall: N GPUs render one tile each, tiles are exchanged over RCCL/xGMI and the
composite is encoded as a single stream (BASELINE.json config 5
"2x2 tiled 8K60 wall: 4-GPU render, RCCL all-gather composite over xGMI").

Per frame, on every rank (one process per GPU, ``torch.distributed`` backend ``nccl`` =
RCCL on ROCm; ``gloo`` for CPU tests):
  1. rank 0 broadcasts a small control tensor (frame id, stop, capture time) -> lockstep;
  2. each rank renders its tile of the wall (HIP synthetic desktop with a tile origin) and
     converts it to NV12 on its own GPU (HIP CSC), so only 1.5 B/pixel cross xGMI;
  3. the tiles reach the encode rank either by a ring ``all_gather_into_tensor``
     (``exchange="allgather"``) or by a direct gather -- one batched send/recv per peer, so
     the encode rank pulls the three tiles over three xGMI links at once
     (``exchange="gather"``; xGMI is point-to-point, a ring is per-link bound);
  4. the encode rank composites the NV12 tiles into the wall frame with one HIP launch
     (k_composite_nv12) and encodes it -- HEVC by default above 4K (an 8K H.264 stream needs
     level 6.x, which browser decoders rarely take; HEVC 8K is level 6.1).
Pipelining on the encode rank: frame n+1's lockstep render + tile exchange is posted (RCCL
runs it on its own stream, the followers render meanwhile) BEFORE frame n is encoded, so
exchange(n+1) overlaps encode(n); the control tensor goes up with one host->device copy.
``MXDESK_WALL_MODE=tiles`` skips the composite: every rank serves its own tile as an
independent stream (port + rank) for clients that cannot decode the full wall's level.
If process-group initialisation fails the launcher falls back to per-GPU sessions
(SURVEY.md §5.3).
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import dataclass
from typing import Any

import numpy as np
import torch
import torch.distributed as dist

from ..models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12
from ..pipeline.stream import EncodedFrame, StreamPipeline, cpu_encoder_class

log = logging.getLogger("mxdesk.wall")

# Followers read the control tensor on the host only every CTRL_POLL frames (to see `stop` and
# check lockstep); in between they enqueue broadcast, render and exchange without a host sync.
# The leader therefore stops only at a frame id that is a multiple of CTRL_POLL.
CTRL_POLL = 8


def parse_layout(layout: str) -> tuple[int, int]:
    c, r = layout.lower().split("x")
    return int(c), int(r)


@dataclass
class WallGeometry:
    cols: int
    rows: int
    tile_w: int
    tile_h: int

    @property
    def width(self) -> int:
        return self.cols * self.tile_w

    @property
    def height(self) -> int:
        return self.rows * self.tile_h

    @property
    def tile_bytes(self) -> int:
        return self.tile_w * self.tile_h * 3 // 2

    def origin(self, rank: int) -> tuple[int, int]:
        return (rank % self.cols) * self.tile_w, (rank // self.cols) * self.tile_h


class TileRenderer:
    """Renders + converts one tile to packed NV12 (Y rows then interleaved UV rows)."""

    def __init__(self, geo: WallGeometry, rank: int, device: torch.device, noise: bool = True):
        self.geo, self.rank, self.device = geo, rank, device
        self.ox, self.oy = geo.origin(rank)
        tw, th = geo.tile_w, geo.tile_h
        self.out = torch.empty(geo.tile_bytes, dtype=torch.uint8, device=device)
        if device.type == "cuda":
            from .. import native

            self.N = native()
            self.pitch = ((tw * 4) + 255) // 256 * 256
            self.bgrx = torch.empty((th, self.pitch), dtype=torch.uint8, device=device)
        else:
            self.N = None
            self.desk = CpuSyntheticDesktop(geo.width, geo.height, noise)

    def render(self, frame_id: int, t: float, ts_us: int) -> torch.Tensor:
        g = self.geo
        if self.N is not None:
            st = torch.cuda.current_stream(self.device).cuda_stream
            self.N.synth(self.bgrx.data_ptr(), g.tile_w, g.tile_h, self.pitch, frame_id, ts_us & 0xFFFFFFFF, t, 1,
                         self.ox, self.oy, g.width, g.height, -1, -1, st)
            y_ptr = self.out.data_ptr()
            uv_ptr = y_ptr + g.tile_w * g.tile_h
            self.N.bgrx_to_nv12(self.bgrx.data_ptr(), self.pitch, g.tile_w, g.tile_h, y_ptr, uv_ptr, g.tile_w,
                                g.tile_w, g.tile_h, st)
            return self.out
        full = self.desk.render(frame_id, t, ts_us)
        tile = np.ascontiguousarray(full[self.oy:self.oy + g.tile_h, self.ox:self.ox + g.tile_w])
        y, uv = bgrx_to_nv12(tile)
        self.out.copy_(torch.from_numpy(np.concatenate([y.reshape(-1), uv.reshape(-1)])))
        return self.out


def host_staged(device: torch.device) -> bool:
    """GPU tiles over a gloo process group (no RCCL, e.g. several ranks sharing one GPU): the
    exchange and the control broadcast go through host tensors."""
    return device.type == "cuda" and dist.is_initialized() and dist.get_backend() == "gloo"


class TileExchange:
    def __init__(self, geo: WallGeometry, rank: int, world: int, device: torch.device, mode: str = "gather",
                 root: int = 0):
        if world != geo.cols * geo.rows:
            raise ValueError(f"wall {geo.cols}x{geo.rows} needs {geo.cols * geo.rows} ranks, got {world}")
        self.geo, self.rank, self.world, self.mode, self.root = geo, rank, world, mode, root
        holds = rank == root or mode == "allgather"
        self.tiles = torch.empty(world * geo.tile_bytes, dtype=torch.uint8, device=device) if holds else None
        self.staged = host_staged(device)
        if self.staged:
            self._tile_h = torch.empty(geo.tile_bytes, dtype=torch.uint8).pin_memory()
            self._tiles_h = torch.empty(world * geo.tile_bytes, dtype=torch.uint8).pin_memory() if holds else None

    def post(self, tile: torch.Tensor) -> list:
        """Start the exchange of this rank's tile; returns the requests to wait for."""
        tiles = self.tiles
        if self.staged:
            self._tile_h.copy_(tile)  # synchronous: the send reads host memory
            tile, tiles = self._tile_h, self._tiles_h
        if self.mode == "allgather":
            return [dist.all_gather_into_tensor(tiles, tile, async_op=True)]
        tb = self.geo.tile_bytes
        if self.rank == self.root:
            tiles[self.root * tb:(self.root + 1) * tb].copy_(tile)
            ops = [dist.P2POp(dist.irecv, tiles[r * tb:(r + 1) * tb], r) for r in range(self.world)
                   if r != self.root]
        else:
            ops = [dist.P2POp(dist.isend, tile, self.root)]
        return dist.batch_isend_irecv(ops) if ops else []  # world size 1: nothing to exchange

    def wait(self, reqs: list) -> torch.Tensor | None:
        for req in reqs:
            req.wait()
        if self.tiles is not None and self.staged:
            self.tiles.copy_(self._tiles_h, non_blocking=True)
        return self.tiles if self.rank == self.root else None

    def exchange(self, tile: torch.Tensor) -> torch.Tensor | None:
        return self.wait(self.post(tile))


def composite_nv12(tiles: torch.Tensor, geo: WallGeometry, y: torch.Tensor, uv: torch.Tensor) -> None:
    """Place packed NV12 tiles into the wall planes y (H, P) and uv (H/2, P): one HIP launch on
    the GPU (k_composite_nv12), tensor copies on the CPU."""
    tb, tw, th = geo.tile_bytes, geo.tile_w, geo.tile_h
    if tiles.device.type == "cuda":
        from .. import native

        native().composite_nv12(tiles.data_ptr(), tw, th, geo.cols, geo.rows, y.data_ptr(), uv.data_ptr(),
                                y.stride(0), torch.cuda.current_stream(tiles.device).cuda_stream)
        return
    for r in range(geo.cols * geo.rows):
        ox, oy = geo.origin(r)
        t = tiles[r * tb:(r + 1) * tb]
        y[oy:oy + th, ox:ox + tw].copy_(t[: tw * th].view(th, tw))
        uv[oy // 2:oy // 2 + th // 2, ox:ox + tw].copy_(t[tw * th:].view(th // 2, tw))


class WallPipeline(StreamPipeline):
    """Rank-0 pipeline: lockstep tile render on every rank, exchange, composite, encode."""

    def __init__(self, geo: WallGeometry, fps: int, rank: int, world: int, device: torch.device,
                 exchange: str = "gather", bitrate_kbps: int = 20000, codec: str | None = None, **kw):
        self.geo, self.rank, self.world, self.dev = geo, rank, world, device
        self.renderer = TileRenderer(geo, rank, device)
        self.xchg = TileExchange(geo, rank, world, device, exchange)
        staged = host_staged(device)
        self.ctrl = torch.zeros(4, dtype=torch.int64, device="cpu" if staged else device)
        self._ctrl_host = torch.zeros(4, dtype=torch.int64).pin_memory() \
            if (device.type == "cuda" and not staged) else self.ctrl
        self._t0 = time.monotonic()
        self._fid = 0
        self._pending = None  # (frame id, capture us, exchange requests) of the posted frame
        # above 4K the wall goes out as HEVC (level 6.1 at 8K; H.264 would need level 6.x)
        wall_codec = codec or ("hevc" if geo.width > 4096 else "h264")
        super().__init__(geo.width, geo.height, fps, backend="gpu" if device.type == "cuda" else "cpu",
                         device=device.index or 0, bitrate_kbps=bitrate_kbps, codec=wall_codec, **kw)

    def _make_session(self) -> None:
        from .. import native

        N = native()
        cw, ch = (self.geo.width + 15) // 16 * 16, (self.geo.height + 15) // 16 * 16
        ec = N.EncoderConfig()
        ec.width, ec.height, ec.fps = self.geo.width, self.geo.height, self.fps
        ec.bitrate_kbps = self._enc_args["bitrate_kbps"]
        ec.search_range = self._enc_args["search_range"]
        ec.subpel = 1 if self._enc_args["subpel"] else 0
        if self.dev.type == "cuda":
            # two frames in flight: submit(n + 1) before collect(n), so the host composites and
            # launches frame n + 1 while the GPU still encodes (and entropy-codes) frame n
            ec.pipeline_depth = 2
            cls = {"h264": N.GpuH264Encoder, "hevc": N.GpuHevcEncoder, "vp8": N.GpuVp8Encoder}[self.codec]
            self.enc = cls(ec, torch.cuda.current_stream(self.dev).cuda_stream)
            pitch = self.enc.pitch
        else:
            ec.search_range = min(ec.search_range, 4)
            ec.subpel = 0
            self.enc = cpu_encoder_class(N, self.codec)(ec)
            pitch = cw
        nbuf = 2 if self.dev.type == "cuda" else 1  # the encoder may still read the previous wall frame
        self._walls = [(torch.zeros((ch, pitch), dtype=torch.uint8, device=self.dev),
                        torch.zeros((ch // 2, pitch), dtype=torch.uint8, device=self.dev)) for _ in range(nbuf)]
        self.wy, self.wuv = self._walls[0]
        self._submitted: list[tuple[int, int]] = []  # (frame id, capture us) submitted, not collected
        self._sess = None
        self._cpu = self.enc if self.dev.type != "cuda" else None

    def set_bitrate(self, kbps: int) -> None:
        self.enc.set_bitrate(int(kbps))

    def _broadcast_ctrl(self, fid: int, stop: bool, t_cap: int) -> None:
        h = self._ctrl_host
        h[0], h[1], h[2], h[3] = fid, 0, int(stop), t_cap
        if h is not self.ctrl:
            self.ctrl.copy_(h, non_blocking=True)  # one host->device copy, not four element writes
        dist.broadcast(self.ctrl, 0)

    def post_frame(self) -> tuple[int, int, list]:
        """Lockstep step of the next frame: control broadcast, own tile render, exchange posted."""
        from .. import native

        t_cap = native().now_us()
        fid = self._fid
        self._fid += 1
        self._broadcast_ctrl(fid, False, t_cap)
        tile = self.renderer.render(fid, fid / self.fps, t_cap)
        return fid, t_cap, self.xchg.post(tile)

    def lockstep_frame(self, force_idr: bool = False, stop: bool = False) -> torch.Tensor | None:
        """One unpipelined lockstep frame (tests / stop): returns the tiles on the encode rank."""
        if stop:
            self._drain()
            from .. import native

            while self._fid % CTRL_POLL:  # followers look at the control word on these frames only
                self.xchg.wait(self.post_frame()[2])
            self._broadcast_ctrl(self._fid, True, native().now_us())
            return None
        self._drain()
        _, _, reqs = self.post_frame()
        tiles = self.xchg.wait(reqs)
        if tiles is not None:
            composite_nv12(tiles, self.geo, self.wy, self.wuv)
        return tiles

    def _drain(self) -> None:
        while getattr(self, "_submitted", None):  # frames still in the encoder
            self.enc.collect()
            self._submitted.pop(0)
        if self._pending is not None:
            self.xchg.wait(self._pending[2])
            self._pending = None

    def _composite_next(self) -> tuple[int, int]:
        """Wait for the posted frame's tiles, composite them into the next wall buffer, post the
        following frame's render + exchange (followers and the RCCL stream run it while this frame
        encodes; the receive is ordered after the composite on the device -- RCCL waits on the
        current stream -- so one tile buffer suffices)."""
        if self._pending is None:
            self._pending = self.post_frame()
        fid, t_cap, reqs = self._pending
        tiles = self.xchg.wait(reqs)
        self.wy, self.wuv = self._walls[fid % len(self._walls)]
        composite_nv12(tiles, self.geo, self.wy, self.wuv)
        self._pending = self.post_frame()
        return fid, t_cap

    def _produce(self, force_idr: bool) -> EncodedFrame:
        from .. import native

        if self.dev.type == "cuda":
            while len(self._submitted) < 2:  # keep two frames in the encoder
                fid, t_cap = self._composite_next()
                self.enc.submit(self.wy.data_ptr(), self.wuv.data_ptr(), force_idr)
                self._submitted.append((fid, t_cap))
                force_idr = False
            au = self.enc.collect()
            fid, t_cap = self._submitted.pop(0)
        else:
            fid, t_cap = self._composite_next()
            au = self.enc.encode(self.wy.numpy()[: self.geo.height], self.wuv.numpy()[: self.geo.height // 2],
                                 force_idr)
        st = self.enc.stats
        return EncodedFrame(fid, t_cap, native().now_us(), bool(st.idr), st.qp, au, self.geo.width, self.geo.height,
                            codec_id=self.codec_id)

    def stop(self) -> None:
        super().stop()
        try:
            self.lockstep_frame(False, stop=True)
        except Exception:
            pass


class TilePipeline(WallPipeline):
    """``MXDESK_WALL_MODE=tiles``: this rank's tile of the wall as an independent stream (no
    exchange, no composite) -- the fallback for clients that cannot decode the whole wall's
    level; a client shows the tiles side by side."""

    def __init__(self, geo: WallGeometry, fps: int, rank: int, device: torch.device, bitrate_kbps: int = 8000,
                 codec: str | None = None, **kw):
        self.tile_geo = WallGeometry(1, 1, geo.tile_w, geo.tile_h)
        self.full_geo, self.rank, self.dev = geo, rank, device
        self.renderer = TileRenderer(geo, rank, device)
        self._fid = 0
        self._pending = None
        self.geo = self.tile_geo  # the encoder / composite see a 1x1 wall of this tile
        StreamPipeline.__init__(self, geo.tile_w, geo.tile_h, fps, backend="gpu" if device.type == "cuda" else "cpu",
                                device=device.index or 0, bitrate_kbps=bitrate_kbps,
                                codec=codec or ("hevc" if geo.tile_w > 4096 else "h264"), **kw)

    def _produce(self, force_idr: bool) -> EncodedFrame:
        from .. import native

        t_cap = native().now_us()
        fid = self._fid
        self._fid += 1
        tile = self.renderer.render(fid, fid / self.fps, t_cap)
        composite_nv12(tile, self.tile_geo, self.wy, self.wuv)
        if self.dev.type == "cuda":
            au = self.enc.encode(self.wy.data_ptr(), self.wuv.data_ptr(), force_idr)
        else:
            g = self.tile_geo
            au = self.enc.encode(self.wy.numpy()[: g.height], self.wuv.numpy()[: g.height // 2], force_idr)
        st = self.enc.stats
        g = self.tile_geo
        return EncodedFrame(fid, t_cap, native().now_us(), bool(st.idr), st.qp, au, g.width, g.height,
                            codec_id=self.codec_id)

    def stop(self) -> None:
        StreamPipeline.stop(self)


def follower_loop(geo: WallGeometry, rank: int, world: int, device: torch.device, exchange: str = "gather",
                  fps: int = 60) -> int:
    """Ranks != 0: render + send tiles in lockstep until rank 0 broadcasts stop.  The frame id
    advances by one per lockstep frame on every rank, so a follower renders from its own counter
    and reads the control tensor on the host only every CTRL_POLL frames (stop + a lockstep
    check); the frames between are enqueued without a host sync.  The capture timestamp only
    feeds the barcode, which lies in rank 0's tile."""
    renderer = TileRenderer(geo, rank, device)
    xchg = TileExchange(geo, rank, world, device, exchange)
    ctrl = torch.zeros(4, dtype=torch.int64, device="cpu" if host_staged(device) else device)
    fid = 0
    while True:
        dist.broadcast(ctrl, 0)
        if fid % CTRL_POLL == 0:
            lfid, _, stop, _ = (int(x) for x in ctrl.tolist())
            if stop:
                return fid
            if lfid != fid:
                raise RuntimeError(f"wall: rank {rank} out of lockstep (frame {fid}, leader {lfid})")
        xchg.exchange(renderer.render(fid, fid / fps, 0))
        fid += 1


def init_distributed(backend: str | None = None) -> tuple[int, int, torch.device]:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    device = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend or ("nccl" if use_gpu else "gloo"),
                                **({"device_id": device} if use_gpu else {}))
    return rank, world, device


def wall_main(cfg: Any, layout: str = "2x2", argv: list[str] | None = None) -> int:
    """``mxdesk wall``: one rank per tile.  Started bare (no WORLD_SIZE) it starts the cols x rows
    rank processes itself (``ranks.run_ranks``: fresh children of the same command, before any
    GPU call, signals forwarded) and returns their exit code; under torchrun WORLD_SIZE must equal
    cols x rows (else 2: a wall never runs with a rank per tile missing)."""
    import sys

    cols, rows = parse_layout(layout)
    need = cols * rows
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and need > 1:
        from .ranks import run_ranks

        print(f"mxdesk wall {cols}x{rows}: starting {need} rank processes", flush=True)
        return run_ranks([sys.executable, "-m", "mxdesk", "wall"] + list(argv or ["--layout", layout]), need)
    if ws is not None and int(ws) != need:
        print(f"mxdesk wall {cols}x{rows} needs {need} ranks (one per tile) but WORLD_SIZE={ws}: start it bare "
              f"(it launches its ranks) or with --nproc-per-node {need}", file=sys.stderr, flush=True)
        return 2
    try:
        rank, world, device = init_distributed()
    except Exception as e:  # degrade to per-GPU sessions
        log.error("wall: process group init failed (%s); falling back to per-GPU sessions", e)
        from .launcher import launch_sessions

        launch_sessions(cfg)
        return 0
    geo = WallGeometry(cols, rows, cfg.sizew, cfg.sizeh)
    exchange = os.environ.get("MXDESK_WALL_EXCHANGE", "gather")
    if os.environ.get("MXDESK_WALL_MODE", "composite") == "tiles":
        from ..server.app import MediaServer, run_forever, ssl_context

        pipe = TilePipeline(geo, cfg.stream_fps, rank, device, bitrate_kbps=cfg.video_bitrate)
        port = cfg.port + rank
        print(f"mxdesk wall {cols}x{rows} tiles: rank {rank} serves its {geo.tile_w}x{geo.tile_h} tile at "
              f"{geo.origin(rank)} on :{port}", flush=True)
        try:
            run_forever(MediaServer(pipe, cfg), cfg.addr, port, ssl_context(cfg))
        finally:
            pipe.stop()
            dist.destroy_process_group()
        return 0
    if rank != 0:
        follower_loop(geo, rank, world, device, exchange, cfg.stream_fps)
        dist.destroy_process_group()
        return 0
    from ..server.app import MediaServer, run_forever, ssl_context

    pipe = WallPipeline(geo, cfg.stream_fps, rank, world, device, exchange, bitrate_kbps=cfg.video_bitrate * 4)
    print(f"mxdesk wall {cols}x{rows}: {geo.width}x{geo.height} on {world} ranks, serving :{cfg.port}", flush=True)
    try:
        run_forever(MediaServer(pipe, cfg), cfg.addr, cfg.port, ssl_context(cfg))
    finally:
        pipe.stop()
        dist.destroy_process_group()
    return 0
