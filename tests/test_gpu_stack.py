"""GPU tests of the stack around the encoder: GPU streaming pipeline through the web server
to a headless viewer, GPU frame grabbing for RFB, and the wall on one rank over RCCL."""
import asyncio
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from mxdesk.codec.h264_decoder import Decoder  # noqa: E402
from mxdesk.models.synthetic import read_barcode  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gpu_pipeline_through_server(gpu):
    from mxdesk.pipeline.stream import StreamPipeline
    from mxdesk.server.app import MediaServer, serve
    from mxdesk.server.client import view
    from mxdesk.utils import config as C

    cfg = C.load(env={"ENABLE_BASIC_AUTH": "false", "SIZEW": "320", "SIZEH": "192"}, argv=[])
    pipe = StreamPipeline(320, 192, 60, backend="gpu", bitrate_kbps=0)
    srv = MediaServer(pipe, cfg)

    async def go():
        port = _free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await view(f"http://127.0.0.1:{port}/mxws", 8)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    frames = Decoder().decode(res.stream)
    assert len(frames) == 8
    for (y, _, _), meta in zip(frames, res.frames):
        assert read_barcode(y)[0] == meta["frame_id"]
    assert res.p50_ms < 50


def test_gpu_pipeline_over_webrtc(gpu, monkeypatch):
    """GPU encoder -> WHEP/DTLS-SRTP -> depacketize -> independent decoder, with NACK + PLI."""
    from mxdesk.pipeline.stream import StreamPipeline
    from mxdesk.server.app import MediaServer, serve
    from mxdesk.server.whep_client import whep_view
    from mxdesk.utils import config as C

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg = C.load(env={"ENABLE_BASIC_AUTH": "false", "SIZEW": "320", "SIZEH": "192"}, argv=[])
    pipe = StreamPipeline(320, 192, 60, backend="gpu", bitrate_kbps=0)
    srv = MediaServer(pipe, cfg)

    async def go():
        port = _free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await whep_view(f"http://127.0.0.1:{port}/whep", 16, drop_seq_every=5, pli_after=6)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    frames = Decoder().decode(res.stream)
    assert len(frames) == 16 and res.rtx == res.lost
    ids = [read_barcode(y)[0] for y, _, _ in frames]
    assert all(b == a + 1 for a, b in zip(ids, ids[1:]))


def test_gpu_pipeline_over_selkies_signalling(gpu, monkeypatch):
    """GPU encoder -> selkies streaming peer on /ws (server offer, client answer) -> DTLS-SRTP
    -> independent decoder; input messages on the server-opened ``input`` channel."""
    from mxdesk.pipeline.stream import StreamPipeline
    from mxdesk.server.app import MediaServer, serve
    from mxdesk.server.selkies_client import selkies_view
    from mxdesk.utils import config as C

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg = C.load(env={"ENABLE_BASIC_AUTH": "false", "SIZEW": "320", "SIZEH": "192"}, argv=[])
    pipe = StreamPipeline(320, 192, 60, backend="gpu", bitrate_kbps=0)
    srv = MediaServer(pipe, cfg)

    async def go():
        port = _free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await selkies_view(f"ws://127.0.0.1:{port}/ws", 12, dc_messages=["m,10,20,0,0"])
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    frames = Decoder().decode(res.stream)
    assert len(frames) == 12 and res.dc_labels == ["input"]
    ids = [read_barcode(y)[0] for y, _, _ in frames]
    assert all(b == a + 1 for a, b in zip(ids, ids[1:]))


def test_gpu_live_resize_and_webrtc_datachannel_input(gpu, monkeypatch):
    """Client-driven resize on the HIP session (new Session at the new size, IDR first, the
    independent decoder sees the new dimensions) and input over the SCTP data channel."""
    from mxdesk.pipeline.stream import StreamPipeline
    from mxdesk.server.app import MediaServer, serve
    from mxdesk.server.whep_client import whep_view
    from mxdesk.utils import config as C

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg = C.load(env={"ENABLE_BASIC_AUTH": "false", "SIZEW": "320", "SIZEH": "192",
                      "WEBRTC_ENABLE_RESIZE": "true"}, argv=[])
    pipe = StreamPipeline(320, 192, 60, backend="gpu", bitrate_kbps=0, paced=False)
    a = pipe.step()
    assert (a.width, a.height) == (320, 192)
    assert pipe.resize(647, 360) == (640, 360)
    frs = [pipe.step() for _ in range(4)]
    assert all((f.width, f.height) == (640, 360) for f in frs) and frs[0].idr
    dec = Decoder().decode(b"".join(f.au for f in frs))
    assert len(dec) == 4 and dec[0][0].shape == (360, 640)
    ids = [read_barcode(y)[0] for y, _, _ in dec]
    assert all(b == x + 1 for x, b in zip(ids, ids[1:]))

    pipe2 = StreamPipeline(320, 192, 60, backend="gpu", bitrate_kbps=0)
    srv = MediaServer(pipe2, cfg)

    async def go():
        port = _free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await whep_view(f"http://127.0.0.1:{port}/whep", 6, dc_messages=["m,10,20,0,0", "kd,97"])
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    assert len(Decoder().decode(res.stream)) == 6
    assert (srv.injector.x, srv.injector.y) == (10, 20) and srv.injector.keys_down == {97}


def test_gpu_framegrab_matches_synth(gpu):
    from mxdesk.server.framegrab import FrameGrabber

    fg = FrameGrabber(320, 192, 60, backend="gpu")
    a = fg.grab()
    assert a.shape == (192, 320, 4) and a[..., 3].min() == 255
    fid, _ = read_barcode(((47 * a[..., 2].astype(int) + 157 * a[..., 1] + 16 * a[..., 0] + 128) >> 8) + 16)
    assert fid == 0


def test_gpu_wall_single_rank_rccl(gpu):
    import torch.distributed as dist

    from mxdesk.parallel.wall import WallGeometry, WallPipeline

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        for mode in ("gather", "allgather"):
            pipe = WallPipeline(WallGeometry(1, 1, 320, 192), 60, 0, 1, torch.device("cuda", 0), mode,
                                bitrate_kbps=0)
            stream = b"".join(pipe.step().au for _ in range(3))
            frames = Decoder().decode(stream)
            assert len(frames) == 3 and read_barcode(frames[2][0])[0] == 2
    finally:
        dist.destroy_process_group()


def test_gpu_composite_nv12_kernel_matches_copies(gpu):
    """k_composite_nv12 (one launch for all tiles and both planes) == per-tile tensor copies."""
    from mxdesk.parallel.wall import WallGeometry

    geo = WallGeometry(2, 2, 96, 32)
    tiles = torch.randint(0, 256, (4 * geo.tile_bytes,), dtype=torch.uint8, device="cuda")
    pitch = 256
    y = torch.zeros((geo.height, pitch), dtype=torch.uint8, device="cuda")
    uv = torch.zeros((geo.height // 2, pitch), dtype=torch.uint8, device="cuda")
    gpu.composite_nv12(tiles.data_ptr(), geo.tile_w, geo.tile_h, 2, 2, y.data_ptr(), uv.data_ptr(), pitch,
                       torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ry, ruv = torch.zeros_like(y), torch.zeros_like(uv)
    tb, tw, th = geo.tile_bytes, geo.tile_w, geo.tile_h
    for r in range(4):
        ox, oy = geo.origin(r)
        t = tiles[r * tb:(r + 1) * tb]
        ry[oy:oy + th, ox:ox + tw] = t[: tw * th].view(th, tw)
        ruv[oy // 2:oy // 2 + th // 2, ox:ox + tw] = t[tw * th:].view(th // 2, tw)
    assert torch.equal(y, ry) and torch.equal(uv, ruv)


def test_gpu_wall_hevc_single_rank(gpu):
    """The wall's HEVC path (its codec above 4K) through RCCL with one rank."""
    import torch.distributed as dist

    from mxdesk.codec.hevc_decoder import Decoder as HevcDecoder
    from mxdesk.parallel.wall import WallGeometry, WallPipeline

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        pipe = WallPipeline(WallGeometry(1, 1, 320, 192), 60, 0, 1, torch.device("cuda", 0), "gather",
                            bitrate_kbps=0, codec="hevc")
        stream = b"".join(pipe.step().au for _ in range(3))
        frames = HevcDecoder().decode(stream)
        assert len(frames) == 3 and read_barcode(frames[2][0])[0] == 2
    finally:
        dist.destroy_process_group()


def test_gpu_telemetry_sysfs(gpu):
    """amdgpu sysfs telemetry of the visible GPU feeds the mxdesk_gpu gauges of /metrics."""
    from mxdesk.utils import devices as D

    vis = D.visible_gpus(D.enumerate_gpus())
    assert vis, "no AMD render node found in sysfs"
    t = D.gpu_telemetry(vis[0].pci_bdf)
    print("telemetry", vis[0].pci_bdf, t)
    assert "vram_total_bytes" in t or "busy_percent" in t


def _gpu_wall_worker(rank, world, port, q):
    import torch.distributed as dist

    from mxdesk.parallel.wall import WallGeometry, WallPipeline, follower_loop

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    geo = WallGeometry(2, 1, 160, 96)
    try:
        if rank != 0:
            follower_loop(geo, rank, world, dev, "gather", fps=60)
            return
        pipe = WallPipeline(geo, 60, 0, world, dev, "gather", bitrate_kbps=0)
        stream = b"".join(pipe.step().au for _ in range(3))
        torch.cuda.synchronize()
        # two frames in flight on the encode rank: frame 2's composite is in wall buffer 2 % 2
        wall_y = pipe._walls[2 % len(pipe._walls)][0].cpu().numpy()[: geo.height, : geo.width].copy()
        pipe.lockstep_frame(False, stop=True)
        q.put((stream, wall_y))
    finally:
        dist.destroy_process_group()


def test_gpu_wall_two_processes_one_gpu():
    """Two wall ranks as two processes on the one GPU (gloo, host-staged tile exchange): the
    HIP render / composite / encode path of a multi-rank wall, decoded and compared with one
    render of the full wall."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_wall_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        stream, wall_y = q.get(timeout=150)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    frames = Decoder().decode(stream)
    assert len(frames) == 3 and frames[0][0].shape == (96, 320)
    assert read_barcode(frames[2][0])[0] == 2
    # the composite equals one render of the full wall (frame 2; barcode timestamp row aside)
    from mxdesk import native

    N = native()
    w, h = 320, 96
    a = torch.zeros((h, w * 4), dtype=torch.uint8, device="cuda")
    N.synth(a.data_ptr(), w, h, w * 4, frame_id=2, t=2 / 60, stream=torch.cuda.current_stream().cuda_stream)
    y = torch.zeros((h, w), dtype=torch.uint8, device="cuda")
    uv = torch.zeros((h // 2, w), dtype=torch.uint8, device="cuda")
    N.bgrx_to_nv12(a.data_ptr(), w * 4, w, h, y.data_ptr(), uv.data_ptr(), w, w, h,
                   torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = y.cpu().numpy()
    mask = np.ones_like(ref, bool)
    mask[8 + 8: 8 + 16, :] = False  # timestamp cells (capture time)
    assert np.array_equal(wall_y[mask], ref[mask])


class _FakeCapture:
    """A capture whose "SHM segment" is a numpy buffer; with ``damage`` it follows
    X11Capture's damage-driven protocol (the segment's undamaged rows keep stale data)."""

    def __init__(self, frames, w, h, damage):
        self.frames, self.w, self.h, self.i = frames, w, h, 0
        self.buf = np.zeros((h, w * 4), np.uint8)
        if damage:
            self.damage = self
            self.full = True
            self.bands_log = []

    def invalidate(self):
        self.full = True

    def shm_buffer(self):
        return (self.buf.ctypes.data, self.buf.nbytes) if hasattr(self, "damage") else None

    def grab(self):
        f = self.frames[self.i]
        self.i += 1
        return f.reshape(self.h, self.w, 4)

    def grab_shm_damage(self):
        f = self.frames[self.i]
        prev = self.frames[self.i - 1] if self.i else None
        self.i += 1
        if self.full or prev is None:
            bands, self.full = [(0, self.h)], False
        else:
            rows = np.nonzero((f != prev).any(axis=1))[0]
            bands = [(int(rows.min()) // 16 * 16, min(self.h, (int(rows.max()) // 16 + 1) * 16))] if len(rows) else []
        self.buf[:] = 0
        for y0, y1 in bands:
            self.buf[y0:y1] = f[y0:y1]
        self.bands_log.append(bands)
        return self.buf.ctypes.data, self.w * 4, bands


def test_gpu_pipeline_damage_capture_matches_full_grab(gpu):
    """StreamPipeline's damage-driven capture path (XDamage bands -> submit_bgrx_damage)
    produces the same access units as full-frame grabs of the same screens."""
    from mxdesk.pipeline.stream import StreamPipeline

    w, h = 320, 192
    rng = np.random.default_rng(5)
    frames = [rng.integers(0, 256, (h, w * 4), dtype=np.uint8)]
    for i in range(4):
        f = frames[-1].copy()
        if i != 1:  # frame 2 is unchanged (no bands)
            f[20 * i + 10: 20 * i + 40, 40:200] = rng.integers(0, 256, (30, 160), dtype=np.uint8)
        frames.append(f)
    full = _FakeCapture(frames, w, h, damage=False)
    dmg = _FakeCapture(frames, w, h, damage=True)
    pa = StreamPipeline(w, h, 60, backend="gpu", bitrate_kbps=0, capture=full)
    pb = StreamPipeline(w, h, 60, backend="gpu", bitrate_kbps=0, capture=dmg)
    for i in range(len(frames)):
        a, b = pa.step(), pb.step()
        assert a.au == b.au, f"frame {i}"
    assert dmg.bands_log[0] == [(0, h)] and dmg.bands_log[2] == []
    assert pb._sess.damage_bytes_uploaded < len(frames) * w * h * 4 // 2


def test_gpu_pipeline_damage_idle_screen_pauses_production(gpu, monkeypatch):
    """Damage-driven frame rate: after MXDESK_IDLE_AFTER frames without damage the pipeline
    produces nothing until the screen changes; the frames it does produce form one decodable
    stream whose last picture is the changed screen."""
    from mxdesk.models.synthetic import bgrx_to_nv12
    from mxdesk.pipeline.stream import StreamPipeline

    monkeypatch.setenv("MXDESK_IDLE_AFTER", "3")
    w, h = 320, 192
    rng = np.random.default_rng(8)
    f0 = rng.integers(0, 256, (h, w * 4), dtype=np.uint8)
    f1 = f0.copy()
    f1[64:128, 64:256] = 30
    frames = [f0] * 8 + [f1, f1]
    cap = _FakeCapture(frames, w, h, damage=True)
    pipe = StreamPipeline(w, h, 60, backend="gpu", bitrate_kbps=0, capture=cap)
    out = [pipe.step() for _ in frames]
    produced = [fr is not None for fr in out]
    assert produced == [True, True, True, True, False, False, False, False, True, True], produced
    assert pipe.frames_idle == 4 and pipe.status()["frames_idle"] == 4
    stream = b"".join(fr.au for fr in out if fr is not None)
    dec = Decoder().decode(stream)
    assert len(dec) == 6
    y_src, _ = bgrx_to_nv12(f1.reshape(h, w, 4))
    err = dec[-1][0].astype(np.float64) - y_src.astype(np.float64)
    assert 10 * np.log10(255 ** 2 / max(1e-9, float((err ** 2).mean()))) > 30


def test_gpu_x11_capture_through_fake_server(gpu, monkeypatch):
    """Real libX11 / libXext / libXdamage / libXfixes against tests/fake_xserver.py: MIT-SHM
    capture registered for zero-copy DMA, XDamage bands, GPU encode; the decoded pictures are
    the X framebuffer's, and a small change uploads only its band."""
    import ctypes.util

    if not all(ctypes.util.find_library(n) for n in ("X11", "Xext", "Xdamage", "Xfixes")):
        pytest.skip("X client libraries not installed")
    from mxdesk.models.synthetic import bgrx_to_nv12
    from mxdesk.models.x11 import X11Capture
    from mxdesk.pipeline.stream import StreamPipeline
    from tests.fake_xserver import FakeXServer

    monkeypatch.setenv("MXDESK_IDLE_AFTER", "2")
    w, h = 320, 192
    srv = FakeXServer(w, h)
    try:
        yy, xx = np.mgrid[0:h, 0:w]
        srv.fb[..., 0] = (xx * 255 // w).astype(np.uint8)
        srv.fb[..., 1] = (yy * 255 // h).astype(np.uint8)
        srv.fb[..., 2] = 128
        cap = X11Capture(srv.display)
        assert cap.enable_damage()
        pipe = StreamPipeline(w, h, 60, backend="gpu", bitrate_kbps=0, capture=cap)
        out = [pipe.step() for _ in range(4)]  # IDR, 2 static frames, then idle
        assert [f is not None for f in out] == [True, True, True, False]
        srv.draw(40, 70, 100, 20, 240)
        out.append(pipe.step())
        assert out[-1] is not None
        up = pipe._sess.damage_bytes_uploaded
        assert up == w * 4 * (h + 32)  # the first frame + one 32-row band (rows 64..96)
        frames = Decoder().decode(b"".join(f.au for f in out if f is not None))
        assert len(frames) == 4
        y_src, _ = bgrx_to_nv12(srv.fb)
        err = frames[-1][0].astype(np.float64) - y_src.astype(np.float64)
        assert 10 * np.log10(255 ** 2 / max(1e-9, float((err ** 2).mean()))) > 35
    finally:
        srv.close()
