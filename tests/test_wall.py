"""Tiled-wall control flow on CPU with torch.distributed gloo (SURVEY.md §4.2 multi-GPU
tier): tiles rendered per rank, exchanged (direct gather and ring all-gather), composited
on rank 0, encoded, decoded and compared with a single-process render of the full wall."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mxdesk.codec.h264_decoder import Decoder
from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12, read_barcode
from mxdesk.parallel.wall import WallGeometry, WallPipeline, follower_loop


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cols, rows, mode, q, codec="h264"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    geo = WallGeometry(cols, rows, 320, 48)
    dev = torch.device("cpu")
    try:
        if rank != 0:
            follower_loop(geo, rank, world, dev, mode, fps=30)
            return
        pipe = WallPipeline(geo, 30, 0, world, dev, mode, bitrate_kbps=0, codec=codec)
        stream = b""
        for _ in range(3):
            stream += pipe.step().au
        wall_y = pipe.wy.numpy()[: geo.height, : geo.width].copy()
        pipe.lockstep_frame(False, stop=True)
        q.put((stream, wall_y))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cols,rows,mode,codec", [(2, 1, "gather", "h264"), (2, 2, "allgather", "h264"),
                                                  (1, 2, "gather", "h264"), (2, 2, "gather", "hevc")])
def test_wall_gloo(cols, rows, mode, codec):
    """The pipelined wall (exchange of frame n+1 posted before frame n is encoded) composes
    exactly the single-process render; the 4-rank HEVC variant is the 8K wall's codec."""
    world = cols * rows
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cols, rows, mode, q, codec)) for r in range(world)]
    for p in procs:
        p.start()
    stream, wall_y = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    geo = WallGeometry(cols, rows, 320, 48)
    ref = CpuSyntheticDesktop(geo.width, geo.height)
    for fid in range(3):  # same rng sequence as every rank
        img = ref.render(fid, fid / 30, 0)
    # composite == single-process render of the full wall (except the barcode timestamp row)
    ry, _ = bgrx_to_nv12(img)
    mask = np.ones_like(ry, bool)
    mask[8 + 8: 8 + 16, :] = False  # timestamp cells differ (capture time)
    assert np.array_equal(wall_y[mask], ry[mask])
    if codec == "hevc":
        from mxdesk.codec.hevc_decoder import Decoder as HevcDecoder

        frames = HevcDecoder().decode(stream)
    else:
        frames = Decoder().decode(stream)
    assert len(frames) == 3 and frames[0][0].shape == (geo.height, geo.width)
    assert read_barcode(frames[2][0])[0] == 2


def test_tile_stream_mode_matches_wall_region():
    """MXDESK_WALL_MODE=tiles: rank 1 of a 2x1 wall serves its own tile as a stream; the decoded
    tile equals that region of the full wall render (no process group needed)."""
    from mxdesk.parallel.wall import TilePipeline

    geo = WallGeometry(2, 1, 160, 48)
    pipe = TilePipeline(geo, 30, 1, torch.device("cpu"), bitrate_kbps=0)
    stream = b"".join(pipe.step().au for _ in range(2))
    frames = Decoder().decode(stream)
    assert len(frames) == 2 and frames[0][0].shape == (48, 160)
    ref = CpuSyntheticDesktop(geo.width, geo.height)
    for fid in range(2):
        img = ref.render(fid, fid / 30, 0)
    ry, _ = bgrx_to_nv12(img)
    rec = pipe.wy.numpy()[:48, :160]
    keep = np.ones((48, 160), bool)
    keep[16:24, :] = False  # barcode timestamp cells (capture time)
    assert np.array_equal(rec[keep], ry[:, 160:320][keep])
