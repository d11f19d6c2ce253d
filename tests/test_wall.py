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


def _worker(rank, world, port, cols, rows, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    geo = WallGeometry(cols, rows, 320, 48)
    dev = torch.device("cpu")
    try:
        if rank != 0:
            follower_loop(geo, rank, world, dev, mode, fps=30)
            return
        pipe = WallPipeline(geo, 30, 0, world, dev, mode, bitrate_kbps=0)
        stream = b""
        for _ in range(3):
            stream += pipe.step().au
        wall_y = pipe.wy.numpy()[: geo.height, : geo.width].copy()
        pipe.lockstep_frame(False, stop=True)
        q.put((stream, wall_y))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cols,rows,mode", [(2, 1, "gather"), (2, 2, "allgather"), (1, 2, "gather")])
def test_wall_gloo(cols, rows, mode):
    world = cols * rows
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cols, rows, mode, q)) for r in range(world)]
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
    frames = Decoder().decode(stream)
    assert len(frames) == 3 and frames[0][0].shape == (geo.height, geo.width)
    assert read_barcode(frames[2][0])[0] == 2
