"""Debug: per-row timing of k_deblock (luma / chroma row waves) on a 1080p session."""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import mxdesk  # noqa: E402

N = mxdesk.native()
N.set_device(0)
khz = N.device_clock_khz()
for content in (1, 0):
    cfg = N.SessionConfig()
    cfg.width, cfg.height, cfg.fps = 1920, 1080, 60
    cfg.enc.bitrate_kbps = 8000
    cfg.enc.deblock = 1
    cfg.enc.pipeline_depth = 1
    cfg.content = content
    s = N.Session(cfg)
    for i in range(40):
        s.step(False)
    raw = np.array(N.h264_deblock_row_stamps(68), dtype=np.float64)
    st = raw[:2 * 68 * 5].reshape(2, 68, 5)
    ph = raw[2 * 68 * 5:2 * 68 * 5 + 68 * 4].reshape(68, 4) / khz * 1000
    ck = raw[2 * 68 * 5 + 68 * 4:].reshape(2, 68)
    dur_us = (st[:, :, 1] - st[:, :, 0]) / khz * 1000
    print("  effective shader clock MHz (cycles / wall us), luma rows 0..7:",
          " ".join(f"{ck[0, y] / dur_us[0, y]:.0f}" for y in range(8)))
    for nm, k in (("head", 0), ("V", 1), ("final", 2), ("H", 3)):
        print(f"  luma phase {nm} us:", " ".join(f"{v:.0f}" for v in ph[:, k]))
    t0 = st[:, :, 0].min()
    print(f"content {content}: kernel span {(st[:, :, 1].max() - t0) / khz * 1000:.1f} us")
    for p, name in ((0, "luma"), (1, "chroma")):
        end = (st[p, :, 1] - t0) / khz * 1000
        w = st[p, :, 2:] / khz * 1000
        print(f"  {name} end us:", " ".join(f"{v:.0f}" for v in end))
        print(f"  {name} wait ring:", " ".join(f"{v:.0f}" for v in w[:, 0]))
        print(f"  {name} wait above:", " ".join(f"{v:.0f}" for v in w[:, 1]))
        print(f"  {name} wait band:", " ".join(f"{v:.0f}" for v in w[:, 2]))
    del s
