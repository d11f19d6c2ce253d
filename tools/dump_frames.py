#!/usr/bin/env python3
"""Dump the bench desktop's NV12 frames (HIP-rendered, deterministic clock) so that encoder
quality work can iterate on the CPU oracle encoder (bit-exact with the GPU encoder) without a
GPU.  Writes an .npz with y[n, H, P] / uv[n, H/2, P] (coded size) and the GPU encoder's
per-frame stats at the bench settings for cross-checking.

    python tools/dump_frames.py --frames 30 --out gpurun_out/frames_1080p.npz
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bitrate-kbps", type=int, default=8000)
    ap.add_argument("--out", default="gpurun_out/frames_1080p.npz")
    ap.add_argument("--content", default="desktop", choices=["desktop", "motion", "subpel"])
    a = ap.parse_args()
    import mxdesk

    N = mxdesk.native()
    N.set_device(0)
    cfg = N.SessionConfig()
    cfg.width, cfg.height, cfg.fps = a.width, a.height, 60
    cfg.fake_clock = 1
    cfg.content = {"desktop": 0, "motion": 1, "subpel": 2}[a.content]
    if a.content != "desktop":
        cfg.noise = 0  # as bench.py: the moving contents carry a video panel instead of the noise panel
    cfg.enc.bitrate_kbps = a.bitrate_kbps
    ow, oh = a.width, a.height
    cfg.mask_x0, cfg.mask_y0 = int(ow * 0.04), int(oh * 0.55)
    cfg.mask_x1, cfg.mask_y1 = cfg.mask_x0 + int(ow * 0.16) + 1, cfg.mask_y0 + int(oh * 0.22) + 1
    s = N.Session(cfg)
    ys, uvs, stats = [], [], []
    for i in range(a.frames):
        r = s.step(False)
        y, uv = s.nv12()
        ys.append(y)
        uvs.append(uv)
        stats.append({"idr": r.idr, "qp": r.qp, "bytes": len(r.au), "psnr_y": r.psnr_y,
                      "psnr_y_masked": r.psnr_y_masked})
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(a.out, y=np.stack(ys), uv=np.stack(uvs), width=a.width, height=a.height,
                        mask=np.array([cfg.mask_x0, cfg.mask_y0, cfg.mask_x1, cfg.mask_y1]))
    Path(a.out).with_suffix(".json").write_text(json.dumps(stats, indent=1))
    print(json.dumps(stats[-3:]))


if __name__ == "__main__":
    main()
