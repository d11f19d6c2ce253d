"""HEVC IDR picture: bytes and luma PSNR with and without the intra transform-tree split
(EncoderConfig.hevc_intra_split), CPU encoder (the GPU's bit-exact oracle), fixed QPs, on the
numpy synthetic desktop.

    python tools/hevc_intra_split_rd.py [--width 1920 --height 1080 --qps 27,32,37,41]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--qps", default="27,32,37,41")
    a = ap.parse_args()
    import mxdesk
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    N = mxdesk.native()
    desk = CpuSyntheticDesktop(a.width, a.height, noise=True)
    y, uv = bgrx_to_nv12(desk.render(0, 0.0, 0))
    rows = []
    for qp in [int(q) for q in a.qps.split(",")]:
        for split in (0, 1):
            cfg = N.EncoderConfig()
            cfg.width, cfg.height, cfg.fps = a.width, a.height, 60
            cfg.bitrate_kbps, cfg.qp = 0, qp
            cfg.hevc_intra_split = split
            enc = N.CpuHevcEncoder(cfg)
            au = enc.encode(y, uv, True)
            ry = enc.recon()[0][: a.height, : a.width].astype(np.float64)
            mse = float(np.mean((ry - y[: a.height, : a.width]) ** 2))
            row = {"qp": qp, "split": split, "bytes": len(au), "psnr_y": round(10 * np.log10(65025 / mse), 3)}
            rows.append(row)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
