"""HEVC IDR picture: bytes and luma PSNR with and without the intra transform-tree split
(EncoderConfig.hevc_intra_split), CPU encoder (the GPU's bit-exact oracle), fixed QPs, on the
numpy synthetic desktop or a frame of the GPU-rendered bench desktop (tools/dump_frames.py --npz).

    python tools/hevc_intra_split_rd.py [--width 1920 --height 1080 --qps 27,32,37,41] [--npz frames.npz]
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
    ap.add_argument("--npz", default="")
    ap.add_argument("--splits", default="0,1")
    a = ap.parse_args()
    import mxdesk
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    N = mxdesk.native()
    if a.npz:
        z = np.load(a.npz)
        a.width, a.height = int(z["width"]), int(z["height"])
        y, uv = np.ascontiguousarray(z["y"][0]), np.ascontiguousarray(z["uv"][0])
    else:
        desk = CpuSyntheticDesktop(a.width, a.height, noise=True)
        y, uv = bgrx_to_nv12(desk.render(0, 0.0, 0))
    mask = np.ones((a.height, a.width), bool)  # the incompressible noise panel left out (--npz)
    if a.npz and "mask" in z:
        x0, y0, x1, y1 = (int(v) for v in z["mask"])
        mask[y0:y1, x0:x1] = False
    rows = []
    for qp in [int(q) for q in a.qps.split(",")]:
        for split in [int(v) for v in a.splits.split(",")]:
            cfg = N.EncoderConfig()
            cfg.width, cfg.height, cfg.fps = a.width, a.height, 60
            cfg.bitrate_kbps, cfg.qp = 0, qp
            cfg.hevc_intra_split = split
            enc = N.CpuHevcEncoder(cfg)
            au = enc.encode(y, uv, True)
            ry = enc.recon()[0][: a.height, : a.width].astype(np.float64)
            e2 = (ry - y[: a.height, : a.width]) ** 2
            mse, msem = float(np.mean(e2)), float(np.mean(e2[mask]))
            cu = np.asarray(enc.cu_info()) if hasattr(enc, "cu_info") else None
            row = {"qp": qp, "split": split, "bytes": len(au), "psnr_y": round(10 * np.log10(65025 / mse), 3),
                   "psnr_y_masked": round(10 * np.log10(65025 / msem), 3),
                   "split_units": int((cu[:, 3] == 2).sum()) if cu is not None else None}
            rows.append(row)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
