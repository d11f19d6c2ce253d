#!/usr/bin/env python3
"""Per-region bit / distortion breakdown of the bench desktop, encoded by the CPU oracle encoder
(bit-exact with the GPU encoder) on frames dumped from the GPU by tools/dump_frames.py.

    python tools/region_report.py /tmp/frames_1080p.npz --frames 25 [--set aq=2 ...]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

W, H = 1920, 1080


def regions(mb_w, mb_h):
    """MB class map from the renderer's layout (csrc/kernels/pixel.hip dyn_boxes / static_px)."""
    cls = np.full((mb_h, mb_w), 0, np.int32)  # 0 wallpaper
    names = ["wallpaper", "taskbar", "document", "noise", "terminal", "gears", "barcode"]
    boxes = {
        1: (0, H - 32, W, H),
        2: (int(W * .25), int(H * .52), int(W * .25) + int(W * .24), int(H * .52) + int(H * .36)),
        4: (int(W * .04), int(H * .10), int(W * .04) + int(W * .42), int(H * .10) + int(H * .38)),
        5: (int(W * .55), int(H * .10), int(W * .55) + int(W * .38), int(H * .10) + int(H * .50)),
        3: (int(W * .04), int(H * .55), int(W * .04) + int(W * .16), int(H * .55) + int(H * .22)),
        6: (0, 0, 8 + 33 * 8, 32),
    }
    for k in (1, 2, 4, 5, 3, 6):
        x0, y0, x1, y1 = boxes[k]
        for my in range(mb_h):
            for mx in range(mb_w):
                cx, cy = mx * 16 + 8, my * 16 + 8
                if x0 <= cx < x1 and y0 <= cy < y1:
                    cls[my, mx] = k
    return cls, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--frames", type=int, default=25)
    ap.add_argument("--kbps", type=int, default=8000)
    ap.add_argument("--window", default="5:25", help="frames averaged (the driver's 20-step window after 5 warmup)")
    ap.add_argument("--set", nargs="*", default=[], help="EncoderConfig overrides name=value")
    ap.add_argument("--per-frame", action="store_true")
    a = ap.parse_args()
    import mxdesk

    N = mxdesk.native()
    d = np.load(a.npz)
    Y, UV = d["y"], d["uv"]
    mask = d["mask"]
    c = N.EncoderConfig()
    c.width, c.height, c.fps = W, H, 60
    c.bitrate_kbps = a.kbps
    c.mask_x0, c.mask_y0, c.mask_x1, c.mask_y1 = (int(v) for v in mask)
    for kv in a.set:
        k, v = kv.split("=")
        setattr(c, k, int(v))
    e = N.CpuH264Encoder(c)
    mb_w, mb_h = (W + 15) // 16, (H + 15) // 16
    cls, names = regions(mb_w, mb_h)
    mmx0, mmy0 = int(mask[0]) // 16, int(mask[1]) // 16
    mmx1, mmy1 = (int(mask[2]) + 15) // 16, (int(mask[3]) + 15) // 16
    lo, hi = (int(v) for v in a.window.split(":"))
    acc_bits = np.zeros(len(names))
    acc_sse = np.zeros(len(names))
    acc_n = np.zeros(len(names))
    tot = {"bytes": [], "psnr": [], "psnr_m": [], "qp": []}
    for f in range(a.frames):
        au = e.encode(Y[f], UV[f])
        ry, _ = e.recon()
        err = (ry[:H, :W].astype(np.int64) - Y[f][:H, :W].astype(np.int64)) ** 2
        errp = np.zeros((mb_h * 16, mb_w * 16), np.int64)
        errp[:H, :W] = err
        mb_sse = errp.reshape(mb_h, 16, mb_w, 16).sum(axis=(1, 3))
        bits = e.mb_bits()
        m = np.ones((mb_h, mb_w), bool)
        m[mmy0:mmy1, mmx0:mmx1] = False
        npx_m = m.sum() * 256 - (mb_h * 16 - H) * 16 * m[-1].sum()
        psnr = 10 * np.log10(65025 * W * H / max(1, err.sum()))
        psnr_m = 10 * np.log10(65025 * npx_m / max(1, mb_sse[m].sum()))
        if a.per_frame:
            print(f"f{f:02d} {'I' if e.stats.idr else 'P'} qp {e.stats.qp} {len(au)} B psnr {psnr:.2f} masked {psnr_m:.2f}")
        if lo <= f < hi:
            tot["bytes"].append(len(au))
            tot["psnr"].append(psnr)
            tot["psnr_m"].append(psnr_m)
            tot["qp"].append(e.stats.qp)
            for k in range(len(names)):
                sel = cls == k
                acc_bits[k] += bits[sel].sum()
                acc_sse[k] += mb_sse[sel].sum()
                acc_n[k] += sel.sum()
    n = hi - lo
    print(f"window {a.window}: {np.mean(tot['bytes']) * 8 * 60 / 1000:.0f} kbps  qp {np.mean(tot['qp']):.2f}  "
          f"psnr {np.mean(tot['psnr']):.2f}  masked {np.mean(tot['psnr_m']):.2f}")
    for k, nm in enumerate(names):
        if acc_n[k] == 0:
            continue
        mse = acc_sse[k] / (acc_n[k] * 256)
        print(f"  {nm:10s} MBs {acc_n[k] / n:6.0f}  kbit/frame {acc_bits[k] / n / 1000:7.1f}  "
              f"psnr {10 * np.log10(65025 / max(mse, 1e-9)):6.2f}")


if __name__ == "__main__":
    main()
