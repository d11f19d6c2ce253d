"""HEVC P-picture chroma vs luma quality on dumped bench frames (tools/dump_frames.py --content
motion), CPU encoder (the GPU's bit-exact oracle), rate control at a given bitrate: mean Y / U / V
PSNR and bytes over the sequence, for EncoderConfig variants given as key=value lists.

    python tools/hevc_chroma_rd.py --npz frames_mot.npz --kbps 4500 [--set hevc_chroma_keep=1 ...]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npz", required=True)
    ap.add_argument("--kbps", type=int, default=4500)
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--set", action="append", default=[], help="variant: k=v[,k=v...] (repeatable)")
    a = ap.parse_args()
    import mxdesk

    N = mxdesk.native()
    z = np.load(a.npz)
    w, h = int(z["width"]), int(z["height"])
    ys, uvs = z["y"], z["uv"]
    n = a.frames or len(ys)
    for var in ([""] + a.set):
        cfg = N.EncoderConfig()
        cfg.width, cfg.height, cfg.fps = w, h, 60
        cfg.bitrate_kbps = a.kbps
        for kv in filter(None, var.split(",")):
            k, v = kv.split("=")
            setattr(cfg, k, int(v))
        enc = N.CpuHevcEncoder(cfg)
        tot, ps = 0, [[], [], []]
        for i in range(n):
            y, uv = np.ascontiguousarray(ys[i]), np.ascontiguousarray(uvs[i])
            tot += len(enc.encode(y, uv, False))
            ry, ruv = enc.recon()
            planes = [(ry[:h, :w], y[:h, :w]), (ruv[:h // 2, 0:w:2], uv[:h // 2, 0:w:2]),
                      (ruv[:h // 2, 1:w:2], uv[:h // 2, 1:w:2])]
            for c, (r, s) in enumerate(planes):
                mse = float(np.mean((r.astype(np.float64) - s) ** 2))
                ps[c].append(99.0 if mse == 0 else 10 * np.log10(65025 / mse))
        skip = 1  # the IDR picture out of the means
        print(json.dumps({"variant": var or "default", "bytes": tot, "y": round(float(np.mean(ps[0][skip:])), 3),
                          "u": round(float(np.mean(ps[1][skip:])), 3), "v": round(float(np.mean(ps[2][skip:])), 3)}),
              flush=True)


if __name__ == "__main__":
    main()
