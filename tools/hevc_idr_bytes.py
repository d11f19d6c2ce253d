"""Size and luma PSNR of a 4K HEVC session's first (IDR) access unit on the GPU -- the I-slice
layout's bit cost (profiles/r05_hevc_islices/NOTES.md).

    python tools/hevc_idr_bytes.py [--width 3840 --height 2160 --bitrate-kbps 18000]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--bitrate-kbps", type=int, default=18000)
    a = ap.parse_args()
    import torch  # noqa: F401

    import mxdesk

    N = mxdesk.native()
    N.set_device(0)
    cfg = N.SessionConfig()
    cfg.width, cfg.height, cfg.fps, cfg.codec = a.width, a.height, 60, "hevc"
    cfg.enc.bitrate_kbps = a.bitrate_kbps
    cfg.enc.pipeline_depth = 1
    s = N.Session(cfg)
    r = s.step(False)
    print(json.dumps({"idr": bool(r.idr), "au_bytes": len(r.au), "qp": r.qp, "psnr_y": round(r.psnr_y, 3)}))


if __name__ == "__main__":
    main()
