"""Per-slice CABAC timing of an HEVC Session on the GPU-rendered bench desktop (the bench's own
content path, unlike hevc_cabac_timing.py's CPU-rendered frames): for the last --report P pictures,
the substream count, token total, the slowest substream and the median, as JSON lines.

    python tools/hevc_session_timing.py --width 3840 --height 2160 --bitrate-kbps 25000
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--bitrate-kbps", type=int, default=25000)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--report", type=int, default=4)
    ap.add_argument("--slice-cost", type=int, default=0)
    ap.add_argument("--dump", default="", help="save per-CU (type, cbf, sum last+1, sub-blocks, est_bytes, tokens) as <dump>_<frame>.npy")
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime initialised the same way as the bench)

    import mxdesk

    N = mxdesk.native()
    N.set_device(0)
    cfg = N.SessionConfig()
    cfg.width, cfg.height, cfg.fps = a.width, a.height, 60
    cfg.codec = "hevc"
    cfg.enc.bitrate_kbps = a.bitrate_kbps
    cfg.enc.pipeline_depth = 1
    if a.slice_cost:
        cfg.enc.hevc_slice_cost = a.slice_cost
    s = N.Session(cfg)
    for f in range(a.frames):
        r = s.step(False)
        if f < a.frames - a.report or s.stats.idr:
            continue
        t = np.array(s.slice_timing(), dtype=np.float64)  # first, ctus, bytes, ticks, start, tokens
        us = t[:, 3] / 100.0
        k = int(np.argmax(us))
        order = np.argsort(-us)[:5]
        if a.dump:
            np.save(f"{a.dump}_{f}.npy", np.array(s.cu_token_table(), dtype=np.uint32))
        print(json.dumps({"frame": f, "au_bytes": len(r.au), "substreams": int(len(t)), "tokens": int(t[:, 5].sum()),
                          "max_us": round(float(us[k]), 1), "median_us": round(float(np.median(us)), 1),
                          "top5": [[int(t[j, 0]), int(t[j, 1]), int(t[j, 2]), int(t[j, 5]), round(float(us[j]), 1)]
                                   for j in order]}), flush=True)


if __name__ == "__main__":
    main()
