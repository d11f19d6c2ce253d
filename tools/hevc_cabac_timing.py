"""Per-slice CABAC timing of the HIP HEVC encoder (GPU): every k_hevc_cabac wave records its
start / end wall clock (100 MHz), GpuHevcEncoder.slice_timing() returns (first CTU, CTUs,
bytes, ticks, start tick, tokens) per substream (slice, or WPP CTU row) of the last picture.
Fits ticks ~ a * CTUs + b * tokens over all substreams, to tell the per-CU fixed cost from the
per-token cost, and reports the slowest substream and (WPP) the latest start -- the wavefront
fill.

    python tools/hevc_cabac_timing.py --width 3840 --height 2160 --bitrate-kbps 25000 --frames 24
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
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--report", type=int, default=4)
    ap.add_argument("--wpp", type=int, default=1)
    ap.add_argument("--wpp-rows", type=int, default=8)
    ap.add_argument("--slice-cost", type=int, default=0, help="P-slice work target (0: encoder default)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import torch

    import mxdesk
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12
    from tests.gpu_util import pitched

    N = mxdesk.native()
    N.set_device(0)
    cfg = N.EncoderConfig()
    cfg.width, cfg.height, cfg.fps = a.width, a.height, 60
    cfg.bitrate_kbps = a.bitrate_kbps
    cfg.hevc_wpp, cfg.hevc_wpp_rows = a.wpp, a.wpp_rows
    if a.slice_cost:
        cfg.hevc_slice_cost = a.slice_cost
    enc = N.GpuHevcEncoder(cfg, torch.cuda.current_stream().cuda_stream)
    desk = CpuSyntheticDesktop(a.width, a.height, True)
    rows, allx, ally = [], [], []
    for f in range(a.frames):
        y, uv = bgrx_to_nv12(desk.render(f, f / 60, 0))
        dy = pitched(y, enc.pitch, enc.coded_height)
        duv = pitched(uv, enc.pitch, enc.coded_height // 2, uv=True)
        torch.cuda.synchronize()
        au = enc.encode(dy.data_ptr(), duv.data_ptr(), False)
        if f < a.frames - a.report or enc.stats.idr:
            continue
        t = np.array(enc.slice_timing(), dtype=np.float64)  # first, ctus, bytes, ticks, start, tokens
        us = t[:, 3] / 100.0
        end_us = (t[:, 3] + t[:, 4]) / 100.0
        k = int(np.argmax(us))
        allx.append(t[:, [1, 5]])
        ally.append(us)
        rows.append({"frame": f, "au_bytes": len(au), "substreams": int(len(t)), "tokens": int(t[:, 5].sum()),
                     "span_us": round(float(end_us.max()), 1), "max_us": round(float(us[k]), 1),
                     "median_us": round(float(np.median(us)), 1), "latest_start_us": round(float(t[:, 4].max() / 100), 1),
                     "slowest_ctus": int(t[k, 1]), "slowest_tokens": int(t[k, 5]), "slowest_bytes": int(t[k, 2]),
                     "max_tokens": int(t[:, 5].max()), "ns_per_token_slowest": round(1e3 * float(us[k] / max(t[k, 5], 1)), 1)})
        print(json.dumps(rows[-1]), flush=True)
    X = np.concatenate(allx)
    Y = np.concatenate(ally)
    coef, *_ = np.linalg.lstsq(X, Y, rcond=None)
    fit = {"us_per_ctu": round(float(coef[0]), 4), "ns_per_token": round(1e3 * float(coef[1]), 2)}
    print(json.dumps({"fit": fit}), flush=True)
    if a.json_out:
        Path(a.json_out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.json_out).write_text(json.dumps({"width": a.width, "height": a.height, "kbps": a.bitrate_kbps,
                                                "pictures": rows, "fit": fit}) + "\n")


if __name__ == "__main__":
    main()
