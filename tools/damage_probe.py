"""Damage-driven vs full-frame capture upload on one GPU (Session.submit_bgrx_damage vs the
registered zero-copy submit_bgrx_ptr): per-frame host time and host->device bytes at
1920x1080 for a static screen, a typing-sized change (one 32-row band) and a window drag
(a 400-row band).  Usage: python tools/damage_probe.py [--frames N] [--json OUT]"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    from mxdesk import native

    N = native()
    N.set_device(0)
    w, h = a.width, a.height
    pitch = w * 4
    rng = np.random.default_rng(1)
    base = rng.integers(0, 256, (h, pitch), dtype=np.uint8)
    cases = {"static": [], "typing_32rows": [(512, 544)], "drag_400rows": [(320, 720)]}
    out = {"width": w, "height": h, "frames": a.frames, "cases": {}}
    for mode in ("full_zero_copy", "damage"):
        for name, bands in cases.items():
            cfg = N.SessionConfig()
            cfg.width, cfg.height, cfg.fps = w, h, 60
            s = N.Session(cfg)
            buf = base.copy()
            s.register_host_buffer(buf.ctypes.data, buf.nbytes)
            times = []
            for i in range(a.frames + 10):
                for y0, y1 in bands:  # the changed rows differ every frame
                    buf[y0:y1, :64] = i & 0xFF
                t0 = time.perf_counter()
                if mode == "damage":
                    s.submit_bgrx_damage(buf.ctypes.data, pitch, buf.nbytes, bands if i else [(0, h)], False)
                else:
                    s.submit_bgrx_ptr(buf.ctypes.data, pitch, buf.nbytes, False)
                s.collect()
                if i >= 10:
                    times.append(time.perf_counter() - t0)
            t = np.array(times) * 1e3
            up = s.damage_bytes_uploaded if mode == "damage" else (a.frames + 10) * w * h * 4
            r = {"ms_per_frame_mean": round(float(t.mean()), 4), "ms_p50": round(float(np.median(t)), 4),
                 "fps": round(1e3 / float(t.mean()), 1), "host_to_device_MB_per_frame": round(up / (a.frames + 10) / 1e6, 3)}
            out["cases"][f"{mode}/{name}"] = r
            print(mode, name, r, flush=True)
            del s
    if a.json:
        Path(a.json).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
