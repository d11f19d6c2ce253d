#!/usr/bin/env python3
"""Summarise bench.py JSON files: one row per file (fps, p50, kbps, QP, masked PSNR, density)."""
import json
import sys


def row(path):
    d = json.load(open(path))
    q = d.get("quality_probe") or {}
    return (f"{path.split('/')[-1]:28s} {d['value']:9.1f} fps  p50 {d['p50_e2e_latency_ms']:6.3f}  "
            f"{d['mean_bitrate_kbps_at_60fps']:8.0f} kbps  qp {d['mean_qp']:5.2f}  "
            f"Ym {d['mean_psnr_y_db_noise_masked']:5.2f}  Um {d.get('mean_psnr_u_db_noise_masked')}  "
            f"db {d.get('deblocked_frames_pct')}%  dens {d.get('sessions_per_gpu_at_60fps_measured')}"
            f"/{d.get('sessions_per_gpu_idr_storm_measured')}  qY {q.get('psnr_y_db')}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        try:
            print(row(p))
        except Exception as e:  # noqa: BLE001
            print(p, "ERR", e)
