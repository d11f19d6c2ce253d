"""Per-slice size report of the HIP HEVC encoder on the bench desktop (GPU): how evenly the
cost-balanced P slices share the CABAC work.  One wave codes one slice, so the k_hevc_cabac
time of a picture is set by its largest slice; this prints, for the last P pictures, the
slice count, the bytes of the largest / median slice and the CTUs per slice.

    python tools/hevc_slice_report.py --width 3840 --height 2160 --bitrate-kbps 25000 --frames 40
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from mxdesk.codec import hevc_decoder as hd  # noqa: E402


def slices_of(au: bytes, ctbs: int):
    out = []
    nb = (ctbs - 1).bit_length()
    for nal in hd.split_nal_units(au):
        typ = (nal[0] >> 1) & 63
        if typ not in (1, 19, 20):
            continue
        r = hd.BitReader(hd.unescape(nal), 16)
        first = r.u(1)
        if typ >= 16:
            r.u(1)
        r.ue()
        addr = 0 if first else r.u(nb)
        out.append((addr, len(nal)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--bitrate-kbps", type=int, default=25000)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--report", type=int, default=5, help="P pictures reported (the last ones)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import mxdesk

    N = mxdesk.native()
    N.set_device(0)
    cfg = N.SessionConfig()
    cfg.width, cfg.height, cfg.fps = a.width, a.height, 60
    cfg.codec = "hevc"
    cfg.enc.bitrate_kbps = a.bitrate_kbps
    cfg.noise = 1
    s = N.Session(cfg)
    ctb_w, ctb_h = (a.width + 15) // 16, (a.height + 15) // 16
    ctbs = ctb_w * ctb_h
    rows = []
    for f in range(a.frames):
        r = s.step(False)
        if f >= a.frames - a.report and not r.idr:
            sl = slices_of(bytes(r.au), ctbs)
            sizes = [n for _, n in sl]
            addrs = [ad for ad, _ in sl] + [ctbs]
            ctus = [addrs[k + 1] - addrs[k] for k in range(len(sl))]
            big = max(range(len(sl)), key=lambda k: sizes[k])
            rows.append({"frame": f, "slices": len(sl), "au_bytes": len(r.au), "max_slice_bytes": max(sizes),
                         "median_slice_bytes": statistics.median(sizes), "ctus_of_largest": ctus[big],
                         "addr_of_largest": addrs[big], "min_ctus": min(ctus), "max_ctus": max(ctus),
                         "qp": r.qp})
            print(json.dumps(rows[-1]), flush=True)
    if a.json_out:
        Path(a.json_out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.json_out).write_text(json.dumps({"width": a.width, "height": a.height, "kbps": a.bitrate_kbps,
                                                "pictures": rows}) + "\n")


if __name__ == "__main__":
    main()
