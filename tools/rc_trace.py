"""Rate-control trace on the GPU: per-frame bits / QP of a CBR session (with forced IDRs), and
the content's rate-QP curves (fixed-QP runs), for tuning h264::EncoderCommon offline.

python tools/rc_trace.py [--codec h264] [--width 1920 --height 1080] [--kbps 8000] [--frames 120]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def session(N, a, kbps, qp, depth):
    cfg = N.SessionConfig()
    cfg.width, cfg.height, cfg.fps = a.width, a.height, 60
    cfg.enc.bitrate_kbps = kbps
    cfg.enc.qp = qp
    cfg.enc.pipeline_depth = depth
    cfg.codec = a.codec
    cfg.fake_clock = 1
    return N.Session(cfg)


def run(s, n, idr_at=()):
    out = []
    s.submit(False)
    for i in range(n):
        if s.depth > 1 and i + 1 < n:
            s.submit(i + 1 in idr_at)
        r = s.collect()
        if s.depth == 1 and i + 1 < n:
            s.submit(i + 1 in idr_at)
        out.append((len(r.au) * 8, r.qp, r.idr))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="h264")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--kbps", type=int, default=8000)
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--qps", default="24,28,32,36,40")
    a = ap.parse_args()
    import mxdesk

    N = mxdesk.native()
    N.set_device(0)
    res = {"T": a.kbps * 1000 / 60}
    for depth in (1, 2):
        res[f"cbr_d{depth}"] = run(session(N, a, a.kbps, 28, depth), a.frames, idr_at=(30, 90))
    for q in map(int, a.qps.replace("/", ",").split(",")):
        res[f"q{q}"] = [b for b, _, _ in run(session(N, a, 0, q, 1), min(a.frames, 60))]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
