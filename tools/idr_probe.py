"""Encode a few 1080p frames (first one IDR) -- used with instrumented kernels."""
import sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mxdesk import native
N = native()
N.set_device(0)
cfg = N.SessionConfig()
cfg.width, cfg.height, cfg.fps = 1920, 1080, 60
cfg.enc.bitrate_kbps = 8000
if len(sys.argv) > 1:
    cfg.enc.intra4x4 = int(sys.argv[1])
s = N.Session(cfg)
for i in range(3):
    r = s.step(i == 2)
    print("frame", i, len(r.au), flush=True)
