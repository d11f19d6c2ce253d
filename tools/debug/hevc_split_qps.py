"""GPU vs CPU HEVC IDR bytes over fixed QPs, and a second forced IDR on the same encoders (stale
reconstruction in the buffers), for one picture size (debug probe).

    python tools/debug/hevc_split_qps.py W H QP[,QP...]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import mxdesk  # noqa: E402
from tests.test_gpu_production_sizes import desktop_nv12, pitched, _stream  # noqa: E402

w, h = int(sys.argv[1]), int(sys.argv[2])
N = mxdesk.native()
N.set_device(0)
y, uv = desktop_nv12(N, w, h, 0)
y1, uv1 = desktop_nv12(N, w, h, 1)
for q in [int(v) for v in sys.argv[3].split(",")]:
    cfg = N.EncoderConfig()
    cfg.width, cfg.height, cfg.fps = w, h, 60
    cfg.bitrate_kbps, cfg.qp = 0, q
    if len(sys.argv) > 4:
        cfg.sao = int(sys.argv[4])
    g = N.GpuHevcEncoder(cfg, _stream())
    c = N.CpuHevcEncoder(cfg)
    ch = g.coded_height
    out = []
    for (yy, uu, idr) in ((y1, uv1, True), (y, uv, True)):
        dy, du = pitched(yy, g.pitch, ch), pitched(uu, g.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        a = g.encode(dy.data_ptr(), du.data_ptr(), idr)
        b = c.encode(yy, uu, idr)
        out.append((len(a), len(b), a == b))
    print("qp", q, out, flush=True)
