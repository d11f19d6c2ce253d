"""GPU HEVC IDR at a given size with / without the intra split (debug probe for one config).

    python tools/debug/hevc_split_probe.py W H SPLIT KBPS [QP]
"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import mxdesk  # noqa: E402
from tests.test_gpu_production_sizes import desktop_nv12, pitched, _stream  # noqa: E402

w, h, split, kbps = (int(v) for v in sys.argv[1:5])
qp = int(sys.argv[5]) if len(sys.argv) > 5 else 40
N = mxdesk.native()
N.set_device(0)
cfg = N.EncoderConfig()
cfg.width, cfg.height, cfg.fps = w, h, 60
cfg.bitrate_kbps, cfg.qp = kbps, qp
cfg.hevc_intra_split = split
genc = N.GpuHevcEncoder(cfg, _stream())
y, uv = desktop_nv12(N, w, h, 0)
ch = genc.coded_height
dy = pitched(y, genc.pitch, ch)
duv = pitched(uv, genc.pitch, ch // 2, uv=True)
torch.cuda.synchronize()
print("encode", w, h, split, kbps, flush=True)
t = time.time()
au = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
print("gpu", len(au), "qp", genc.stats.qp, round(time.time() - t, 2), flush=True)
cenc = N.CpuHevcEncoder(cfg)
cau = cenc.encode(y, uv, False)
print("cpu", len(cau), "qp", cenc.stats.qp, "equal", cau == au, flush=True)
y1, uv1 = desktop_nv12(N, w, h, 1)
dy1 = pitched(y1, genc.pitch, ch)
duv1 = pitched(uv1, genc.pitch, ch // 2, uv=True)
torch.cuda.synchronize()
t = time.time()
au1 = genc.encode(dy1.data_ptr(), duv1.data_ptr(), False)
print("gpu P", len(au1), "qp", genc.stats.qp, round(time.time() - t, 2), flush=True)
cau1 = cenc.encode(y1, uv1, False)
print("cpu P", len(cau1), "qp", cenc.stats.qp, "equal", cau1 == au1, flush=True)
for q in (39, 40, 41, 42):  # fixed-QP sizes of the same picture, GPU and CPU
    cfg.bitrate_kbps, cfg.qp = 0, q
    g2 = N.GpuHevcEncoder(cfg, _stream())
    a2 = g2.encode(dy.data_ptr(), duv.data_ptr(), False)
    c2 = N.CpuHevcEncoder(cfg).encode(y, uv, False)
    print("fixed", q, len(a2), len(c2), a2 == c2, flush=True)
