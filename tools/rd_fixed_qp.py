import sys, numpy as np
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))
from mxdesk import native
from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12
N = native()
W, H = 960, 544
def psnr(a, b):
    d = a.astype(np.float64) - b; return 10 * np.log10(255 ** 2 / max((d * d).mean(), 1e-9))
def run(kind, qp, frames=6):
    ec = N.EncoderConfig(); ec.width, ec.height, ec.fps = W, H, 60; ec.bitrate_kbps = 0; ec.qp = qp
    ec.search_range = 8; ec.subpel = 1
    enc = N.CpuHevcEncoder(ec) if kind == "hevc" else N.CpuH264Encoder(ec)
    desk = CpuSyntheticDesktop(W, H, False)
    out = []
    for f in range(frames):
        y, uv = bgrx_to_nv12(desk.render(f, f / 60, 0))
        au = enc.encode(y, uv, False)
        ry, ruv = enc.recon()
        out.append((len(au), round(psnr(ry[:H, :W], y[:H, :W]), 2), round(psnr(ruv[:H//2, :W], uv[:H//2, :W]), 2)))
    return out
for qp in (22, 28, 34):
    for k in ("h264", "hevc"):
        print(k, qp, run(k, qp))
