"""Quick HEVC GPU timing: GpuHevcEncoder on a moving synthetic NV12 picture already in HBM.
Usage: python tools/hevc_quick.py W H frames"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from mxdesk import native  # noqa: E402

N = native()
W, H, F = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cfg = N.EncoderConfig()
cfg.width, cfg.height, cfg.fps = W, H, 60
cfg.bitrate_kbps = int(sys.argv[4]) if len(sys.argv) > 4 else 25000
enc = N.GpuHevcEncoder(cfg, torch.cuda.current_stream().cuda_stream)
ch = enc.coded_height
yy, xx = np.mgrid[0:ch, 0:enc.pitch]
base = ((np.sin(xx / 37.0) * 60 + np.cos(yy / 23.0) * 50 + 128)).astype(np.uint8)
y = torch.from_numpy(base).cuda()
uv = torch.full((ch // 2, enc.pitch), 128, dtype=torch.uint8, device="cuda")
times, sizes = [], []
for f in range(F):
    # scroll a band and repaint a noise box so P frames carry motion + texture
    y[:, :] = torch.roll(torch.from_numpy(base).cuda(), shifts=2 * f, dims=1)
    y[H // 3: H // 3 + 64, W // 4: W // 4 + 256] = torch.randint(0, 255, (64, 256), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    au = enc.encode(y.data_ptr(), uv.data_ptr(), False)
    times.append((time.perf_counter() - t) * 1e3)
    sizes.append(len(au))
st = enc.stats
p = np.array(times[2:])
print(f"hevc {W}x{H}: first(I) {times[0]:.2f} ms, P median {np.median(p):.3f} ms p95 {np.percentile(p, 95):.3f} ms "
      f"-> {1000 / np.median(p):.0f} fps; bytes I {sizes[0]} P~{int(np.median(sizes[2:]))}; qp {st.qp} "
      f"gpu encode_ms {st.encode_ms:.3f}")
