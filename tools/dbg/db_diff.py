"""Debug: GPU vs CPU reconstruction after in-loop deblocking, per-position diff histogram."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import torch

import mxdesk
from tests.gpu_util import pitched
from tests.test_cpu_encoder import synthetic_nv12

N = mxdesk.native()
N.set_device(0)
for (w, h, qp) in [(64, 48, 24), (320, 192, 30)]:
    cfg = N.EncoderConfig()
    cfg.width, cfg.height = w, h
    cfg.bitrate_kbps, cfg.qp, cfg.deblock, cfg.search_range = 0, qp, 1, 8
    g = N.GpuH264Encoder(cfg, torch.cuda.current_stream().cuda_stream)
    c = N.CpuH264Encoder(cfg)
    for t in range(2):
        y, uv = synthetic_nv12(w, h, t, seed=0)
        dy = pitched(y, g.pitch, g.coded_height)
        duv = pitched(uv, g.pitch, g.coded_height // 2, uv=True)
        torch.cuda.synchronize()
        ga = g.encode(dy.data_ptr(), duv.data_ptr(), False)
        ca = c.encode(y, uv, False)
        gy, guv = g.recon()
        cy, cuv = c.recon()
        gy, cy = gy[:h, :w].astype(int), cy[:h, :w].astype(int)
        d = gy != cy
        print(f"{w}x{h} frame {t}: stream equal {ga == ca}; luma diffs {d.sum()} chroma diffs {(guv[:h//2,:w] != cuv[:h//2,:w]).sum()}")
        if d.any():
            ys, xs = np.nonzero(d)
            print("  x%16 hist", np.bincount(xs % 16, minlength=16))
            print("  y%16 hist", np.bincount(ys % 16, minlength=16))
            print("  first", list(zip(ys[:12], xs[:12])), "gpu", gy[ys[:12], xs[:12]], "cpu", cy[ys[:12], xs[:12]])
        if not (ga == ca):
            break
