"""Ad-hoc: where does the GPU VP8 key frame first differ from the CPU oracle?"""
import numpy as np
import torch

import mxdesk
from tests.gpu_util import pitched
from tests.test_cpu_encoder import synthetic_nv12

N = mxdesk.native()
N.set_device(0)
w, h = 96, 64
cfg = N.EncoderConfig()
cfg.width, cfg.height, cfg.qp, cfg.bitrate_kbps, cfg.search_range = w, h, 28, 0, 8
g = N.GpuVp8Encoder(cfg, torch.cuda.current_stream().cuda_stream)
c = N.CpuVp8Encoder(cfg)
y, uv = synthetic_nv12(w, h, 0, seed=0)
dy, duv = pitched(y, g.pitch, g.coded_height), pitched(uv, g.pitch, g.coded_height // 2, uv=True)
torch.cuda.synchronize()
ga = g.encode(dy.data_ptr(), duv.data_ptr(), False)
ca = c.encode(y, uv, False)
print("bytes", len(ga), len(ca))
print("gpu modes\n", g.mb_info()[:, :2].reshape(4, 6, 2).transpose(2, 0, 1))
print("cpu modes\n", c.mb_info()[:, :2].reshape(4, 6, 2).transpose(2, 0, 1))
gy, guv = g.recon()
cy, cuv = c.recon()
for name, a, b in (("Y", gy, cy), ("UV", guv, cuv)):
    d = np.argwhere(a != b)
    print(name, "diffs", len(d), "first", d[:8].tolist())
    if len(d):
        r, col = d[0]
        print(" gpu row", a[r, max(0, col - 4): col + 8].tolist())
        print(" cpu row", b[r, max(0, col - 4): col + 8].tolist())
