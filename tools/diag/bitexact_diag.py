"""Localise a GPU-vs-CPU encoder mismatch: per frame, compare reconstructions (analysis
kernels) and bitstreams (entropy kernels)."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else str(ROOT))  # package location (variant builds)
sys.path.insert(0, str(ROOT / "tests"))
from gpu_util import pitched  # noqa: E402
from test_cpu_encoder import synthetic_nv12  # noqa: E402

import mxdesk  # noqa: E402

print("mxdesk from", mxdesk.__file__, flush=True)
N = mxdesk.native()
N.set_device(0)
for (w, h, subpel, sr) in [(64, 48, 1, 8), (160, 96, 0, 16), (100, 60, 1, 16)]:
    cfg = N.EncoderConfig()
    cfg.width, cfg.height, cfg.bitrate_kbps, cfg.qp, cfg.search_range, cfg.subpel = w, h, 0, 28, sr, subpel
    st = torch.cuda.current_stream().cuda_stream
    g, c = N.GpuH264Encoder(cfg, st), N.CpuH264Encoder(cfg)
    ch = g.coded_height
    for t in range(5):
        y, uv = synthetic_nv12(w, h, t)
        dy, duv = pitched(y, g.pitch, ch), pitched(uv, g.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        ga, ca = g.encode(dy.data_ptr(), duv.data_ptr(), False), c.encode(y, uv, False)
        gy, guv = g.recon()
        cy, cuv = c.recon()
        ry = np.array_equal(gy[:ch, :cy.shape[1]], cy[:ch]) if gy.shape[1] >= cy.shape[1] else None
        print(f"{w}x{h} sp{subpel} sr{sr} frame {t}: recon_y_equal={ry} au_equal={ga == ca} "
              f"len {len(ga)} vs {len(ca)}", flush=True)
        if ga != ca:
            d = next(i for i, (a, b) in enumerate(zip(ga, ca)) if a != b) if len(ga) and len(ca) else -1
            print("   first differing byte", d, flush=True)
