"""Lanczos scaler forms at one size, for kernel profiling (rocprofv3 --kernel-trace --stats):
VALU, MFMA tile and MFMA strip kernels, `--reps` launches each on a synthetic desktop.

    python tools/scale_probe.py --src 3840x2160 --dst 1920x1080 --reps 50 --forms tile,strip
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mxdesk import _native as gpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="3840x2160")
    ap.add_argument("--dst", default="1920x1080")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--forms", default="valu,tile,strip", help="comma- or plus-separated")
    a = ap.parse_args()
    w, h = map(int, a.src.split("x"))
    ow, oh = map(int, a.dst.split("x"))
    cw, ch = (ow + 15) // 16 * 16, (oh + 15) // 16 * 16
    src = torch.zeros((h, w * 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    gpu.synth(src.data_ptr(), w, h, w * 4, frame_id=7, t=0.25, noise=1, stream=stream)
    xs, wx, tx = gpu.lanczos_table(w, ow)
    ys, wy, ty = gpu.lanczos_table(h, oh)
    dev = [torch.from_numpy(v).cuda() for v in (xs, wx, ys, wy)]
    y = torch.zeros((ch, cw), dtype=torch.uint8, device="cuda")
    uv = torch.zeros((ch // 2, cw), dtype=torch.uint8, device="cuda")
    for form in a.forms.replace("+", ",").split(","):
        for _ in range(a.reps):
            gpu.scale_to_nv12(src.data_ptr(), w * 4, w, h, ow, oh, dev[0].data_ptr(), dev[1].data_ptr(), tx,
                              dev[2].data_ptr(), dev[3].data_ptr(), ty, y.data_ptr(), uv.data_ptr(), cw, cw, ch, stream,
                              mfma=form != "valu", strip=form == "strip")
        torch.cuda.synchronize()
        print(form, "done", flush=True)


if __name__ == "__main__":
    main()
