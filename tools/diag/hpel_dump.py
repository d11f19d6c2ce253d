"""Dump GPU k_hpel planes and the numpy reference for one random picture (debug aid)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from mxdesk import native  # noqa: E402
from tests.test_gpu_pipeline import _hpel_reference  # noqa: E402

N = native()
N.set_device(0)
w, h = 160, 96
rng = np.random.default_rng(w + h)
ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
buf = np.zeros((h, 256), np.uint8)
buf[:, :w] = ref
got = [np.asarray(p) for p in N.h264.hpel_planes(buf, w)]
want = _hpel_reference(ref)
out = ROOT / "gpurun_out" / "dbg"
out.mkdir(parents=True, exist_ok=True)
np.savez(out / "hpel.npz", ref=ref, **{f"got{n}": g for n, g in zip("FHVJ", got)}, **{f"want{n}": x for n, x in zip("FHVJ", want)})
print("saved")
