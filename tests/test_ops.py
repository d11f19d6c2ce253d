"""mxdesk.ops: host-side validation (CPU) and HIP kernels vs numpy references (GPU)."""
import numpy as np
import pytest
import torch

from mxdesk import ops
from mxdesk.models.synthetic import bgrx_to_nv12 as np_bgrx_to_nv12
from mxdesk.models.synthetic import read_barcode


def test_ops_reject_host_tensors_before_launch():
    x = torch.zeros(16, 16, 4, dtype=torch.uint8)
    with pytest.raises(ValueError, match="GPU tensor"):
        ops.bgrx_to_nv12(x)
    with pytest.raises(ValueError, match="GPU tensor"):
        ops.synth_desktop(x)
    with pytest.raises(ValueError, match="GPU tensor"):
        ops.composite(x, x, 0, 0)


@pytest.mark.gpu
def test_ops_csc_matches_numpy(gpu):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (64, 96, 4), dtype=np.uint8)
    y, uv = ops.bgrx_to_nv12(torch.from_numpy(img).cuda())
    torch.cuda.synchronize()
    ry, ruv = np_bgrx_to_nv12(img)
    assert np.abs(y[:64, :96].cpu().numpy().astype(int) - ry).max() <= 1
    assert np.abs(uv[:32, :96].cpu().numpy().astype(int) - ruv.reshape(32, 96)).max() <= 1


@pytest.mark.gpu
def test_ops_synth_composite_scale(gpu):
    a = torch.empty(192, 320, 4, dtype=torch.uint8, device="cuda")
    ops.synth_desktop(a, frame_id=4242, timestamp_us=777, t=0.5)
    wall = torch.zeros(192, 640, 4, dtype=torch.uint8, device="cuda")
    ops.composite(a, wall, 320, 0)
    torch.cuda.synchronize()
    assert torch.equal(wall[:, 320:], a) and int(wall[:, :320].sum()) == 0
    y, _ = ops.bgrx_to_nv12(a)
    torch.cuda.synchronize()
    assert read_barcode(y[:192, :320].cpu().numpy())[0] == 4242
    ys, uvs = ops.scale_to_nv12(a, 160, 96)
    torch.cuda.synchronize()
    assert ys.shape[0] == 96 and uvs.shape[0] == 48
    with pytest.raises(ValueError):
        ops.composite(a, wall, 400, 0)
