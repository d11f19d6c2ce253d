"""GPU == CPU for 16x8 / 8x16 partitions (k_me_full's quadrant search, per-partition quarter-pel
refinement, k_inter_encode's per-partition motion compensation, k_cavlc's partition mvds), and
the decoder reproduces the GPU reconstruction."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from mxdesk.codec.h264_decoder import Decoder  # noqa: E402

from .gpu_util import pitched  # noqa: E402
from .test_partitions import _split_motion  # noqa: E402


@pytest.mark.parametrize("vertical,coarse,subpel", [(True, 0, 1), (False, 0, 1), (True, 1, 1), (False, 1, 0)])
def test_gpu_partitions_bit_exact(gpu, vertical, coarse, subpel):
    w, h = 128, 64
    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height = w, h
    cfg.bitrate_kbps, cfg.qp, cfg.search_range = 0, 28, 8
    cfg.me_coarse, cfg.subpel = coarse, subpel
    genc = gpu.GpuH264Encoder(cfg, torch.cuda.current_stream().cuda_stream)
    cenc = gpu.CpuH264Encoder(cfg)
    stream, grec, nparts = b"", [], 0
    for t in range(5):
        y, uv = _split_motion(w, h, t, vertical)
        dy, duv = pitched(y, genc.pitch, genc.coded_height), pitched(uv, genc.pitch, genc.coded_height // 2, uv=True)
        torch.cuda.synchronize()
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
        cau = cenc.encode(y, uv, False)
        assert bool(gau == cau), f"frame {t}: GPU {len(gau)} B vs CPU {len(cau)} B"
        stream += gau
        grec.append(genc.recon())
        nparts += int((cenc.mb_info()[..., 8] > 0).sum())
    assert nparts > 8
    dec = Decoder()
    dec.decode(stream)
    for (yy, u, v), (ry, ruv) in zip(dec.frames_coded, grec):
        assert np.array_equal(yy, ry[:h, :w]) and np.array_equal(u, ruv[:h // 2, 0:w:2])
