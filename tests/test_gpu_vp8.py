"""HIP VP8 encoder (WEBRTC_ENCODER=vp8enc, reference README.md:21,35).

The GPU encoder's frames are byte-for-byte the CPU oracle's (tests/test_vp8.py pins the oracle to
libwebp for key frames and to the in-tree RFC 6386 decoder for inter frames), reconstructions
included; GPU key frames also go through libwebp (Pillow) directly, at 1080p too."""
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from mxdesk.codec.vp8_decoder import Decoder, webp_container  # noqa: E402

from .gpu_util import pitched  # noqa: E402
from .test_cpu_encoder import synthetic_nv12  # noqa: E402
from .test_gpu_production_sizes import _stream, desktop_nv12  # noqa: E402
from .test_vp8 import _picture, libwebp_rgb  # noqa: E402


def _pair(gpu, w, h, kbps=0, qp=30, sr=8, depth=1, deblock=-1):
    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height, cfg.fps = w, h, 60
    cfg.bitrate_kbps, cfg.qp, cfg.search_range = kbps, qp, sr
    cfg.pipeline_depth, cfg.deblock = depth, deblock
    return gpu.GpuVp8Encoder(cfg, _stream()), gpu.CpuVp8Encoder(cfg)


def _dev(genc, y, uv):
    ch = genc.coded_height
    dy, duv = pitched(y, genc.pitch, ch), pitched(uv, genc.pitch, ch // 2, uv=True)
    torch.cuda.synchronize()
    return dy, duv


def _check(genc, cenc, gau, cau, w, h, t):
    gm, cm = genc.mb_info(), cenc.mb_info()
    bad = np.nonzero((gm != cm).any(axis=1))[0]
    assert bad.size == 0, f"{w}x{h} frame {t}: MB {bad[:5]} GPU {gm[bad[:3]]} CPU {cm[bad[:3]]}"
    gy, guv = genc.recon()
    cy, cuv = cenc.recon()
    assert np.array_equal(gy, cy), f"{w}x{h} frame {t}: luma reconstruction"
    assert np.array_equal(guv, cuv), f"{w}x{h} frame {t}: chroma reconstruction"
    assert gau == cau, f"{w}x{h} frame {t}: GPU {len(gau)} B vs CPU {len(cau)} B"


@pytest.mark.parametrize("w,h,kbps,qp", [(96, 64, 0, 28), (100, 60, 300, 30), (320, 192, 600, 24), (176, 144, 0, 44)])
def test_gpu_vp8_bit_exact_vs_cpu(gpu, w, h, kbps, qp):
    """Key + P frames of a moving scene (vectors of both chroma phases), a forced key frame, rate
    control on / off: bitstreams, reconstructions and decisions equal the CPU oracle's."""
    genc, cenc = _pair(gpu, w, h, kbps=kbps, qp=qp)
    frames = []
    for t in range(7):
        y, uv = synthetic_nv12(w, h, t, seed=t % 3)
        dy, duv = _dev(genc, y, uv)
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), t == 4)
        cau = cenc.encode(y, uv, t == 4)
        _check(genc, cenc, gau, cau, w, h, t)
        frames.append(gau)
    dec = Decoder()
    dec.decode(frames)
    assert dec.stats["key"] == 2 and dec.stats["inter"] == 5


def test_gpu_vp8_key_frame_through_libwebp(gpu):
    pil = pytest.importorskip("PIL.Image")
    w, h = 176, 144
    y, uv = _picture(w, h, 5)
    genc, _ = _pair(gpu, w, h, qp=26)
    dy, duv = _dev(genc, y, uv)
    frame = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
    ry, ruv = genc.recon()
    rgb = np.asarray(pil.open(io.BytesIO(webp_container(frame))).convert("RGB")).astype(np.int64)
    ref = libwebp_rgb(ry[:h, :w].astype(np.int64), ruv[:h // 2, 0:w:2].astype(np.int64),
                      ruv[:h // 2, 1:w:2].astype(np.int64))
    assert np.array_equal(rgb, ref)


def test_gpu_vp8_1080p_desktop(gpu):
    """The synthetic desktop at 1920x1080 with rate control: GPU == CPU for a key frame and P
    frames; the key frame decodes through libwebp to the encoder's reconstruction."""
    pil = pytest.importorskip("PIL.Image")
    w, h = 1920, 1080
    genc, cenc = _pair(gpu, w, h, kbps=8000, sr=16)
    for t in range(3):
        y, uv = desktop_nv12(gpu, w, h, t)
        dy, duv = _dev(genc, y, uv)
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
        cau = cenc.encode(y, uv, False)
        _check(genc, cenc, gau, cau, w, h, t)
        if t == 0:
            ry, ruv = genc.recon()
            rgb = np.asarray(pil.open(io.BytesIO(webp_container(gau))).convert("RGB")).astype(np.int64)
            ref = libwebp_rgb(ry[:h, :w].astype(np.int64), ruv[:h // 2, 0:w:2].astype(np.int64),
                              ruv[:h // 2, 1:w:2].astype(np.int64))
            assert np.array_equal(rgb, ref)
    st = genc.stats
    assert not st.idr and st.skipped_mbs > 0


@pytest.mark.parametrize("depth", [2, 3, 4])
def test_gpu_vp8_pipelined_matches(gpu, depth):
    """Depth 2 / 3 (the bitstreams of the frames in flight written concurrently by per-slot
    writer threads, beside the GPU analysis of the next frame) produce the depth-1 bitstream
    (fixed QP: with rate control the pipelined QP lags)."""
    w, h = 320, 192
    a, _ = _pair(gpu, w, h, qp=30)
    b, _ = _pair(gpu, w, h, qp=30, depth=depth)
    srcs = [_dev(a, *synthetic_nv12(w, h, t, seed=1)) for t in range(8)]
    ref = [a.encode(dy.data_ptr(), duv.data_ptr(), False) for dy, duv in srcs]
    out = []
    for t in range(len(srcs)):
        if t >= depth:
            out.append(b.collect())
        b.submit(srcs[t][0].data_ptr(), srcs[t][1].data_ptr(), False)
    while len(out) < len(srcs):
        out.append(b.collect())
    assert out == ref


def _sse(ry, ruv, y, uv, w, h):
    e = lambda a, b: int(((a.astype(np.int64) - b.astype(np.int64)) ** 2).sum())  # noqa: E731
    cw, chh = (w + 1) // 2, (h + 1) // 2
    return (e(ry[:h, :w], y[:h, :w]), e(ruv[:chh, 0:2 * cw:2], uv[:chh, 0:2 * cw:2]),
            e(ruv[:chh, 1:2 * cw:2], uv[:chh, 1:2 * cw:2]))


@pytest.mark.parametrize("w,h,qp,aq", [(96, 64, 28, 4), (100, 60, 44, 2), (320, 192, 24, 4), (176, 144, 54, 4)])
def test_gpu_vp8_loop_filter_bit_exact_vs_cpu(gpu, w, h, qp, aq):
    """The loop filter forced on (deblock 1): k_vp8_lf's wavefront gives the CPU oracle's filtered
    reconstruction, bitstream and records for key and inter frames (per-segment levels with aq 4);
    the frame statistics' distortion is the filtered picture's; the in-tree decoder agrees."""
    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height, cfg.fps, cfg.qp, cfg.bitrate_kbps, cfg.search_range = w, h, 60, qp, 0, 8
    cfg.deblock, cfg.aq = 1, aq
    genc, cenc = gpu.GpuVp8Encoder(cfg, _stream()), gpu.CpuVp8Encoder(cfg)
    frames = []
    for t in range(7):
        y, uv = synthetic_nv12(w, h, t, seed=t % 3)
        dy, duv = _dev(genc, y, uv)
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), t == 4)
        cau = cenc.encode(y, uv, t == 4)
        _check(genc, cenc, gau, cau, w, h, t)
        gy, guv = genc.recon()
        assert tuple(genc.stats.sse) == _sse(gy, guv, y, uv, w, h), f"frame {t}"
        frames.append(gau)
    dec = Decoder()
    dec.decode(frames)
    assert dec.stats["filtered"] == 7


def test_gpu_vp8_adaptive_loop_filter_1080p_pan(gpu):
    """1080p synthetic desktop panning 2 px per frame (coherent motion), adaptive filter
    (deblock 2): GPU == CPU through the switch-on kStatsLag frames in, and depth 4 (frames in
    flight, writer threads) gives the depth-1 bitstream."""
    w, h = 1920, 1080
    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height, cfg.fps, cfg.qp, cfg.bitrate_kbps, cfg.search_range = w, h, 60, 34, 0, 16
    cfg.deblock = 2
    genc, cenc = gpu.GpuVp8Encoder(cfg, _stream()), gpu.CpuVp8Encoder(cfg)
    y0, uv0 = desktop_nv12(gpu, w + 64, h, 0)
    srcs = [(np.ascontiguousarray(y0[:, 2 * t:2 * t + w]), np.ascontiguousarray(uv0[:, 2 * t:2 * t + w]))
            for t in range(8)]
    devs = [_dev(genc, y, uv) for y, uv in srcs]
    ref, flags = [], []
    for t, ((y, uv), (dy, duv)) in enumerate(zip(srcs, devs)):
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
        cau = cenc.encode(y, uv, False)
        _check(genc, cenc, gau, cau, w, h, t)
        assert genc.stats.deblocked == cenc.stats.deblocked
        flags.append(int(genc.stats.deblocked))
        ref.append(gau)
    assert flags == [0, 0, 0, 0, 0, 1, 1, 1], flags
    cfg.pipeline_depth = 4
    b = gpu.GpuVp8Encoder(cfg, _stream())
    out = []
    for t, (dy, duv) in enumerate(devs):
        if t >= 4:
            out.append(b.collect())
        b.submit(dy.data_ptr(), duv.data_ptr(), False)
    while len(out) < len(devs):
        out.append(b.collect())
    assert out == ref


@pytest.mark.parametrize("w,h,qp,lf", [(640, 368, 20, 0), (640, 368, 34, 1), (1920, 1080, 46, 1), (100, 60, 30, 1)])
def test_gpu_vp8_bpred_key_frames_bit_exact_vs_cpu(gpu, w, h, qp, lf):
    """B_PRED key frames (k_vp8_key's sub-block steps, the modes handed down the wavefront as
    contexts; the loop filter's inner edges in every B_PRED macroblock): GPU == CPU, B_PRED
    macroblocks present, then P frames on top of the B_PRED reference."""
    genc, cenc = _pair(gpu, w, h, qp=qp, deblock=lf)
    frames = []
    for t in range(3):
        y, uv = desktop_nv12(gpu, w, h, t)
        dy, duv = _dev(genc, y, uv)
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
        cau = cenc.encode(y, uv, False)
        _check(genc, cenc, gau, cau, w, h, t)
        frames.append(gau)
    if w * h > 640 * 368:  # (the pure-Python decoder: small pictures only)
        assert genc.stats.bytes > 0
        return
    dec = Decoder()
    dec.decode(frames)
    assert dec.stats.get("bpred", 0) > 0 and dec.stats["key"] == 1
    assert np.array_equal(dec.frames_coded[-1][0], genc.recon()[0])


@pytest.mark.parametrize("qp,lf", [(24, 0), (44, 1)])
def test_gpu_vp8_intra_in_inter_bit_exact_vs_cpu(gpu, qp, lf):
    """Intra macroblocks in inter frames (k_vp8_intra_cand / k_vp8_intra_code after k_vp8_inter):
    GPU == CPU, the stream decodes to the reconstruction, intra macroblocks present."""
    w, h = 320, 192
    genc, cenc = _pair(gpu, w, h, qp=qp, deblock=lf)
    frames = []
    for t in range(5):
        y, uv = synthetic_nv12(w, h, t, seed=t % 3)
        dy, duv = _dev(genc, y, uv)
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
        cau = cenc.encode(y, uv, False)
        _check(genc, cenc, gau, cau, w, h, t)
        frames.append(gau)
    dec = Decoder()
    dec.decode(frames)
    assert dec.stats.get("intra_p", 0) > 0
    assert np.array_equal(dec.frames_coded[-1][0], genc.recon()[0])
