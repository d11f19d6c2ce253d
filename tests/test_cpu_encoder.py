"""CPU H.264 encoder (the no-GPU plumbing encoder and the GPU oracle) -> independent
decoder: the decoded pictures must equal the encoder's reconstruction bit-exactly."""
import numpy as np
import pytest

from mxdesk.codec.h264_decoder import Decoder, psnr


def synthetic_nv12(w, h, t, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    y = 128 + 60 * np.sin((xx + 3 * t) / 7.0) + 40 * np.cos((yy + 2 * t) / 5.0)
    y = y.astype(np.uint8)
    y[h // 4: h // 2, 8 + 2 * t: 24 + 2 * t] = 230
    y[h // 2:, : w // 3] = rng.integers(0, 255, (h - h // 2, w // 3)).astype(np.uint8)  # noise patch
    uv = np.empty((h // 2, w), np.uint8)
    uv[:, 0::2] = (128 + 30 * np.sin(xx[::2, ::2] / 9.0 + t)).astype(np.uint8)
    uv[:, 1::2] = (128 + 30 * np.cos(yy[::2, ::2] / 7.0)).astype(np.uint8)
    return y, uv


def encode_decode(native, w, h, frames, **kw):
    cfg = native.EncoderConfig()
    cfg.width, cfg.height = w, h
    cfg.bitrate_kbps = kw.get("bitrate_kbps", 0)
    cfg.qp = kw.get("qp", 28)
    cfg.search_range = kw.get("search_range", 8)
    cfg.subpel = kw.get("subpel", 1)
    cfg.keyint = kw.get("keyint", 0)
    cfg.intra_in_p = kw.get("intra_in_p", 1)
    enc = native.CpuH264Encoder(cfg)
    stream, recon, src, sizes = b"", [], [], []
    for t in range(frames):
        y, uv = synthetic_nv12(w, h, t)
        au = enc.encode(y, uv, False)
        sizes.append(len(au))
        stream += au
        recon.append(tuple(p.copy() for p in enc.recon()))
        src.append(y)
    dec = Decoder()
    out = dec.decode(stream)
    return dec, out, recon, src, sizes, enc


@pytest.mark.parametrize("w,h,subpel", [(64, 48, 1), (96, 64, 0), (100, 60, 1), (48, 32, 1)])
def test_roundtrip_bit_exact(native, w, h, subpel):
    dec, out, recon, src, sizes, _ = encode_decode(native, w, h, 4, subpel=subpel)
    assert len(out) == 4
    for (y, u, v), (ry, ruv) in zip(dec.frames_coded, recon):
        assert np.array_equal(y, ry)
        assert np.array_equal(u, ruv[:, 0::2])
        assert np.array_equal(v, ruv[:, 1::2])
    for (y, _, _), s in zip(out, src):
        assert y.shape == (h, w)
        assert psnr(y, s) > 30


def test_static_content_skips(native):
    cfg = native.EncoderConfig()
    cfg.width, cfg.height, cfg.bitrate_kbps, cfg.qp, cfg.subpel = 64, 48, 0, 30, 0
    enc = native.CpuH264Encoder(cfg)
    y, uv = synthetic_nv12(64, 48, 0)
    big = len(enc.encode(y, uv, False))
    # aq 4 (default): the unchanged source (zero vector) is "static" content, refined once 9 QP
    # finer than the IDR, then skipped
    enc.encode(y, uv, False)
    small = len(enc.encode(y, uv, False))
    assert enc.stats.skipped_mbs >= 6
    assert small < big / 4
    cfg.aq = 2  # residual-energy classes: skipped right away
    enc = native.CpuH264Encoder(cfg)
    big = len(enc.encode(y, uv, False))
    small = len(enc.encode(y, uv, False))
    assert enc.stats.skipped_mbs >= 6
    assert small < big / 4


def test_forced_idr_and_keyint(native):
    dec, out, recon, src, sizes, enc = encode_decode(native, 64, 48, 5, keyint=2, intra_in_p=0)
    assert dec.stats["i16"] + dec.stats["i4"] == 12 * 3  # IDR at frames 0, 2, 4


def test_intra4x4_and_intra_in_p_round_trip(native):
    """Intra4x4 IDR macroblocks and intra macroblocks inside P slices (a new high-contrast patch
    every frame that inter prediction cannot follow) decode to the reconstruction."""
    w, h = 96, 64
    cfg = native.EncoderConfig()
    cfg.width, cfg.height, cfg.bitrate_kbps, cfg.qp = w, h, 0, 26
    cfg.intra_in_p = 1
    enc = native.CpuH264Encoder(cfg)
    rng = np.random.default_rng(7)
    stream, recon = b"", []
    for t in range(4):
        y, uv = synthetic_nv12(w, h, t)
        # text-like glyph patch at a fresh position: sharp edges, no temporal match
        gy, gx = 4 + 8 * t, 40 + 10 * t
        glyph = (rng.integers(0, 2, (16, 16)) * 200 + 20).astype(np.uint8)
        y[gy:gy + 16, gx:gx + 16] = glyph
        stream += enc.encode(y, uv, False)
        recon.append(enc.recon()[0].copy())
    dec = Decoder()
    dec.decode(stream)
    assert dec.stats["i4"] > 0, dec.stats
    p_intra = dec.stats["i4"] + dec.stats["i16"] - 24  # minus the 24 IDR macroblocks
    assert p_intra > 0, dec.stats
    for i, (yd, _, _) in enumerate(dec.frames_coded):
        assert np.array_equal(yd, recon[i]), i


def test_rate_control_moves_qp(native):
    cfg = native.EncoderConfig()
    cfg.width, cfg.height, cfg.fps, cfg.bitrate_kbps, cfg.qp = 96, 64, 30, 20, 20
    cfg.qp_min, cfg.qp_max = 10, 51
    enc = native.CpuH264Encoder(cfg)
    qps = []
    for t in range(12):
        y, uv = synthetic_nv12(96, 64, t)
        enc.encode(y, uv, False)
        qps.append(enc.stats.qp)
    # a starved budget (20 kbps) drives the QP up immediately (probe-sized first IDR, bit-budget
    # model), not one step per frame
    assert min(qps[:3]) >= 40 and qps[-1] >= 40, qps


def test_adaptive_quantisation_roundtrip_and_saves_bits(native):
    """Noise that changes every frame (incompressible after motion compensation) gets a coarser
    macroblock QP via mb_qp_delta; the stream still decodes bit-exactly to the reconstruction."""
    w, h = 96, 64

    def run(aq):
        cfg = native.EncoderConfig()
        cfg.width, cfg.height, cfg.bitrate_kbps, cfg.qp, cfg.search_range = w, h, 0, 24, 8
        cfg.aq = aq
        enc = native.CpuH264Encoder(cfg)
        stream, recon = b"", []
        for t in range(4):
            y, uv = synthetic_nv12(w, h, t, seed=t)  # fresh noise every frame
            stream += enc.encode(y, uv, False)
            recon.append(tuple(p.copy() for p in enc.recon()))
        return stream, recon

    s_on, rec_on = run(1)
    s_off, _ = run(0)
    assert len(s_on) < 0.9 * len(s_off)
    # aq=2 adds the rate-distortion residual drop for noise-like MBs: fewer bits again
    s_drop, rec_drop = run(2)
    assert len(s_drop) <= len(s_on)
    dec2 = Decoder()
    dec2.decode(s_drop)
    for (y, u, v), (ry, ruv) in zip(dec2.frames_coded, rec_drop):
        assert np.array_equal(y, ry) and np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2])
    dec = Decoder()
    dec.decode(s_on)
    for (y, u, v), (ry, ruv) in zip(dec.frames_coded, rec_on):
        assert np.array_equal(y, ry) and np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2])


def test_multi_slice_idr_round_trip(native):
    """IDR pictures are coded as <= 4-MB-row slices (the GPU wavefront's workgroup per slice,
    idr_slice_rows): 10 MB rows -> 3 slices of 4/4/2 rows, no intra prediction across them;
    the independent decoder reproduces the reconstruction."""
    w, h = 64, 160
    dec, out, recon, _, _, _ = encode_decode(native, w, h, 2, intra_in_p=0)
    cfg = native.EncoderConfig()
    cfg.width, cfg.height, cfg.bitrate_kbps, cfg.qp = w, h, 0, 28
    enc = native.CpuH264Encoder(cfg)
    y, uv = synthetic_nv12(w, h, 0)
    au = enc.encode(y, uv, False)
    nal_types = [au[i + 3] & 0x1F for i in range(len(au) - 3) if au[i:i + 3] == b"\x00\x00\x01"]
    assert nal_types.count(5) == 3, nal_types
    for (yd, ud, vd), (ry, ruv) in zip(dec.frames_coded, recon):
        assert np.array_equal(yd, ry)
        assert np.array_equal(ud, ruv[:, 0::2])
        assert np.array_equal(vd, ruv[:, 1::2])
