"""HEVC encoder tests.

CPU tier: the C++ CPU HEVC encoder (same decisions as the HIP kernels) is decoded by the
independent pure-Python decoder (mxdesk/codec/hevc_decoder.py) and the decoded pictures
must equal the encoder's reconstruction exactly.  No HEVC reference decoder exists in
this image (no ffmpeg / libde265), so conformance to other decoders is "parity
unpinned"; the tables are additionally checked against their closed-form definitions.

GPU tier: the HIP encoder's bitstream must be bit-identical to the CPU encoder's, and its
reconstruction must equal the decoded pictures.
"""
import math

import numpy as np
import pytest

from mxdesk.codec import hevc_decoder as hd
from mxdesk.codec.hevc_decoder import Decoder, psnr

from .test_cpu_encoder import synthetic_nv12


def _cfg(native, w, h, fps=60, qp=28, bitrate=0, aq=1, sr=8, tu_split=0):
    cfg = native.EncoderConfig()
    cfg.tu_split = tu_split
    cfg.width, cfg.height, cfg.fps = w, h, fps
    cfg.bitrate_kbps = bitrate
    cfg.qp = qp
    cfg.aq = aq
    cfg.search_range = sr
    return cfg


def _cpu_roundtrip(native, w, h, frames, fps=60, qp=28, bitrate=0, fresh=False, idr_at=(), tu_split=0, wpp=None):
    cfg = _cfg(native, w, h, fps, qp, bitrate, tu_split=tu_split)
    if wpp is not None:
        cfg.hevc_wpp = wpp
    enc = native.CpuHevcEncoder(cfg)
    stream, recon, src, sizes = b"", [], [], []
    for t in range(frames):
        y, uv = synthetic_nv12(w, h, t, seed=t if fresh else 0)
        au = enc.encode(y, uv, t in idr_at)
        stream += au
        sizes.append(len(au))
        recon.append(tuple(p.copy() for p in enc.recon()))
        src.append(y)
    dec = Decoder()
    frames_out = dec.decode(stream)
    assert len(dec.frames_coded) == frames
    for i, ((y, u, v), (ry, ruv)) in enumerate(zip(dec.frames_coded, recon)):
        assert np.array_equal(y, ry), f"frame {i}: luma differs"
        assert np.array_equal(u, ruv[:, 0::2]), f"frame {i}: Cb differs"
        assert np.array_equal(v, ruv[:, 1::2]), f"frame {i}: Cr differs"
    return frames_out, src, sizes, dec, enc


@pytest.mark.parametrize("w,h,qp", [(64, 48, 28), (128, 96, 4), (128, 96, 51), (100, 60, 30), (320, 192, 22)])
def test_cpu_hevc_decodes_to_reconstruction(native, w, h, qp):
    out, src, sizes, dec, _ = _cpu_roundtrip(native, w, h, 3, qp=qp, fresh=True)
    assert out[0][0].shape == (h, w)  # conformance window crops the coded size
    if qp <= 30:
        assert psnr(out[0][0], src[0]) > 30
    assert dec.stats["intra"] == ((w + 15) // 16) * ((h + 15) // 16)


def test_cpu_hevc_static_frames_are_skipped(native):
    enc = native.CpuHevcEncoder(_cfg(native, 128, 64, qp=22))
    yy, xx = np.mgrid[0:64, 0:128]
    y = (40 + xx + yy).astype(np.uint8)
    uv = np.full((32, 128), 128, np.uint8)
    stream = enc.encode(y, uv, False)
    p = enc.encode(y, uv, False)
    stream += p
    assert set(enc.cu_types()) == {0}  # every CU skipped
    assert len(p) < 120  # 4 slice headers + one bin per CU
    Decoder().decode(stream)


def test_cpu_hevc_rate_control_and_idr(native):
    out, _, sizes, dec, enc = _cpu_roundtrip(native, 160, 96, 6, bitrate=300, idr_at=(3,))
    assert dec.stats["intra"] == 2 * 60  # two IDR pictures of 10 x 6 CUs
    assert enc.stats.idr == 0


def test_cpu_hevc_two_row_slices(native):
    # 192x544 @ 30 fps is level 2 (16 slice segments) -> 17 CTB rows need 2-row slices, which
    # exercises above-neighbour intra references, merge/AMVP B candidates and skip contexts
    _, _, _, dec, enc = _cpu_roundtrip(native, 192, 544, 2, fps=30, qp=30, wpp=1)
    assert enc.slice_rows == 2
    assert dec.stats["slices"] == 9 + 3  # 9 two-row slices in the IDR picture, 8-row WPP slices in the P picture
    assert dec.stats["substreams"] == 17 + 17  # one per CTB row: 9 slices (8 x 2 rows + 1), then 17 rows


@pytest.mark.parametrize("w,h,wpp,rows", [(16, 64, 1, 0), (32, 48, 1, 0), (160, 96, 1, 0), (160, 96, 0, 0),
                                           (200, 120, 1, 0), (160, 96, 1, 2), (200, 120, 1, 3)])
def test_cpu_hevc_wpp_substreams_decode(native, w, h, wpp, rows):
    """Wavefront substreams (one per CTB row; context sync from the row above's second CTB, none
    for a one-CTB-wide picture; QP predictor reset per row; entry points = escaped substream
    sizes, checked by the decoder) decode to the reconstruction, I and P pictures, with the
    slice-per-substream layout (wpp 0) as the control; rows > 0 splits P pictures into slices of
    that many CTB rows, each with its own wavefront (fresh contexts at every slice start)."""
    cfg = _cfg(native, w, h, qp=26, aq=1)
    cfg.hevc_wpp = wpp
    cfg.hevc_wpp_rows = rows
    enc = native.CpuHevcEncoder(cfg)
    stream, recon = b"", []
    for t in range(4):
        y, uv = synthetic_nv12(w, h, t, seed=t)
        stream += enc.encode(y, uv, t == 2)
        recon.append(tuple(p.copy() for p in enc.recon()))
    dec = Decoder()
    dec.decode(stream)
    for (yy, u, v), (ry, ruv) in zip(dec.frames_coded, recon):
        assert np.array_equal(yy, ry) and np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2])
    ctb_h = (h + 31) // 32  # 32x32 CTB rows
    assert dec.stats.get("substreams", 0) == (4 * ctb_h if wpp else 0)
    if wpp and rows:
        assert dec.stats["slices"] >= 4 * -(-ctb_h // rows)


def test_cpu_hevc_cost_balanced_p_slices(native):
    """P pictures are split into raster runs of equal estimated CABAC work (not CTU rows): a
    picture whose bottom half is noise gets most slice boundaries in the noisy half, slices
    start mid-row, and the stream still decodes to the reconstruction."""
    from mxdesk.codec import hevc_decoder as hd

    w, h = 320, 192
    cfg = _cfg(native, w, h, qp=22, aq=0)
    cfg.hevc_wpp = 0  # cost-balanced slices are the layout without wavefront substreams
    enc = native.CpuHevcEncoder(cfg)
    rng = np.random.default_rng(5)
    stream, recon = b"", []
    for t in range(3):
        y = np.full((h, w), 90, np.uint8)
        y[h // 2:] = rng.integers(0, 255, (h - h // 2, w))
        uv = np.full((h // 2, w), 128, np.uint8)
        stream += enc.encode(y, uv, False)
        recon.append(enc.recon())
    addrs = []
    for nal in hd.split_nal_units(stream):
        if (nal[0] >> 1) & 63 == 1:  # TRAIL_R slice: first_slice flag + address
            r = hd.BitReader(hd.unescape(nal), 16)
            first = r.u(1)
            r.ue()
            addrs.append(0 if first else r.u((12 * 20 - 1).bit_length()))
    ctb_w = w // 16
    p_addrs = addrs[: len(addrs) // 2]
    assert len(p_addrs) > 3 and any(a % ctb_w for a in p_addrs)  # mid-row slice starts
    assert sum(a >= (h // 32) * ctb_w for a in p_addrs) > len(p_addrs) // 2  # mostly in the noisy half
    dec = Decoder()
    dec.decode(stream)
    for (yy, u, v), (ry, ruv) in zip(dec.frames_coded, recon):
        assert np.array_equal(yy, ry) and np.array_equal(u, ruv[:, 0::2])


def test_hevc_level_selection(native):
    assert native.hevc_level(1920, 1080, 60) == 123  # 4.1
    assert native.hevc_level(3840, 2160, 60) == 153  # 5.1
    assert native.hevc_level(7680, 4320, 60) == 183  # 6.1
    assert native.hevc_level(1280, 720, 30) == 93  # 3.1


def test_decoder_tables_match_closed_forms():
    # CABAC rangeTabLps follows p_s = 0.5 * alpha^s, alpha = (0.01875 / 0.5)^(1/63), scaled by
    # the quantised range midpoints (rows 0-2 of column 0 are clipped to 128)
    alpha = (0.01875 / 0.5) ** (1 / 63)
    for s, row in enumerate(hd._RANGE_LPS[:63]):
        for q, v in enumerate(row):
            est = 0.5 * alpha ** s * (288 + 64 * q)
            if not (s < 3 and q == 0):
                assert abs(v - est) <= 3.5, (s, q, v, est)
    # transIdxLps follows p' = alpha * p + (1 - alpha)
    for s in range(1, 63):
        p = 0.5 * alpha ** s
        target = math.log((alpha * p + 1 - alpha) / 0.5) / math.log(alpha)
        assert abs(hd._TRANS_LPS[s] - target) <= 1.0, (s, hd._TRANS_LPS[s], target)
    # core transform: rows nearly orthogonal with norm 64^2 * N
    for n in (4, 8, 16, 32):
        t = hd._tmat(n).astype(np.float64)
        g = t @ t.T
        assert np.allclose(np.diag(g), 64 * 64 * n, rtol=0.01)
        off = g - np.diag(np.diag(g))
        assert np.abs(off).max() < 0.01 * 64 * 64 * n


def test_decoder_rejects_truncated_stream(native):
    enc = native.CpuHevcEncoder(_cfg(native, 64, 48))
    y, uv = synthetic_nv12(64, 48, 0)
    au = enc.encode(y, uv, False)
    with pytest.raises(Exception):
        Decoder().decode(au[:-3])


# ---------------------------------------------------------------------------- GPU tier
def _gpu_vs_cpu(gpu, w, h, frames, fps=60, qp=26, fresh=True, sr=8, tu_split=0, aq=1, desktop=False, sao=1,
                wpp=0, wpp_rows=8, intra_split=None, idr_at=()):
    import torch

    from .gpu_util import pitched

    cfg = _cfg(gpu, w, h, fps, qp, sr=sr, tu_split=tu_split, aq=aq)
    cfg.sao = sao
    cfg.hevc_wpp, cfg.hevc_wpp_rows = wpp, wpp_rows
    if intra_split is not None:
        cfg.hevc_intra_split = intra_split
    desk = None
    if desktop:
        from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

        desk = CpuSyntheticDesktop(w, h, True)
    stream = torch.cuda.current_stream().cuda_stream
    genc = gpu.GpuHevcEncoder(cfg, stream)
    cenc = gpu.CpuHevcEncoder(cfg)
    ch = genc.coded_height
    gs, grec = b"", []
    for t in range(frames):
        if desk is not None:
            y, uv = bgrx_to_nv12(desk.render(t, t / 60, 0))
        else:
            y, uv = synthetic_nv12(w, h, t, seed=t if fresh else 0)
        dy = pitched(y, genc.pitch, ch)
        duv = pitched(uv, genc.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), t in idr_at)
        cau = cenc.encode(y, uv, t in idr_at)
        assert bool(gau == cau), f"frame {t}: GPU HEVC bitstream differs from the CPU encoder ({len(gau)} vs {len(cau)})"
        gs += gau
        grec.append(genc.recon())
        cs = cenc.stats
        assert tuple(genc.stats.sse) == tuple(cs.sse)
    dec = Decoder()
    dec.decode(gs)
    if tu_split:
        assert dec.stats.get("tu_split", 0) > 0, "no CU chose the split transform tree"
    for (yy, u, v), (ry, ruv) in zip(dec.frames_coded, grec):
        assert np.array_equal(yy, ry)
        assert np.array_equal(u, ruv[:, 0::2])
        assert np.array_equal(v, ruv[:, 1::2])


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,fps,qp", [(64, 48, 60, 26), (100, 60, 60, 30), (320, 192, 60, 22), (352, 288, 30, 30),
                                        (128, 96, 60, 4)])
def test_gpu_hevc_bit_exact_vs_cpu(gpu, w, h, fps, qp):
    _gpu_vs_cpu(gpu, w, h, 3, fps=fps, qp=qp)


@pytest.mark.gpu
@pytest.mark.parametrize("intra_split", [0, 1])
@pytest.mark.parametrize("w,h,qp", [(320, 192, 22), (352, 288, 34), (1920, 1080, 40)])
def test_gpu_hevc_intra_split_bit_exact_vs_cpu(gpu, w, h, qp, intra_split):
    """IDR pictures with and without the intra transform-tree split (the second one forced, into
    reconstruction buffers that hold a previous picture): GPU == CPU == decoder, on the desktop."""
    _gpu_vs_cpu(gpu, w, h, 3, qp=qp, desktop=True, intra_split=intra_split, idr_at=(2,))


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,qp", [(160, 96, 30), (320, 192, 24), (100, 60, 38)])
def test_gpu_hevc_tu_split_bit_exact_vs_cpu(gpu, w, h, qp):
    """Split transform trees (8x8 luma / 4x4 chroma TUs), chosen per CU by the same rule on
    both sides: GPU bitstream == CPU bitstream, decoded == reconstruction (deblocking on)."""
    _gpu_vs_cpu(gpu, w, h, 4, qp=qp, tu_split=1)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,qp,desktop", [(64, 48, 26, False), (160, 96, 30, False), (320, 192, 28, True),
                                            (1920, 1080, 34, True)])
def test_gpu_hevc_4x4_luma_tus_bit_exact_vs_cpu(gpu, w, h, qp, desktop):
    """tu_split 2 on the GPU (split4_luma: sixteen 4x4 luma TUs on 4 lanes each, per-node SSE +
    lambda * bits choice against the 8x8 TU) == the CPU encoder, bit for bit; decoded ==
    reconstruction (CU32 / CU16 coding trees, deblocking, SAO on)."""
    _gpu_vs_cpu(gpu, w, h, 4, qp=qp, tu_split=2, aq=4 if desktop else 1, desktop=desktop)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,qp,tu_split,aq", [(320, 192, 30, 0, 3), (320, 192, 26, 1, 3), (1920, 1080, 34, 1, 3),
                                                 (320, 192, 30, 1, 4), (1920, 1080, 34, 1, 6)])
def test_gpu_hevc_temporal_classes_bit_exact_vs_cpu(gpu, w, h, qp, tu_split, aq):
    """aq 3+ on the synthetic desktop (animated noise panel = changing content, static windows =
    static / persistent; aq 4+ refines the static class 9+ QP finer): temporal classes, chroma drop
    and the luma residual drop decide the same on the GPU and the CPU, bit for bit, and the stream
    decodes to the GPU reconstruction."""
    _gpu_vs_cpu(gpu, w, h, 4, qp=qp, tu_split=tu_split, aq=aq, desktop=True)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,qp,sao", [(160, 96, 30, 0), (320, 192, 38, 1), (1920, 1080, 40, 1)])
def test_gpu_hevc_sao_bit_exact_vs_cpu(gpu, w, h, qp, sao):
    """SAO on the GPU (k_hevc_sao: CTB-parallel statistics, decision and offsets, CABAC sao()
    syntax) == the CPU encoder, bit for bit, at toy size and 1080p; sao=0 keeps the plain path."""
    _gpu_vs_cpu(gpu, w, h, 4, qp=qp, tu_split=1, aq=3, desktop=True, sao=sao)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,qp,rows", [(320, 192, 26, 0), (320, 192, 30, 2), (200, 120, 30, 0), (1920, 1080, 34, 8)])
def test_gpu_hevc_wpp_bit_exact_vs_cpu(gpu, w, h, qp, rows):
    """Wavefront substreams on the GPU (one k_hevc_arith wave per CTU row, contexts handed down
    from the row above's second CTU by release/acquire flags; slices of `rows` CTU rows, 0 = one
    per picture) == the CPU encoder bit for bit, and the decoder checks the entry points."""
    _gpu_vs_cpu(gpu, w, h, 4, qp=qp, tu_split=1, aq=3, desktop=True, wpp=1, wpp_rows=rows)


@pytest.mark.gpu
def test_gpu_session_hevc_stream(gpu):
    from .test_gpu_pipeline import _read_barcode

    cfg = gpu.SessionConfig()
    cfg.width, cfg.height, cfg.fps = 320, 192, 60
    cfg.codec = "hevc"
    cfg.enc.bitrate_kbps = 0
    cfg.enc.qp = 24
    s = gpu.Session(cfg)
    assert s.codec == "hevc"
    stream, ids = b"", []
    for _ in range(4):
        r = s.step(False)
        stream += r.au
        ids.append(r.frame_id)
        assert r.psnr_y > 30
    s.request_idr()
    r = s.step(False)
    assert r.idr == 1
    stream += r.au
    ids.append(r.frame_id)
    frames = Decoder().decode(stream)
    assert len(frames) == 5
    for (y, _, _), fid in zip(frames, ids):
        assert _read_barcode(y, gpu.BARCODE_CELL, gpu.BARCODE_X, gpu.BARCODE_Y)[0] == fid


def test_cpu_hevc_deblocking(native):
    """In-loop deblocking (8.7.2): the filtered reconstruction is what the decoder outputs,
    it differs from the unfiltered one at a coarse QP, and it is closer to the source."""
    out = {}
    for db in (0, 1):
        cfg = _cfg(native, 160, 96, qp=40)
        cfg.deblock = db
        enc = native.CpuHevcEncoder(cfg)
        stream, recon, err = b"", [], 0.0
        for t in range(3):
            y, uv = synthetic_nv12(160, 96, t)
            stream += enc.encode(y, uv, False)
            recon.append(enc.recon()[0].copy())
            err += float(((recon[-1][:96, :160].astype(np.int64) - y) ** 2).sum())
        dec = Decoder()
        dec.decode(stream)
        assert all(np.array_equal(a[0], b) for a, b in zip(dec.frames_coded, recon))
        out[db] = (recon, err)
    assert not np.array_equal(out[0][0][0], out[1][0][0])
    assert out[1][1] < out[0][1]


@pytest.mark.parametrize("w,h,qp", [(64, 48, 28), (160, 96, 30), (100, 60, 40), (320, 192, 22)])
def test_cpu_hevc_tu_split_decodes_to_reconstruction(native, w, h, qp):
    """Inter transform trees split into 8x8 luma / 4x4 chroma TUs where SSE + lambda * bits
    prefers it; the independent decoder (with deblocking of the internal TU edges) must
    reproduce the reconstruction exactly and must actually see split trees."""
    out, src, sizes, dec, _ = _cpu_roundtrip(native, w, h, 4, qp=qp, fresh=True, tu_split=1)
    assert dec.stats.get("tu_split", 0) > 0


@pytest.mark.parametrize("qp", [22, 30, 38])
def test_cpu_hevc_intra_split_decodes_to_reconstruction(native, qp):
    """Intra units coded as four 8x8 luma / 4x4 chroma TUs, each predicted from the TUs before it,
    with the mode-dependent (horizontal / vertical) scans: the independent decoder reproduces the
    reconstruction exactly (IDR pictures, inter frames after them), sees split intra trees with
    every scanIdx, and with hevc_intra_split = 0 none."""
    from mxdesk.codec import hevc_decoder

    seen = set()
    orig = hevc_decoder.Decoder._residual

    def spy(self, cab, log2, cidx, intra_mode):
        if intra_mode is not None and (log2 == 2 or (log2 == 3 and cidx == 0)):
            seen.add(2 if 6 <= intra_mode <= 14 else (1 if 22 <= intra_mode <= 30 else 0))
        return orig(self, cab, log2, cidx, intra_mode)

    hevc_decoder.Decoder._residual = spy
    try:
        out, src, sizes, dec, _ = _cpu_roundtrip(native, 320, 192, 3, qp=qp, fresh=True, idr_at=(2,))
    finally:
        hevc_decoder.Decoder._residual = orig
    assert dec.stats.get("tu_split", 0) > 0
    assert seen == {0, 1, 2}
    cfg = _cfg(native, 320, 192, qp=qp)
    cfg.hevc_intra_split = 0
    enc = native.CpuHevcEncoder(cfg)
    y, uv = synthetic_nv12(320, 192, 0, seed=0)
    dec0 = Decoder()
    dec0.decode(enc.encode(y, uv, True))
    assert dec0.stats.get("tu_split", 0) == 0


@pytest.mark.parametrize("w,h,qp", [(64, 48, 26), (160, 96, 30), (320, 192, 34)])
def test_cpu_hevc_4x4_luma_tus_decode_to_reconstruction(native, w, h, qp):
    """tu_split 2: 8x8 luma nodes of split inter trees may code four 4x4 TUs (split_transform_flag
    at the 8x8 node, cbf_luma and cu_qp_delta per 4x4 TU, the node's chroma after the fourth) --
    the decoder reproduces the reconstruction and sees 4x4 trees."""
    cfg = _cfg(native, w, h, qp=qp, tu_split=2)
    enc = native.CpuHevcEncoder(cfg)
    stream, recon, n4 = b"", [], 0
    for t in range(4):
        y, uv = synthetic_nv12(w, h, t, seed=t)
        stream += enc.encode(y, uv, False)
        recon.append(tuple(p.copy() for p in enc.recon()))
        n4 += int((enc.cu_info()[:, 5] != 0).sum())
    dec = Decoder()
    dec.decode(stream)
    for (yy, u, v), (ry, ruv) in zip(dec.frames_coded, recon):
        assert np.array_equal(yy, ry) and np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2])
    assert n4 > 0, "no unit chose 4x4 luma TUs"


def test_cpu_hevc_4x4_luma_tus_save_bits_on_desktop(native):
    """On the synthetic desktop (text, window edges) 4x4 luma TUs code P pictures in fewer bytes at
    no worse PSNR than 8x8-only split trees."""
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    res = {}
    for split in (1, 2):
        enc = native.CpuHevcEncoder(_cfg(native, 320, 192, qp=30, tu_split=split, aq=4))
        desk = CpuSyntheticDesktop(320, 192, False)
        nbytes, err = 0, 0.0
        for f in range(8):
            y, uv = bgrx_to_nv12(desk.render(f, f / 60, 0))
            au = enc.encode(y, uv, False)
            if f:
                nbytes += len(au)
                err += float(((enc.recon()[0][:192, :320].astype(np.int64) - y) ** 2).sum())
        res[split] = (nbytes, err)
    assert res[2][0] < res[1][0] * 0.95 and res[2][1] <= res[1][1], res


def test_cpu_hevc_tu_split_saves_bits_on_desktop_content(native):
    """On the synthetic desktop the split tree codes P pictures in fewer bytes at a higher
    PSNR than 16x16-only TUs (profiles/r01_rd)."""
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    res = {}
    for split in (0, 1):
        enc = native.CpuHevcEncoder(_cfg(native, 320, 192, qp=32, tu_split=split))
        desk = CpuSyntheticDesktop(320, 192, False)
        nbytes, err = 0, 0.0
        for f in range(6):
            y, uv = bgrx_to_nv12(desk.render(f, f / 60, 0))
            au = enc.encode(y, uv, False)
            if f:
                nbytes += len(au)
                err += float(((enc.recon()[0][:192, :320].astype(np.int64) - y) ** 2).sum())
        res[split] = (nbytes, err)
    assert res[1][0] < res[0][0] and res[1][1] <= res[0][1] * 1.02


@pytest.mark.parametrize("tu_split", [0, 1])
def test_cpu_hevc_temporal_classes(native, tu_split):
    """Temporal AQ classes (aq 3, shared with H.264: h264_mb.h temporal_class): on the synthetic
    desktop the animated noise panel is 'changing' (QP + 6, chroma residual dropped, luma kept
    only when it pays for its bits), static content 'persistent' (QP - 6); the stream decodes to
    the reconstruction and noise CUs actually drop their residual."""
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    w, h, qp = 640, 384, 40  # (a noise panel of ~12 units: some drop their residual)
    enc = native.CpuHevcEncoder(_cfg(native, w, h, qp=qp, aq=3, tu_split=tu_split))
    desk = CpuSyntheticDesktop(w, h, True)
    stream, recon, infos = b"", [], []
    for f in range(6):
        y, uv = bgrx_to_nv12(desk.render(f, f / 60, 0))
        stream += enc.encode(y, uv, False)
        recon.append(tuple(p.copy() for p in enc.recon()))
        if f:
            infos.append(enc.cu_info())
    info = np.concatenate(infos)
    qps = set(info[:, 1].tolist())
    assert qp + 6 in qps and qp - 6 in qps, qps
    changing = info[info[:, 1] == qp + 6]
    if not tu_split:  # (8x8 TUs code noise efficiently enough to keep it at this QP)
        assert (changing[:, 2] == 0).sum() > 0, "no changing CU dropped its residual"
    assert not (changing[:, 2] & 6).any(), "changing CUs must not code chroma"
    dec = Decoder()
    dec.decode(stream)
    for (yy, u, v), (ry, ruv) in zip(dec.frames_coded, recon):
        assert np.array_equal(yy, ry) and np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2])


def test_cpu_hevc_sao(native):
    """Sample adaptive offset (8.7.3): CTBs choose band and edge offsets (and merge with equal
    neighbours); the decoder's SAO output equals the encoder's reconstruction, and at equal QP
    SAO lowers the distortion of the synthetic desktop (text / window edges ring at coarse QPs)."""
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    w, h = 320, 192
    res = {}
    for sao in (0, 1):
        cfg = _cfg(native, w, h, qp=38, aq=3, tu_split=1)
        cfg.sao = sao
        enc = native.CpuHevcEncoder(cfg)
        desk = CpuSyntheticDesktop(w, h, True)
        stream, recon, err = b"", [], 0
        for f in range(4):
            y, uv = bgrx_to_nv12(desk.render(f, f / 60, 0))
            stream += enc.encode(y, uv, False)
            recon.append(tuple(p.copy() for p in enc.recon()))
            err += sum(enc.stats.sse)
        dec = Decoder()
        dec.decode(stream)
        for (yy, u, v), (ry, ruv) in zip(dec.frames_coded, recon):
            assert np.array_equal(yy, ry) and np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2])
        res[sao] = (err, len(stream), dec.stats)
    st = res[1][2]
    assert st.get("sao_band", 0) > 0 and st.get("sao_edge", 0) > 0 and st.get("sao_merge", 0) > 0, st
    assert "sao_band" not in res[0][2]
    assert res[1][0] < res[0][0] * 0.97, (res[0][:2], res[1][:2])


def test_hevc_sao_edge_categories():
    """The decoder's edge-offset categories follow 8.7.3.2 (edgeIdx = 2 + sign + sign, with
    0, 1, 2 remapped to 1, 2, 0)."""
    # edge categories: valley, concave corner, flat, convex corner, peak
    cat = hd._SAO_EDGE_CAT
    for c, a, b, want in [(1, 5, 5, 1), (1, 1, 5, 2), (3, 3, 3, 0), (5, 5, 1, 3), (9, 1, 1, 4), (2, 1, 3, 0)]:
        e = 2 + int(np.sign(c - a)) + int(np.sign(c - b))
        assert cat[e] == want, (c, a, b)


def test_token_path_matches_direct_cabac(native):
    """Two-phase CABAC (binarise every CTU into bin tokens, then the arithmetic coder over the
    token run: what k_hevc_bins / k_hevc_arith do) is byte-identical to coding the syntax
    directly, on random slices covering every CU type, split transform trees, escape-range
    levels, long motion-vector differences and SAO merge / band / edge parameters."""
    for seed in (1, 2, 3, 4):
        assert native.hevc_token_selftest(seed, 200) == 200


def _adaptive_frames(w, h):
    from .test_deblock import _pan_frames

    frames = [(y, uv, t == 4) for t, (y, uv) in enumerate(_pan_frames(w, h, 6))]
    return frames + [(y, uv, False) for y, uv in _pan_frames(w, h, 5, still=True)]


def test_cpu_hevc_adaptive_deblocking_follows_motion(native):
    """deblock=2: the pan's P pictures (and the forced IDR after them) are filtered, the still
    stretch is not; the PPS enables the slice override and every picture decodes exactly."""
    w, h = 192, 96
    cfg = _cfg(native, w, h, qp=34)
    cfg.deblock = 2
    enc = native.CpuHevcEncoder(cfg)
    stream, recon, flags = b"", [], []
    for y, uv, idr in _adaptive_frames(w, h):
        stream += enc.encode(y, uv, idr)
        recon.append(tuple(p.copy() for p in enc.recon()))
        flags.append(enc.stats.deblocked)
    assert flags[0] == 0 and flags[1:5] == [1, 1, 1, 1] and flags[-1] == 0, flags
    dec = Decoder()
    dec.decode(stream)
    for i, ((yy, u, v), (ry, ruv)) in enumerate(zip(dec.frames_coded, recon)):
        assert np.array_equal(yy, ry), f"frame {i}"
        assert np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2]), f"frame {i}"


@pytest.mark.gpu
@pytest.mark.parametrize("sao", [0, 1])
def test_gpu_hevc_adaptive_deblocking_bit_exact_vs_cpu(gpu, sao):
    """k_hevc_db_auto's decision equals the CPU encoder's: identical streams through a pan, a
    forced IDR and a still stretch."""
    import torch

    from .gpu_util import pitched

    w, h = 192, 96
    cfg = _cfg(gpu, w, h, qp=34)
    cfg.deblock, cfg.sao = 2, sao
    genc = gpu.GpuHevcEncoder(cfg, torch.cuda.current_stream().cuda_stream)
    cenc = gpu.CpuHevcEncoder(cfg)
    ch = genc.coded_height
    flags = []
    for t, (y, uv, idr) in enumerate(_adaptive_frames(w, h)):
        dy = pitched(y, genc.pitch, ch)
        duv = pitched(uv, genc.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), idr)
        cau = cenc.encode(y, uv, idr)
        assert bool(gau == cau), f"frame {t}: GPU HEVC bitstream differs from the CPU encoder"
        assert genc.stats.deblocked == cenc.stats.deblocked, t
        flags.append(genc.stats.deblocked)
    assert flags[1:5] == [1, 1, 1, 1], flags  # (the still stretch's decisions depend on the SAO setting)
