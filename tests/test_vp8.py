"""VP8 encoder (RFC 6386; WEBRTC_ENCODER=vp8enc, reference README.md:21,35).

Key frames are pinned to a real VP8 decoder: lossy WebP *is* a VP8 key frame, so the encoder's
key frames, wrapped in a RIFF/WEBP container, go through libwebp (Pillow) and must come out as
exactly the encoder's reconstruction -- luma through libwebp's YUV->RGB formula, chroma through a
model of its 'fancy' (9-3-3-1) upsampler, every RGB sample equal.  Inter frames have no decoder
in the image besides the in-tree one (mxdesk/codec/vp8_decoder.py, written from the decoding
side of the RFC), so their parity beyond it is unpinned."""
import io

import numpy as np
import pytest

from mxdesk.codec.vp8_decoder import Decoder, webp_container

from .test_cpu_encoder import synthetic_nv12

Image = pytest.importorskip("PIL.Image")
pytestmark = pytest.mark.skipif(not __import__("PIL.features").features.check("webp"), reason="Pillow without WebP")


def libwebp_rgb(Y, U, V):
    """libwebp's RGB output for 4:2:0 planes: fancy upsampling (row pairs, 9-3-3-1 weights) then
    the 14-bit fixed-point YUV->RGB of its yuv.h."""
    h, w = Y.shape
    out = np.zeros((h, w, 3), np.int64)
    mh = lambda v, c: (v * c) >> 8  # noqa: E731

    def emit(yrow, u, v, dst):
        dst[:, 0] = np.clip((mh(yrow, 19077) + mh(v, 26149) - 14234) >> 6, 0, 255)
        dst[:, 1] = np.clip((mh(yrow, 19077) - mh(u, 6419) - mh(v, 13320) + 8708) >> 6, 0, 255)
        dst[:, 2] = np.clip((mh(yrow, 19077) + mh(u, 33050) - 17685) >> 6, 0, 255)

    def pair(tu, cu, n):
        top, bot = np.zeros(n, np.int64), np.zeros(n, np.int64)
        tl, lf = int(tu[0]), int(cu[0])
        top[0], bot[0] = (3 * tl + lf + 2) >> 2, (3 * lf + tl + 2) >> 2
        for x in range(1, ((n - 1) >> 1) + 1):
            t, c = int(tu[x]), int(cu[x])
            avg = tl + t + lf + c + 8
            d12, d03 = (avg + 2 * (t + lf)) >> 3, (avg + 2 * (tl + c)) >> 3
            top[2 * x - 1], top[2 * x] = (d12 + tl) >> 1, (d03 + t) >> 1
            bot[2 * x - 1], bot[2 * x] = (d03 + lf) >> 1, (d12 + c) >> 1
            tl, lf = t, c
        if not n & 1:
            top[n - 1], bot[n - 1] = (3 * tl + lf + 2) >> 2, (3 * lf + tl + 2) >> 2
        return top, bot

    emit(Y[0], pair(U[0], U[0], w)[0], pair(V[0], V[0], w)[0], out[0])
    k = 1
    while 2 * k - 1 < h:
        ut, ub = pair(U[k - 1], U[min(k, U.shape[0] - 1)], w)
        vt, vb = pair(V[k - 1], V[min(k, V.shape[0] - 1)], w)
        emit(Y[2 * k - 1], ut, vt, out[2 * k - 1])
        if 2 * k < h:
            emit(Y[2 * k], ub, vb, out[2 * k])
        k += 1
    if not h & 1:
        emit(Y[h - 1], pair(U[h // 2 - 1], U[h // 2 - 1], w)[0], pair(V[h // 2 - 1], V[h // 2 - 1], w)[0], out[h - 1])
    return out


def _picture(w, h, seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    y = (40 + 60 * np.sin(xx / 7.0) + 50 * np.cos(yy / 5.0) + rng.integers(0, 40, (h, w))).clip(16, 235)
    cy, cx = np.mgrid[0:h // 2, 0:w // 2]
    u = (128 + 50 * np.sin(cx / 5.0) + rng.integers(-20, 20, (h // 2, w // 2))).clip(16, 240)
    v = (128 + 50 * np.cos(cy / 4.0) + rng.integers(-20, 20, (h // 2, w // 2))).clip(16, 240)
    uv = np.zeros((h // 2, w), np.uint8)
    uv[:, 0::2], uv[:, 1::2] = u, v
    return y.astype(np.uint8), uv


def _encoder(native, w, h, **kw):
    c = native.EncoderConfig()
    c.width, c.height = w, h
    c.bitrate_kbps, c.qp, c.search_range = kw.get("kbps", 0), kw.get("qp", 30), kw.get("sr", 8)
    c.aq = kw.get("aq", c.aq)
    return native.CpuVp8Encoder(c)


@pytest.mark.parametrize("w,h,qp", [(96, 64, 20), (176, 144, 30), (64, 48, 44), (100, 60, 26)])
def test_key_frame_decodes_through_libwebp(native, w, h, qp):
    y, uv = _picture(w, h, qp)
    enc = _encoder(native, w, h, qp=qp)
    frame = enc.encode(y, uv)
    assert enc.stats.idr == 1 and not frame[0] & 1  # frame tag: key frame
    ry, ruv = enc.recon()
    rgb = np.asarray(Image.open(io.BytesIO(webp_container(frame))).convert("RGB")).astype(np.int64)
    ref = libwebp_rgb(ry[:h, :w].astype(np.int64), ruv[:h // 2, 0:w:2].astype(np.int64),
                      ruv[:h // 2, 1:w:2].astype(np.int64))
    assert rgb.shape == ref.shape and np.array_equal(rgb, ref), int((rgb != ref).any(axis=2).sum())


def test_gray_key_frame_luma_through_libwebp(native):
    # constant chroma: libwebp's RGB is a function of the luma alone -> equal to the formula
    w, h = 176, 96
    y, _ = _picture(w, h, 3)
    uv = np.full((h // 2, w), 128, np.uint8)
    enc = _encoder(native, w, h, qp=24)
    frame = enc.encode(y, uv)
    ry, ruv = enc.recon()
    assert (ruv == 128).all()
    rgb = np.asarray(Image.open(io.BytesIO(webp_container(frame))).convert("RGB")).astype(np.int64)
    Y = ry[:h, :w].astype(np.int64)
    assert np.array_equal(rgb[..., 0], np.clip((((Y * 19077) >> 8) + ((128 * 26149) >> 8) - 14234) >> 6, 0, 255))


@pytest.mark.parametrize("w,h,kbps,qp", [(96, 64, 0, 28), (160, 96, 0, 40), (100, 60, 300, 30), (320, 192, 600, 30)])
def test_inter_frames_decode_to_reconstruction(native, w, h, kbps, qp):
    """I + P frames of a moving scene (full-sample vectors of every parity -> the chroma six-tap
    half-sample phase), a forced key frame in the middle, rate control on / off."""
    enc = _encoder(native, w, h, kbps=kbps, qp=qp)
    frames, recs = [], []
    for t in range(7):
        y, uv = synthetic_nv12(w, h, t, seed=t % 3)
        frames.append(enc.encode(y, uv, t == 4))
        recs.append(tuple(a.copy() for a in enc.recon()))
    dec = Decoder()
    dec.decode(frames)
    for t, ((yy, u, v), (ry, ruv)) in enumerate(zip(dec.frames_coded, recs)):
        assert np.array_equal(yy, ry), f"frame {t} luma"
        assert np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2]), f"frame {t} chroma"
    assert dec.stats["key"] == 2 and dec.stats["inter"] == 5
    assert dec.stats["new"] > 0  # coded vectors


def test_vp8_psnr_and_motion(native):
    # the encoder tracks a translating picture: P frames are far smaller than the key frame
    # (aq 2: one quantiser; with the temporal classes the first P frame refines the moving picture)
    w, h = 192, 128
    base, uv0 = _picture(w + 32, h, 7)
    enc = _encoder(native, w, h, qp=26, sr=16, aq=2)
    sizes, psnrs = [], []
    for t in range(5):
        y = np.ascontiguousarray(base[:, 2 * t: 2 * t + w])
        uv = np.ascontiguousarray(uv0[:, 2 * t: 2 * t + w])
        sizes.append(len(enc.encode(y, uv)))
        ry, _ = enc.recon()
        mse = np.mean((ry[:h, :w].astype(float) - y) ** 2)
        psnrs.append(10 * np.log10(255 ** 2 / mse))
    assert min(psnrs) > 32, psnrs
    assert max(sizes[1:]) < sizes[0] / 3, sizes


@pytest.mark.parametrize("aq", [3, 4])
def test_segmented_inter_frames_decode_to_reconstruction(native, aq):
    """Inter frames segmented by the temporal classes (9.3: static / persistent windows finer,
    the animated noise panel coarser, segment map in every inter frame, absolute segment
    quantisers): the in-tree decoder reproduces the reconstruction and sees several segments; the
    static class lowers the distortion of the unchanged windows against aq 2."""
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    w, h = 640, 368
    desk = CpuSyntheticDesktop(w, h, True)
    srcs = [bgrx_to_nv12(desk.render(t, t / 60, 0)) for t in range(4)]

    def run(a):
        enc = _encoder(native, w, h, qp=34, sr=8, aq=a)
        frames, recs = [], []
        for y, uv in srcs:
            frames.append(enc.encode(y, uv))
            recs.append(tuple(x.copy() for x in enc.recon()))
        return frames, recs

    frames, recs = run(aq)
    dec = Decoder()
    dec.decode(frames)
    for t, ((yy, u, v), (ry, ruv)) in enumerate(zip(dec.frames_coded, recs)):
        assert np.array_equal(yy, ry), f"frame {t} luma"
        assert np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2]), f"frame {t} chroma"
    segs = {k: v for k, v in dec.stats.items() if k.startswith("seg")}
    assert len(segs) >= 2, segs
    if aq >= 4:
        assert segs.get("seg1", 0) > 0, segs  # the static class
    y4, _ = srcs[-1]
    flat, _ = run(2)
    dflat = Decoder()
    dflat.decode(flat)
    keep = np.ones((h, w), bool)  # outside the animated noise panel (the renderer's rectangle, bench.py)
    keep[int(h * 0.55) - 16:int(h * 0.77) + 17, int(w * 0.04) - 16:int(w * 0.20) + 17] = False
    err = lambda d: float(np.mean(((d.frames_coded[-1][0][:h, :w].astype(float) - y4[:h, :w]) ** 2)[keep]))  # noqa: E731
    assert err(dec) < 0.5 * err(dflat), (err(dec), err(dflat))


@pytest.mark.parametrize("w,h,qp", [(96, 64, 20), (176, 144, 34), (100, 60, 44), (64, 48, 54)])
def test_loop_filtered_key_frame_through_libwebp(native, w, h, qp):
    """The normal loop filter (section 15; levels 6..40 here, every hev threshold): libwebp's
    decode of the filtered key frame is the encoder's reconstruction -- which pins the filter's
    arithmetic, its edge order and intra prediction from the unfiltered picture to a real decoder."""
    y, uv = _picture(w, h, qp + 1)
    c = native.EncoderConfig()
    c.width, c.height, c.qp, c.bitrate_kbps, c.deblock = w, h, qp, 0, 1
    enc = native.CpuVp8Encoder(c)
    frame = enc.encode(y, uv)
    ry, ruv = enc.recon()
    rgb = np.asarray(Image.open(io.BytesIO(webp_container(frame))).convert("RGB")).astype(np.int64)
    ref = libwebp_rgb(ry[:h, :w].astype(np.int64), ruv[:h // 2, 0:w:2].astype(np.int64),
                      ruv[:h // 2, 1:w:2].astype(np.int64))
    assert np.array_equal(rgb, ref), int((rgb != ref).any(axis=2).sum())
    dec = Decoder()
    dec.decode([frame])
    assert dec.stats.get("filtered") == 1 and np.array_equal(dec.frames_coded[0][0], ry)
    c.deblock = 0  # the filter changed the picture
    ry0, _ = (lambda e: (e.encode(y, uv), e.recon())[1])(native.CpuVp8Encoder(c))
    assert not np.array_equal(ry0, ry)


@pytest.mark.parametrize("aq", [2, 4])
def test_loop_filtered_inter_frames_decode_to_reconstruction(native, aq):
    """Filtered key and inter frames (aq 4: per-segment levels, the static segment unfiltered):
    the in-tree decoder reproduces every reconstruction."""
    w, h = 160, 96
    c = native.EncoderConfig()
    c.width, c.height, c.qp, c.bitrate_kbps, c.search_range, c.deblock, c.aq = w, h, 36, 0, 8, 1, aq
    enc = native.CpuVp8Encoder(c)
    frames, recs = [], []
    for t in range(7):
        y, uv = synthetic_nv12(w, h, t, seed=t % 3)
        frames.append(enc.encode(y, uv, t == 4))
        recs.append(tuple(a.copy() for a in enc.recon()))
    dec = Decoder()
    dec.decode(frames)
    for t, ((yy, u, v), (ry, ruv)) in enumerate(zip(dec.frames_coded, recs)):
        assert np.array_equal(yy, ry), f"frame {t} luma"
        assert np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2]), f"frame {t} chroma"
    assert dec.stats["filtered"] == 7


def test_adaptive_loop_filter_follows_coherent_motion(native):
    """deblock 2 (adaptive): a still picture is never filtered; a pan switches the filter on
    kStatsLag (4) frames after the first panned frame, and the bitstream says so.  The default,
    -1, is the same adaptive rule."""
    w, h = 192, 128
    base, uv0 = _picture(w + 64, h, 9)

    def run(pan, mode=2):
        c = native.EncoderConfig()
        c.width, c.height, c.qp, c.bitrate_kbps, c.search_range, c.deblock = w, h, 32, 0, 16, mode
        enc = native.CpuVp8Encoder(c)
        frames = []
        for t in range(9):
            s = 2 * t if pan else 0
            frames.append(enc.encode(np.ascontiguousarray(base[:, s:s + w]), np.ascontiguousarray(uv0[:, s:s + w])))
        return frames

    dflt = native.EncoderConfig()
    assert dflt.deblock == -1
    for pan, want in ((False, 0), (True, 4)):
        frames = run(pan)
        dec = Decoder()
        filtered = []
        for f in frames:
            n = dec.stats.get("filtered", 0)
            dec.decode_frame(f)
            filtered.append(dec.stats.get("filtered", 0) - n)
        if pan:
            assert filtered[:5] == [0] * 5 and filtered[5:] == [1] * 4, filtered
        else:
            assert sum(filtered) == want, filtered
        assert run(pan, -1) == frames  # the default


@pytest.mark.parametrize("qp", [20, 34, 46])
def test_bpred_key_frame_through_libwebp(native, qp):
    """B_PRED key frames (12.3 sub-block modes under the contextual key-frame probabilities, no Y2
    block, type-3 luma tokens, the Y2 context carried past B_PRED macroblocks, inner loop-filter
    edges always): on the synthetic desktop the macroblocks mix B_PRED and 16x16 modes, skipped and
    coded; libwebp and the in-tree decoder both reproduce the reconstruction, and B_PRED saves bits
    at equal or better PSNR."""
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    w, h = 640, 368
    y, uv = bgrx_to_nv12(CpuSyntheticDesktop(w, h, True).render(0, 0, 0))
    out = {}
    for bp, lf in ((0, 0), (1, 0), (1, 1)):
        c = native.EncoderConfig()
        c.width, c.height, c.qp, c.bitrate_kbps, c.deblock, c.vp8_bpred = w, h, qp, 0, lf, bp
        enc = native.CpuVp8Encoder(c)
        frame = enc.encode(y, uv)
        ry, ruv = enc.recon()
        dec = Decoder()
        dec.decode([frame])
        assert np.array_equal(dec.frames_coded[0][0], ry) and np.array_equal(dec.frames_coded[0][1], ruv[:, 0::2])
        rgb = np.asarray(Image.open(io.BytesIO(webp_container(frame))).convert("RGB")).astype(np.int64)
        ref = libwebp_rgb(ry[:h, :w].astype(np.int64), ruv[:h // 2, 0:w:2].astype(np.int64),
                          ruv[:h // 2, 1:w:2].astype(np.int64))
        assert np.array_equal(rgb, ref), int((rgb != ref).any(axis=2).sum())
        mse = float(np.mean((ry[:h, :w].astype(float) - y) ** 2))
        out[(bp, lf)] = (len(frame), 10 * np.log10(255 ** 2 / max(mse, 1e-9)), dec.stats.get("bpred", 0),
                         dec.stats.get("skip", 0))
    nb = out[(1, 0)][2]
    assert 0 < nb < (w // 16) * (h // 16) and out[(0, 0)][2] == 0, out
    assert out[(1, 0)][0] < out[(0, 0)][0] and out[(1, 0)][1] > out[(0, 0)][1] - 0.05, out


@pytest.mark.parametrize("qp,lf", [(24, 0), (34, 1), (44, 1)])
def test_intra_macroblocks_in_inter_frames(native, qp, lf):
    """Intra macroblocks in inter frames (vp8_core.h vp8_intra_candidate: the two parallel passes
    after the inter coding -- candidates from the inter reconstruction, then the candidates without
    a candidate causal neighbour): the in-tree decoder parses them (is_inter_mb 0, the inter-frame
    mode trees, intra prediction from the frame being decoded) and reproduces the reconstruction,
    with the loop filter too; vp8_intra = 0 codes none."""
    w, h = 320, 192
    counts = {}
    for vi in (0, 1):
        c = native.EncoderConfig()
        c.width, c.height, c.qp, c.bitrate_kbps, c.deblock, c.vp8_intra = w, h, qp, 0, lf, vi
        enc = native.CpuVp8Encoder(c)
        frames, recs = [], []
        for t in range(5):
            y, uv = synthetic_nv12(w, h, t, seed=t % 3)
            frames.append(enc.encode(y, uv))
            recs.append(tuple(a.copy() for a in enc.recon()))
        dec = Decoder()
        dec.decode(frames)
        for t, ((yy, u, v), (ry, ruv)) in enumerate(zip(dec.frames_coded, recs)):
            assert np.array_equal(yy, ry), f"frame {t} luma"
            assert np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2]), f"frame {t} chroma"
        counts[vi] = dec.stats.get("intra_p", 0)
    assert counts[0] == 0 and counts[1] > 0, counts
