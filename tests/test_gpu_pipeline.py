"""GPU tests (MI355X): HIP pixel kernels vs float references, the HIP H.264 encoder vs
the CPU encoder (bit-exact) and vs the independent decoder, and the session pipeline."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from mxdesk.codec.h264_decoder import Decoder, psnr  # noqa: E402

from .gpu_util import bt709_nv12_reference, pitched, to_dev  # noqa: E402
from .test_cpu_encoder import synthetic_nv12  # noqa: E402


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_csc_matches_float_reference(gpu):
    rng = np.random.default_rng(0)
    h, w = 68, 120
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    img[..., 3] = 255
    pitch_in = w * 4 + 64
    src = np.zeros((h, pitch_in), np.uint8)
    src[:, : w * 4] = img.reshape(h, w * 4)
    d_in = to_dev(src)
    cw, ch, op = 128, 80, 128
    y = torch.zeros((ch, op), dtype=torch.uint8, device="cuda")
    uv = torch.zeros((ch // 2, op), dtype=torch.uint8, device="cuda")
    gpu.bgrx_to_nv12(d_in.data_ptr(), pitch_in, w, h, y.data_ptr(), uv.data_ptr(), op, cw, ch, _stream())
    torch.cuda.synchronize()
    ry, ru, rv = bt709_nv12_reference(img)
    Y = y.cpu().numpy()
    UV = uv.cpu().numpy()
    assert np.abs(Y[:h, :w].astype(np.float64) - ry).max() <= 1.0
    assert np.abs(UV[: h // 2, 0:w:2].astype(np.float64) - ru).max() <= 1.5
    assert np.abs(UV[: h // 2, 1:w:2].astype(np.float64) - rv).max() <= 1.5
    # padding replicates the last column / row
    assert np.array_equal(Y[:h, w:cw], np.repeat(Y[:h, w - 1: w], cw - w, axis=1))
    assert np.array_equal(Y[h:ch, :], np.repeat(Y[h - 1: h, :], ch - h, axis=0))


def _lanczos_ref(img, xs, wx, ys, wy):
    h, w = img.shape[:2]
    f = img[..., :3].astype(np.float64)
    tx, ty = wx.shape[1], wy.shape[1]
    cols = np.clip(xs[:, None] + np.arange(tx)[None, :], 0, w - 1)
    hz = np.einsum("hokc,ok->hoc", f[:, cols.reshape(-1)].reshape(h, len(xs), tx, 3), wx)  # noqa
    rows = np.clip(ys[:, None] + np.arange(ty)[None, :], 0, h - 1)
    out = np.einsum("okxc,ok->oxc", hz[rows.reshape(-1)].reshape(len(ys), ty, hz.shape[1], 3), wy)
    return np.clip(np.rint(out), 0, 255)


@pytest.mark.parametrize("mfma,strip", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("src_hw,dst_hw", [((96, 160), (48, 80)), ((64, 96), (96, 128)), ((90, 150), (60, 100)),
                                           ((270, 500), (108, 200)), ((200, 330), (100, 166)), ((540, 960), (270, 480))])
def test_lanczos_scale_matches_reference(gpu, src_hw, dst_hw, mfma, strip):
    rng = np.random.default_rng(1)
    (h, w), (oh, ow) = src_hw, dst_hw
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.zeros((h, w, 4), np.uint8)
    img[..., 0] = (128 + 100 * np.sin(xx / 5.0)).astype(np.uint8)
    img[..., 1] = (128 + 100 * np.cos(yy / 7.0)).astype(np.uint8)
    img[..., 2] = rng.integers(0, 256, (h, w))
    xs, wx, tx = gpu.lanczos_table(w, ow)
    ys, wy, ty = gpu.lanczos_table(h, oh)
    d_in = to_dev(img.reshape(h, w * 4))
    dx, dwx, dy, dwy = to_dev(xs), to_dev(wx), to_dev(ys), to_dev(wy)
    cw, ch = (ow + 15) // 16 * 16, (oh + 15) // 16 * 16
    y = torch.zeros((ch, cw), dtype=torch.uint8, device="cuda")
    uv = torch.zeros((ch // 2, cw), dtype=torch.uint8, device="cuda")
    gpu.scale_to_nv12(d_in.data_ptr(), w * 4, w, h, ow, oh, dx.data_ptr(), dwx.data_ptr(), tx, dy.data_ptr(),
                      dwy.data_ptr(), ty, y.data_ptr(), uv.data_ptr(), cw, cw, ch, _stream(), mfma=mfma, strip=strip)
    torch.cuda.synchronize()
    rgb = _lanczos_ref(img, xs, wx, ys, wy)
    ref_bgrx = np.zeros((oh, ow, 4), np.uint8)
    ref_bgrx[..., :3] = rgb.astype(np.uint8)
    ry, ru, rv = bt709_nv12_reference(ref_bgrx)
    Y = y.cpu().numpy()[:oh, :ow].astype(np.float64)
    assert np.abs(Y - ry).max() <= 1.5
    UV = uv.cpu().numpy().astype(np.float64)
    assert np.abs(UV[: oh // 2, 0:ow:2] - ru).max() <= 2.0
    assert np.abs(UV[: oh // 2, 1:ow:2] - rv).max() <= 2.0
    # coded padding replicates the last column / row
    Yc = y.cpu().numpy()
    assert np.array_equal(Yc[:oh, ow:cw], np.repeat(Yc[:oh, ow - 1: ow], cw - ow, axis=1))
    assert np.array_equal(Yc[oh:ch, :], np.repeat(Yc[oh - 1: oh, :], ch - oh, axis=0))


def test_lanczos_mfma_matches_valu_at_4k_to_1080p(gpu):
    """Production size: the matrix-core scaler against the VALU one on a synthetic 4K desktop."""
    w, h, ow, oh = 3840, 2160, 1920, 1080
    src = torch.zeros((h, w * 4), dtype=torch.uint8, device="cuda")
    gpu.synth(src.data_ptr(), w, h, w * 4, frame_id=7, t=0.25, noise=1, stream=_stream())
    xs, wx, tx = gpu.lanczos_table(w, ow)
    ys, wy, ty = gpu.lanczos_table(h, oh)
    dx, dwx, dy, dwy = to_dev(xs), to_dev(wx), to_dev(ys), to_dev(wy)
    out = {}
    for form in ("valu", "tile", "strip"):
        y = torch.zeros((1088, 1920), dtype=torch.uint8, device="cuda")
        uv = torch.zeros((544, 1920), dtype=torch.uint8, device="cuda")
        gpu.scale_to_nv12(src.data_ptr(), w * 4, w, h, ow, oh, dx.data_ptr(), dwx.data_ptr(), tx, dy.data_ptr(),
                          dwy.data_ptr(), ty, y.data_ptr(), uv.data_ptr(), 1920, 1920, 1088, _stream(),
                          mfma=form != "valu", strip=form == "strip")
        torch.cuda.synchronize()
        out[form] = (y.cpu().numpy().astype(np.int32), uv.cpu().numpy().astype(np.int32))
    for form in ("tile", "strip"):  # both matrix-core forms against the VALU kernel
        dyp = np.abs(out[form][0] - out["valu"][0])
        duv = np.abs(out[form][1] - out["valu"][1])
        assert dyp.max() <= 1 and duv.max() <= 1, (form, dyp.max(), duv.max())
        assert (dyp > 0).mean() < 0.02 and (duv > 0).mean() < 0.02, (form, (dyp > 0).mean(), (duv > 0).mean())


def _read_barcode(y_plane, cell, bx, by):
    vals = []
    for row in range(2):
        v = 0
        for i in range(32):
            cx, cy = bx + i * cell + cell // 2, by + row * cell + cell // 2
            v = (v << 1) | int(y_plane[cy, cx] > 128)
        vals.append(v)
    return vals


def test_synth_deterministic_and_barcode(gpu):
    w, h = 512, 288
    pitch = w * 4
    a = torch.zeros((h, pitch), dtype=torch.uint8, device="cuda")
    b = torch.zeros((h, pitch), dtype=torch.uint8, device="cuda")
    gpu.synth(a.data_ptr(), w, h, pitch, frame_id=1234567, timestamp_us=89012345, t=1.5, stream=_stream())
    gpu.synth(b.data_ptr(), w, h, pitch, frame_id=1234567, timestamp_us=89012345, t=1.5, stream=_stream())
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    img = a.cpu().numpy().reshape(h, w, 4)
    ry, _, _ = bt709_nv12_reference(img)
    fid, ts = _read_barcode(ry, gpu.BARCODE_CELL, gpu.BARCODE_X, gpu.BARCODE_Y)
    assert (fid, ts) == (1234567, 89012345)


def _gpu_cpu_encode(gpu, w, h, frames, **kw):
    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height = w, h
    cfg.bitrate_kbps = 0
    cfg.qp = kw.get("qp", 28)
    cfg.search_range = kw.get("search_range", 8)
    cfg.subpel = kw.get("subpel", 1)
    cfg.intra_in_p = kw.get("intra_in_p", 1)
    cfg.aq = kw.get("aq", 1)
    cfg.me_coarse = kw.get("me_coarse", 1)
    cfg.intra4x4 = kw.get("intra4x4", 1)
    cfg.deblock = kw.get("deblock", 0)
    genc = gpu.GpuH264Encoder(cfg, _stream())
    cenc = gpu.CpuH264Encoder(cfg)
    gs, cs, grec = b"", b"", []
    ch = genc.coded_height
    for t in range(frames):
        y, uv = synthetic_nv12(w, h, t, seed=t if kw.get("fresh_noise") else 0)
        dy = pitched(y, genc.pitch, ch)
        duv = pitched(uv, genc.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
        cau = cenc.encode(y, uv, False)
        gs += gau
        cs += cau
        grec.append(genc.recon())
        assert bool(gau == cau), f"frame {t}: GPU bitstream differs from CPU encoder ({len(gau)} vs {len(cau)} bytes)"
    return gs, grec


@pytest.mark.parametrize("w,h,aq", [(320, 192, 3), (320, 192, 4), (640, 368, 6)])
def test_gpu_temporal_classes_desktop_bit_exact_vs_cpu(gpu, w, h, aq):
    """H.264 temporal AQ classes on the synthetic desktop (noise panel changing, static windows:
    with aq >= 4 the static class -- identical source, zero vector -- refines 9+ QP finer): the GPU
    stream equals the CPU encoder's bit for bit and decodes to the GPU reconstruction."""
    from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height = w, h
    cfg.bitrate_kbps, cfg.qp, cfg.aq = 0, 30, aq
    genc = gpu.GpuH264Encoder(cfg, _stream())
    cenc = gpu.CpuH264Encoder(cfg)
    desk = CpuSyntheticDesktop(w, h, True)
    ch = genc.coded_height
    gs, grec, qps = b"", [], set()
    for t in range(5):
        y, uv = bgrx_to_nv12(desk.render(t, t / 60, 0))
        dy = pitched(y, genc.pitch, ch)
        duv = pitched(uv, genc.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
        cau = cenc.encode(y, uv, False)
        assert bool(gau == cau), f"aq {aq} frame {t}: GPU bitstream differs from CPU encoder ({len(gau)} vs {len(cau)} bytes)"
        gs += gau
        grec.append(genc.recon())
    dec = Decoder()
    dec.decode(gs)
    for (yy, _, _), (ry, _) in zip(dec.frames_coded, grec):
        assert np.array_equal(yy, ry)


@pytest.mark.parametrize("w,h,subpel,sr,fresh,db", [(64, 48, 1, 8, 0, 1), (160, 96, 0, 16, 0, 0),
                                                    (100, 60, 1, 16, 0, 1), (320, 192, 1, 32, 0, 1),
                                                    (96, 64, 1, 8, 1, 1), (80, 48, 1, 8, 1, 0),
                                                    (48, 48, 0, 8, 1, 1), (576, 64, 1, 8, 1, 1)])
def test_gpu_encoder_bit_exact_vs_cpu(gpu, w, h, subpel, sr, fresh, db):
    # fresh=1: new noise every frame -> adaptive quantisation (mb_qp_delta != 0) is exercised;
    # db=1: in-loop deblocking (k_deblock) on
    stream, grec = _gpu_cpu_encode(gpu, w, h, 4, subpel=subpel, search_range=sr, fresh_noise=fresh, qp=24,
                                   deblock=db)
    dec = Decoder()
    dec.decode(stream)
    for (y, u, v), (ry, ruv) in zip(dec.frames_coded, grec):
        assert np.array_equal(y, ry)
        assert np.array_equal(u, ruv[:, 0::2])


@pytest.mark.parametrize("me_coarse,sr", [(0, 16), (1, 16), (1, 32)])
def test_gpu_me_modes_bit_exact_vs_cpu(gpu, me_coarse, sr):
    """Exhaustive and coarse-grid (even offsets + integer neighbours) motion search: GPU ==
    CPU oracle, decodes to the reconstruction."""
    stream, grec = _gpu_cpu_encode(gpu, 160, 96, 4, search_range=sr, fresh_noise=0, qp=26, me_coarse=me_coarse)
    dec = Decoder()
    dec.decode(stream)
    for (y, u, v), (ry, ruv) in zip(dec.frames_coded, grec):
        assert np.array_equal(y, ry)


def test_gpu_intra16x16_only_bit_exact_vs_cpu(gpu):
    """intra4x4=0 (the fast-IDR setting): GPU == CPU oracle, decodes to the reconstruction."""
    stream, grec = _gpu_cpu_encode(gpu, 160, 96, 3, fresh_noise=1, qp=28, intra4x4=0)
    dec = Decoder()
    dec.decode(stream)
    for (y, u, v), (ry, ruv) in zip(dec.frames_coded, grec):
        assert np.array_equal(y, ry)


@pytest.mark.parametrize("qp", [30, 44])
def test_gpu_residual_drop_bit_exact_vs_cpu(gpu, qp):
    """aq=2: noise-like MBs keep their residual only when it pays at lambda(QP); GPU == CPU
    bitstream and the decoder reproduces the reconstruction."""
    stream, grec = _gpu_cpu_encode(gpu, 160, 96, 4, fresh_noise=1, qp=qp, aq=2)
    dec = Decoder()
    dec.decode(stream)
    for (y, u, v), (ry, ruv) in zip(dec.frames_coded, grec):
        assert np.array_equal(y, ry)
        assert np.array_equal(u, ruv[:, 0::2]) and np.array_equal(v, ruv[:, 1::2])


def test_session_stream_decodes_with_barcodes(gpu):
    cfg = gpu.SessionConfig()
    cfg.width, cfg.height, cfg.fps = 320, 192, 60
    cfg.enc.bitrate_kbps = 0
    cfg.enc.qp = 24
    s = gpu.Session(cfg)
    stream = b""
    ids = []
    for _ in range(4):
        r = s.step(False)
        stream += r.au
        ids.append((r.frame_id, r.t_capture_us))
        assert r.t_encoded_us >= r.t_capture_us
    dec = Decoder()
    frames = dec.decode(stream)
    assert len(frames) == 4
    for (y, _, _), (fid, ts) in zip(frames, ids):
        got = _read_barcode(y, gpu.BARCODE_CELL, gpu.BARCODE_X, gpu.BARCODE_Y)
        assert got[0] == fid


def test_session_scaled_output(gpu):
    cfg = gpu.SessionConfig()
    cfg.width, cfg.height = 640, 384
    cfg.out_width, cfg.out_height = 320, 192
    cfg.enc.bitrate_kbps = 0
    s = gpu.Session(cfg)
    stream = b"".join(s.step(False).au for _ in range(2))
    frames = Decoder().decode(stream)
    assert frames[0][0].shape == (192, 320)


@pytest.mark.parametrize("intra_in_p", [0, 1])
def test_session_masked_psnr_from_encoder(gpu, intra_in_p):
    """The H.264 encoder's 4th distortion channel (luma outside the macroblocks touching the
    mask rectangle) equals the PSNR of the decoded picture over those samples (IDR wavefront,
    inter and intra-in-P paths)."""
    cfg = gpu.SessionConfig()
    cfg.width, cfg.height, cfg.fps = 200, 120, 60
    cfg.enc.bitrate_kbps = 0
    cfg.enc.qp = 30
    cfg.enc.intra_in_p = intra_in_p
    cfg.mask_x0, cfg.mask_y0, cfg.mask_x1, cfg.mask_y1 = 20, 40, 90, 75  # -> MBs x 1..5, y 2..4
    s = gpu.Session(cfg)
    stream, res, srcs = b"", [], []
    for _ in range(4):
        r = s.step(False)
        stream += r.au
        res.append(r)
        srcs.append(s.nv12()[0][:120, :200].astype(np.float64))
    frames = Decoder().decode(stream)
    keep = np.ones((120, 200), bool)
    keep[32:80, 16:96] = False
    for (dy, _, _), sy, r in zip(frames, srcs, res):
        mse = np.mean(((dy.astype(np.float64) - sy) ** 2)[keep])
        want = 99.0 if mse == 0 else min(99.0, 10 * np.log10(255.0 ** 2 / mse))
        assert abs(want - r.psnr_y_masked) < 1e-6, (want, r.psnr_y_masked)


def test_session_reports_psnr_of_reconstruction(gpu):
    """Encoder-side SSE (k_inter_encode / k_intra_rows -> k_scan) equals the PSNR of the
    independently decoded picture against the source, over the display area only."""
    cfg = gpu.SessionConfig()
    cfg.width, cfg.height, cfg.fps = 200, 120, 60  # coded 208x128: padding must be excluded
    cfg.enc.bitrate_kbps = 0
    cfg.enc.qp = 30
    s = gpu.Session(cfg)
    stream, res, srcs = b"", [], []
    for _ in range(3):
        r = s.step(False)
        stream += r.au
        res.append(r)
        y, uv = s.nv12()
        srcs.append((y[:120, :200].astype(np.float64), uv[:60, :200].astype(np.float64)))
    frames = Decoder().decode(stream)

    def psnr(a, b):
        mse = np.mean((a - b) ** 2)
        return 99.0 if mse == 0 else min(99.0, 10 * np.log10(255.0 ** 2 / mse))

    for (dy, du, dv), (sy, suv), r in zip(frames, srcs, res):
        assert abs(psnr(dy.astype(np.float64), sy) - r.psnr_y) < 1e-6
        assert abs(psnr(du.astype(np.float64), suv[:, 0::2]) - r.psnr_u) < 1e-6
        assert abs(psnr(dv.astype(np.float64), suv[:, 1::2]) - r.psnr_v) < 1e-6
        assert 25 < r.psnr_y < 99


def test_graph_replay_matches_stream_launches(gpu):
    """hipGraph replay of the per-frame chain (synth -> CSC -> encoder) produces the same
    bitstream as eager launches, across P frames, a forced IDR and all pool slots."""
    def run(use_graph):
        cfg = gpu.SessionConfig()
        cfg.width, cfg.height, cfg.fps = 320, 192, 60
        cfg.enc.bitrate_kbps = 500  # rate control active: QP changes between frames
        cfg.use_graph = use_graph
        cfg.enc.deblock = 0  # graph replay needs a fixed H.264 filter (Session: adaptive -> off); eager alike
        cfg.fake_clock = 1
        s = gpu.Session(cfg)
        aus = [s.step(i == 5).au for i in range(9)]
        return aus, s.graphs_built

    eager, g0 = run(0)
    graph, g1 = run(1)
    assert g0 == 0 and 3 <= g1 <= 6
    for i, (a, b) in enumerate(zip(eager, graph)):
        assert a == b, f"frame {i} differs"
    assert len(Decoder().decode(b"".join(graph))) == 9


def _run_pipelined(gpu, depth, kbps, n=8, codec="h264", idr_at=5, use_graph=0):
    """n frames with up to `depth` in flight (submit ahead, then collect / submit), a forced IDR
    at frame idr_at."""
    cfg = gpu.SessionConfig()
    cfg.width, cfg.height, cfg.fps = 320, 192, 60
    cfg.codec = codec
    cfg.enc.bitrate_kbps = kbps
    cfg.enc.pipeline_depth = depth
    cfg.use_graph = use_graph
    if codec == "h264":  # graph replay needs a fixed H.264 filter (Session: adaptive -> off)
        cfg.enc.deblock = 0
    cfg.fake_clock = 1
    s = gpu.Session(cfg)
    out, sent = [], 0
    while sent < min(depth, n):
        s.submit(sent == idr_at)
        sent += 1
    for _ in range(n):
        out.append(s.collect())
        if sent < n:
            s.submit(sent == idr_at)
            sent += 1
    assert s.in_flight == 0
    return out, s.graphs_built


@pytest.mark.parametrize("depth", [2, 3])
def test_pipelined_depth_matches_depth1(gpu, depth):
    """Two / three frames in flight (entropy of frame n on a second stream, overlapping analysis
    of n+1; with three the next frame's launches queue while the host collects): constant-QP
    output is bit-identical to depth 1; with CBR the stream still decodes and frame ids / capture
    times come back in submission order."""
    a, b = _run_pipelined(gpu, 1, 0)[0], _run_pipelined(gpu, depth, 0)[0]
    assert [r.au for r in a] == [r.au for r in b]
    assert [r.frame_id for r in b] == list(range(8)) and [r.idr for r in b][5] == 1
    c = _run_pipelined(gpu, depth, 600)[0]
    frames = Decoder().decode(b"".join(r.au for r in c))
    ids = [_read_barcode(y, gpu.BARCODE_CELL, gpu.BARCODE_X, gpu.BARCODE_Y)[0] for y, _, _ in frames]
    assert ids == list(range(8))
    assert all(r2.t_capture_us >= r1.t_capture_us for r1, r2 in zip(c, c[1:]))


def _hpel_reference(ref, pad=48):
    """numpy 6-tap half-sample planes of a clamped reference (8.4.2.2.1), padded by `pad`."""
    h, w = ref.shape
    ys = np.clip(np.arange(-pad - 2, h + pad + 3), 0, h - 1)
    xs = np.clip(np.arange(-pad - 2, w + pad + 3), 0, w - 1)
    e = ref[np.ix_(ys, xs)].astype(np.int64)  # extended by pad+2 / pad+3
    H, W = h + 2 * pad, w + 2 * pad
    t = lambda a, b, c, d, e_, f: a - 5 * b + 20 * c + 20 * d - 5 * e_ + f
    F = e[2:2 + H, 2:2 + W]
    b1 = t(*(e[:, k:k + W] for k in range(6)))  # rows of e, horizontal taps -> (H+5, W)
    Hh = np.clip((b1[2:2 + H] + 16) >> 5, 0, 255)
    v1 = t(*(e[k:k + H, 2:2 + W] for k in range(6)))
    V = np.clip((v1 + 16) >> 5, 0, 255)
    j1 = t(*(b1[k:k + H] for k in range(6)))
    J = np.clip((j1 + 512) >> 10, 0, 255)
    return [p.astype(np.uint8) for p in (F, Hh, V, J)]


@pytest.mark.parametrize("w,h", [(64, 48), (160, 96), (112, 64), (416, 240)])  # 416x240: interior tiles
def test_hpel_planes_match_reference(gpu, w, h):
    rng = np.random.default_rng(w + h)
    ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
    pitch = (w + 255) // 256 * 256
    buf = np.zeros((h, pitch), np.uint8)
    buf[:, :w] = ref
    planes = gpu.h264.hpel_planes(buf, w)
    want = _hpel_reference(ref)
    for name, got, exp in zip("FHVJ", planes, want):
        g = got[: exp.shape[0], : exp.shape[1]]
        bad = np.argwhere(g != exp)
        assert bad.size == 0, f"plane {name}: {len(bad)} mismatches, first at {bad[:3].tolist()}"


def test_synth_static_cache_matches_full_render(gpu):
    """k_synth with the static-layer cache == the full per-pixel render, at several animation
    times (moving window, cursor) and sizes."""
    for w, h in [(512, 288), (1920, 1080)]:
        pitch = w * 4
        bg = torch.zeros((h, pitch), dtype=torch.uint8, device="cuda")
        gpu.synth_static(bg.data_ptr(), w, h, pitch, _stream())
        for t in (0.0, 0.37, 1.9, 7.25):
            a = torch.zeros((h, pitch), dtype=torch.uint8, device="cuda")
            b = torch.zeros((h, pitch), dtype=torch.uint8, device="cuda")
            gpu.synth(a.data_ptr(), w, h, pitch, frame_id=5, timestamp_us=7, t=t, stream=_stream())
            gpu.synth(b.data_ptr(), w, h, pitch, frame_id=5, timestamp_us=7, t=t, stream=_stream(),
                      static_bg=bg.data_ptr())
            torch.cuda.synchronize()
            assert torch.equal(a, b), (w, h, t)


def test_zero_copy_registered_capture_matches_staged_upload(gpu):
    """A frame inside a registered (page-locked) host buffer -- the XShm segment in production --
    is DMA'd straight to the GPU; the access units equal the staged-copy path's."""
    w, h, pitch = 320, 192, 320 * 4 + 256  # padded rows like an XImage
    rng = np.random.default_rng(3)
    frames = [rng.integers(0, 256, (h, pitch), dtype=np.uint8) for _ in range(3)]

    def session():
        cfg = gpu.SessionConfig()
        cfg.width, cfg.height, cfg.fps = w, h, 60
        cfg.enc.bitrate_kbps = 0
        cfg.enc.qp = 26
        return gpu.Session(cfg)

    staged, zc = session(), session()
    buf = np.zeros((h, pitch), np.uint8)  # the "capture segment", registered once
    zc.register_host_buffer(buf.ctypes.data, buf.nbytes)
    for f in frames:
        staged.submit_bgrx(np.ascontiguousarray(f[:, : w * 4]).reshape(h, w, 4), False)
        a = staged.collect().au
        buf[:] = f
        zc.submit_bgrx_ptr(buf.ctypes.data, pitch, buf.nbytes, False)
        buf[:] = 0  # the DMA has read the frame when submit returns
        b = zc.collect().au
        assert a == b
    # a span that does not fit the declared buffer is refused before any copy (no overread)
    with pytest.raises(ValueError):
        zc.submit_bgrx_ptr(buf.ctypes.data, pitch, pitch * (h - 1) + w * 4 - 1, False)


@pytest.mark.parametrize("registered", [True, False])
def test_damage_driven_capture_matches_full_upload(gpu, registered):
    """Damage-driven capture (XDamage bands -> Session.submit_bgrx_damage): only the changed
    row bands are read from host memory into the session's device-resident screen.  Rows
    outside the bands are zeroed in the host buffer to prove they are never read; the access
    units equal a session fed every whole frame."""
    w, h, pitch = 320, 192, 320 * 4 + 256
    rng = np.random.default_rng(11)
    f0 = rng.integers(0, 256, (h, pitch), dtype=np.uint8)
    f1 = f0.copy()
    f1[48:96] = rng.integers(0, 256, (48, pitch), dtype=np.uint8)
    f2 = f1.copy()
    f2[0:16] = 7
    f2[160:176] = 200
    # (frame, damage bands): whole first frame, one band, nothing changed, two bands
    seq = [(f0, [(0, h)]), (f1, [(48, 96)]), (f1, []), (f2, [(0, 16), (160, 176)])]

    def session():
        cfg = gpu.SessionConfig()
        cfg.width, cfg.height, cfg.fps = w, h, 60
        cfg.enc.bitrate_kbps = 0
        cfg.enc.qp = 26
        return gpu.Session(cfg)

    full, dmg = session(), session()
    buf = np.zeros((h, pitch), np.uint8)
    if registered:
        dmg.register_host_buffer(buf.ctypes.data, buf.nbytes)
    for i, (f, bands) in enumerate(seq):
        full.submit_bgrx(np.ascontiguousarray(f[:, : w * 4]).reshape(h, w, 4), False)
        a = full.collect().au
        buf[:] = 0
        for y0, y1 in bands:
            buf[y0:y1] = f[y0:y1]
        dmg.submit_bgrx_damage(buf.ctypes.data, pitch, buf.nbytes, bands, False)
        b = dmg.collect().au
        assert a == b, f"frame {i}"
    assert dmg.damage_bytes_uploaded == w * 4 * (h + 48 + 32)
    # after invalidate_screen the next submit reads the whole frame again
    dmg.invalidate_screen()
    buf[:] = f2
    dmg.submit_bgrx_damage(buf.ctypes.data, pitch, buf.nbytes, [], False)
    dmg.collect()
    assert dmg.damage_bytes_uploaded == w * 4 * (2 * h + 48 + 32)
    with pytest.raises(ValueError):
        dmg.submit_bgrx_damage(buf.ctypes.data, pitch, buf.nbytes, [(0, h + 16)], False)
    with pytest.raises(ValueError):
        dmg.submit_bgrx_damage(buf.ctypes.data, pitch, pitch * (h - 1), [], False)


@pytest.mark.parametrize("codec", ["h264", "hevc"])
def test_depth3_hevc_h264_match_depth1(gpu, codec):
    """Three frames in flight == one, constant QP, both codecs (eager and graph replay)."""
    a = _run_pipelined(gpu, 1, 0, n=10, codec=codec)[0]
    b = _run_pipelined(gpu, 3, 0, n=10, codec=codec)[0]
    g, built = _run_pipelined(gpu, 3, 0, n=10, codec=codec, use_graph=1)
    assert built >= 4
    for i, (x, y, z) in enumerate(zip(a, b, g)):
        assert x.au == y.au == z.au, f"frame {i} differs"


def test_hevc_graph_depth1_idr_same_key_matches_eager(gpu):
    """HEVC, one frame in flight, temporal AQ: forced IDRs at frames 3 and 6 (frame 0, the CBR
    probe frame, runs eagerly) reuse the same graph key (pool slot 0 of 3, encoder slot) with the
    reconstruction / source buffers swapped; the IDR's source copy
    must follow the frame (read on the device), or the next P picture's temporal classes compare
    against a stale source and the graph output diverges from eager launches."""
    def run(use_graph):
        cfg = gpu.SessionConfig()
        cfg.width, cfg.height, cfg.fps = 320, 192, 60
        cfg.codec = "hevc"
        cfg.enc.bitrate_kbps = 600
        cfg.enc.aq = 3
        cfg.pool_slots = 3
        cfg.use_graph = use_graph
        cfg.fake_clock = 1
        s = gpu.Session(cfg)
        return [s.step(i in (3, 6)).au for i in range(9)], s.graphs_built

    eager, _ = run(0)
    graph, built = run(1)
    assert built >= 2
    for i, (a, b) in enumerate(zip(eager, graph)):
        assert a == b, f"frame {i} differs"


@pytest.mark.parametrize("codec", ["h264", "hevc"])
def test_graph_replay_depth2_matches_eager(gpu, codec):
    """Two frames in flight with the per-frame chain replayed as two hipGraphs (analysis on the
    session stream, entropy on the encoder's entropy stream, linked by an event per frame):
    bit-identical to eager launches under CBR, across every (frame slot, encoder slot) pair and
    a forced IDR."""
    def run(use_graph, n=12):
        cfg = gpu.SessionConfig()
        cfg.width, cfg.height, cfg.fps = 320, 192, 60
        cfg.codec = codec
        cfg.enc.bitrate_kbps = 600
        cfg.enc.pipeline_depth = 2
        cfg.use_graph = use_graph
        if codec == "h264":  # graph replay needs a fixed H.264 filter (Session: adaptive -> off)
            cfg.enc.deblock = 0
        cfg.fake_clock = 1
        s = gpu.Session(cfg)
        out = []
        s.submit(False)
        for i in range(n):
            if i + 1 < n:
                s.submit(i + 1 == 7)
            out.append(s.collect())
        assert s.in_flight == 0
        return [r.au for r in out], s.graphs_built

    eager, g0 = run(0)
    graph, g1 = run(1)
    assert g0 == 0 and g1 >= 4
    for i, (a, b) in enumerate(zip(eager, graph)):
        assert a == b, f"frame {i} differs"


def test_session_hevc_masked_psnr_from_encoder(gpu):
    """HEVC with SAO: k_hevc_sao's 4th distortion channel (luma of the CTBs outside the mask
    rectangle, the same 16-aligned region as H.264's) equals the PSNR of the decoded picture
    over those samples, IDR and P pictures; no separate masked-SSE pass runs."""
    from mxdesk.codec.hevc_decoder import Decoder as HevcDecoder

    cfg = gpu.SessionConfig()
    cfg.width, cfg.height, cfg.fps = 200, 120, 60
    cfg.codec = "hevc"
    cfg.enc.bitrate_kbps = 0
    cfg.enc.qp = 30
    cfg.mask_x0, cfg.mask_y0, cfg.mask_x1, cfg.mask_y1 = 20, 40, 90, 75  # -> CTBs x 1..5, y 2..4
    s = gpu.Session(cfg)
    stream, res, srcs = b"", [], []
    for _ in range(4):
        r = s.step(False)
        stream += r.au
        res.append(r)
        srcs.append(s.nv12()[0][:120, :200].astype(np.float64))
    frames = HevcDecoder().decode(stream)
    assert len(frames) == 4
    keep = np.ones((120, 200), bool)
    keep[32:80, 16:96] = False
    for (dy, _, _), sy, r in zip(frames, srcs, res):
        mse = np.mean(((dy[:120, :200].astype(np.float64) - sy) ** 2)[keep])
        want = 99.0 if mse == 0 else min(99.0, 10 * np.log10(255.0 ** 2 / mse))
        assert abs(want - r.psnr_y_masked) < 1e-6, (want, r.psnr_y_masked)


@pytest.mark.parametrize("depth", [1, 3])
def test_device_clock_frame_times(gpu, depth):
    """H.264 frames carry device wall-clock stamps (render start, encoder first kernel, end of
    k_pack) instead of timing events: every frame reports a positive GPU time, the encoder's own
    share is no larger than the whole frame's, and both stay below the frame's host latency."""
    out = _run_pipelined(gpu, depth, 600, n=10)[0]
    for r in out:
        host_ms = (r.t_encoded_us - r.t_capture_us) / 1000.0
        assert 0.0 < r.gpu_ms < host_ms + 0.5, (r.frame_id, r.gpu_ms, host_ms)
    cfg = gpu.SessionConfig()
    cfg.width, cfg.height = 320, 192
    s = gpu.Session(cfg)
    for _ in range(3):
        r = s.step(False)
        assert 0.0 < s.stats.encode_ms <= r.gpu_ms + 1e-6


def _adaptive_frames():
    from .test_deblock import _pan_frames

    w, h = 192, 96
    frames = [(y, uv, t == 6) for t, (y, uv) in enumerate(_pan_frames(w, h, 10))]
    frames += [(y, uv, False) for y, uv in _pan_frames(w, h, 6, still=True)]
    return w, h, frames


@pytest.mark.parametrize("depth", [1, 3])
def test_gpu_adaptive_deblock_bit_exact_vs_cpu(gpu, depth):
    """deblock=2: the class counts k_scan_rows reports and the host's fixed-lag decision (picture n
    from picture n - kDbLag) equal the CPU encoder's, so the streams match bit for bit through a
    pan, a forced IDR and a still stretch (synchronous encode() at depth 1 and 3)."""
    w, h, frames = _adaptive_frames()
    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height = w, h
    cfg.bitrate_kbps, cfg.qp, cfg.search_range, cfg.deblock = 0, 34, 8, 2
    cfg.pipeline_depth = depth
    genc = gpu.GpuH264Encoder(cfg, _stream())
    cenc = gpu.CpuH264Encoder(cfg)
    ch = genc.coded_height
    flags = []
    for t, (y, uv, idr) in enumerate(frames):
        dy = pitched(y, genc.pitch, ch)
        duv = pitched(uv, genc.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), idr)
        cau = cenc.encode(y, uv, idr)
        assert bool(gau == cau), f"frame {t}: GPU bitstream differs from CPU encoder"
        gst, cst = genc.stats, cenc.stats
        assert (gst.deblocked, gst.db_coherent, gst.db_changed, gst.db_moving) == \
            (cst.deblocked, cst.db_coherent, cst.db_changed, cst.db_moving), t
        assert np.array_equal(genc.recon()[0], cenc.recon()[0]), t
        flags.append(genc.stats.deblocked)
    assert flags[:5] == [0] * 5 and flags[5:10] == [1] * 5 and flags[-1] == 0, flags


@pytest.mark.parametrize("depth", [3, 4])
def test_gpu_adaptive_deblock_in_flight_vs_cpu(gpu, depth):
    """ADVICE r5 h264_encoder.cpp:696: with `depth` frames really in flight (submit ahead, collect
    behind) the adaptive decision of every picture is still the CPU oracle's -- it comes from
    picture n - kDbLag, whose classes the host always holds when picture n is prepared."""
    w, h, frames = _adaptive_frames()
    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height = w, h
    cfg.bitrate_kbps, cfg.qp, cfg.search_range, cfg.deblock = 0, 34, 8, 2
    cfg.pipeline_depth = depth
    genc = gpu.GpuH264Encoder(cfg, _stream())
    cenc = gpu.CpuH264Encoder(cfg)
    ch = genc.coded_height
    want, flags_c = [], []
    for y, uv, idr in frames:
        want.append(cenc.encode(y, uv, idr))
        flags_c.append(cenc.stats.deblocked)
    keep, got, flags = [], [], []
    for t, (y, uv, idr) in enumerate(frames):
        if len(keep) - len(got) == depth:  # pipeline full: collect the oldest frame first
            got.append(genc.collect())
            flags.append(genc.stats.deblocked)
        dy = pitched(y, genc.pitch, ch)
        duv = pitched(uv, genc.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        keep.append((dy, duv))
        genc.submit(dy.data_ptr(), duv.data_ptr(), idr)
    while len(got) < len(frames):
        got.append(genc.collect())
        flags.append(genc.stats.deblocked)
    for t, (g, c) in enumerate(zip(got, want)):
        assert g == c, f"frame {t}: GPU bitstream (depth {depth}, in flight) differs from CPU encoder"
    assert flags == flags_c and 1 in flags and flags[-1] == 0, (flags, flags_c)


@pytest.mark.parametrize("w,h,qp", [(320, 192, 40), (352, 288, 46), (1920, 1088, 44)])
def test_gpu_deblock_strong_filtering_bit_exact_vs_cpu(gpu, w, h, qp):
    """The edge-parallel k_deblock (all four edges of a direction settled in 1-3 passes) against the
    CPU's serial 8.7 order at high QP (large alpha / beta / tC0: most edges filter, bS 4 strong
    filters on the IDR and on intra macroblocks of P pictures): GPU == CPU, decoded == recon."""
    from .test_deblock import _pan_frames

    cfg = gpu.EncoderConfig()
    cfg.width, cfg.height = w, h
    cfg.bitrate_kbps, cfg.qp, cfg.search_range, cfg.deblock, cfg.intra_in_p = 0, qp, 8, 1, 1
    genc = gpu.GpuH264Encoder(cfg, _stream())
    cenc = gpu.CpuH264Encoder(cfg)
    ch = genc.coded_height
    stream, grec = b"", []
    for t, (y, uv) in enumerate(_pan_frames(w, h, 4)):
        if t == 2:
            y = y.copy()
            y[16:64, 32:96] = 255 - y[16:64, 32:96]  # new content: intra macroblocks in a P picture
        dy = pitched(y, genc.pitch, ch)
        duv = pitched(uv, genc.pitch, ch // 2, uv=True)
        torch.cuda.synchronize()
        gau = genc.encode(dy.data_ptr(), duv.data_ptr(), False)
        cau = cenc.encode(y, uv, False)
        assert bool(gau == cau), f"frame {t}"
        assert np.array_equal(genc.recon()[0], cenc.recon()[0]) and np.array_equal(genc.recon()[1], cenc.recon()[1])
        stream += gau
        grec.append(genc.recon())
    if w * h <= 352 * 288:
        dec = Decoder()
        dec.decode(stream)
        for (yy, u, v), (ry, ruv) in zip(dec.frames_coded, grec):
            assert np.array_equal(yy, ry[:h, :w]) and np.array_equal(u, ruv[:h // 2, 0:w:2])
