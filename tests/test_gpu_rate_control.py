"""CBR on the production path: a 1920x1080@60 GPU session at the headline 8 Mbps must hold
its budget from the start (the driver's 5-warm-up / 20-step window) and recover within 10
frames after a forced IDR (viewer join / PLI).  Reference: nvh264enc low-latency CBR
(reference Dockerfile:210)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _session(gpu, codec="h264", w=1920, h=1080, kbps=8000, depth=2):
    cfg = gpu.SessionConfig()
    cfg.width, cfg.height, cfg.fps = w, h, 60
    cfg.enc.bitrate_kbps = kbps
    cfg.enc.pipeline_depth = depth
    cfg.codec = codec
    cfg.fake_clock = 1
    return gpu.Session(cfg)


def _run(s, n, idr_at=()):
    bits, qps, idr = [], [], []
    s.submit(False)
    for i in range(n):
        if i + 1 < n:
            s.submit(i + 1 in idr_at)
        r = s.collect()
        bits.append(len(r.au) * 8)
        qps.append(r.qp)
        idr.append(r.idr)
    return np.array(bits, float), np.array(qps, float), idr


def test_gpu_cbr_1080p_on_budget_and_recovers_after_idr(gpu):
    s = _session(gpu)
    bits, qps, idr = _run(s, 60, idr_at=(30,))
    T = 8000e3 / 60
    assert idr[0] == 1 and idr[30] == 1 and sum(idr) == 2
    assert bits[0] < 7 * T and bits[30] < 7 * T, (bits[0] / T, bits[30] / T)  # IDR budget: 5 frames
    window = bits[5:25]  # the driver's --warmup 5 --steps 20 window
    assert abs(window.mean() / T - 1) < 0.10, window.mean() / T
    # per-10-frame windows: on budget before the IDR and again 10 frames after it
    for a in (10, 20, 40, 50):
        assert abs(bits[a:a + 10].mean() / T - 1) < 0.15, (a, bits[a:a + 10].mean() / T)
    assert abs(qps[45:55].mean() - qps[20:30].mean()) <= 2.0, qps  # QP back 15 frames after the IDR


def test_gpu_cbr_hevc_4k_on_budget(gpu):
    s = _session(gpu, "hevc", 3840, 2160, 25000)
    bits, qps, _ = _run(s, 25)
    T = 25000e3 / 60
    assert bits[0] < 7 * T
    assert abs(bits[5:].mean() / T - 1) < 0.10, bits[5:].mean() / T


def test_gpu_cbr_desktop_keyframes_pinned(gpu):
    """The loosened bounds above cover any content; on the bench desktop itself the intended
    behaviour is tighter and pinned here: every IDR (first picture and a forced one) within 5.5
    frame budgets -- its send time on the wire stays about 90 ms at the headline rate -- and the
    driver's 20-frame window within +-10 %."""
    s = _session(gpu)
    bits, _, idr = _run(s, 40, idr_at=(25,))
    T = 8000e3 / 60
    assert idr[0] == 1 and idr[25] == 1
    assert bits[0] <= 5.5 * T and bits[25] <= 5.5 * T, (bits[0] / T, bits[25] / T)
    assert abs(bits[5:25].mean() / T - 1) < 0.10, bits[5:25].mean() / T
