#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): encoded FPS + p50 end-to-end latency of a
1080p60 H.264 desktop session per MI355X; concurrent sessions/node.

One process per GPU (torchrun / torch.distributed over RCCL for N > 1).  Each rank runs
one 1920x1080 session of the flagship pipeline on its GPU:

    HIP synthetic desktop render (animated noise + gears + scrolling text + moving window,
    frame-id/timestamp barcode) -> BT.709 NV12 (HIP) -> H.264 encode (HIP: ME, transform,
    quant, recon, CAVLC, bit packing) -> Annex-B access unit in host memory

A "step" is one encoded frame.  Frames are encoded back-to-back (unpaced) to measure the
encoder's capacity, with two frames in flight per session by default (frame n's entropy
coding overlaps frame n+1's analysis on a second HIP stream, as hardware encoders pipeline);
E2E latency is render-start -> access unit available on the host, per frame, measured in the
same run (so it includes the pipelining queueing).  `value` is the whole-job aggregate encoded FPS (sum over GPUs, total frames /
slowest rank's time).  Weak scaling: per-GPU work is fixed as N grows.

The reference publishes no numbers, so vs_baseline is null; the reference's
operating point (60 encoded FPS per session, one session per GPU) is reported as
`vs_operating_point` = value / (60 * N).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))


# codec -> (name, encoder element, bitstream profile)
CODEC_LABEL = {
    "h264": ("H.264", "mxh264enc", "H.264 Constrained Baseline"),
    "hevc": ("HEVC", "mxh265enc", "HEVC Main profile"),
    "vp8": ("VP8", "mxvp8enc", "VP8 (RFC 6386) key + inter frames"),
}

REGION_NAMES = ["wallpaper", "taskbar", "document", "noise", "terminal", "gears", "barcode", "video"]


def desktop_regions(W: int, H: int):
    """Pixel class map of the synthetic desktop in desktop coordinates (the renderer's layout,
    csrc/kernels/pixel.hip static_px / desktop_px; indices into REGION_NAMES)."""
    import numpy as np

    cls = np.zeros((H, W), np.int8)
    boxes = {  # (x0, y0, x1, y1), later entries on top as in the renderer's order
        2: (int(W * .25), int(H * .52), int(W * .25) + int(W * .24), int(H * .52) + int(H * .36)),
        1: (0, H - 32, W, H),
        3: (int(W * .04), int(H * .55), int(W * .04) + int(W * .16), int(H * .55) + int(H * .22)),
        4: (int(W * .04), int(H * .10), int(W * .04) + int(W * .42), int(H * .10) + int(H * .38)),
        5: (int(W * .55), int(H * .10), int(W * .55) + int(W * .38), int(H * .10) + int(H * .50)),
    }
    for k in (2, 1, 3, 4, 5):
        x0, y0, x1, y1 = boxes[k]
        cls[y0:y1, x0:x1] = k
    return cls


def quality_probe(s, W: int, H: int, content: int, noise: int, n: int = 30) -> dict:
    """Not timed: n more frames of the same session with the source and the reconstruction read
    back, for per-region luma PSNR (regions of the renderer's layout; with motion content the
    desktop regions pan under the screen-fixed barcode and video panel) and chroma PSNR."""
    import numpy as np

    base = desktop_regions(W, H)
    if not noise:
        base[base == 3] = 0
    sse = np.zeros(len(REGION_NAMES))
    cnt = np.zeros(len(REGION_NAMES))
    suv = [0.0, 0.0]
    suv_m, cnt_m = [0.0, 0.0], 0
    for _ in range(n):
        r = s.step(False)
        sy, su = s.nv12()
        ry, ru = s.recon()
        if content in (1, 2):
            f = r.frame_id
            # the renderer's pan (pix pan_of / pan_q4), to the nearest sample for the region map
            px, py = ((3 * f) % W, f % H) if content == 1 else (((10 * f) % (4 * W) + 2) // 4, ((3 * f) % (4 * H) + 2) // 4)
            cls = np.roll(base, (-py, -px), axis=(0, 1))
            vx0, vy0 = int(W * 0.60), int(H * 0.56)
            cls[vy0:vy0 + int(H * 0.36), vx0:vx0 + int(W * 0.34)] = 7
        else:
            cls = base.copy()
        cls[0:8 + 3 * 8, 0:8 + 33 * 8] = 6  # barcode (screen-fixed, kBarX/kBarY/kBarCell = 8)
        e = (ry[:H, :W].astype(np.int64) - sy[:H, :W].astype(np.int64)) ** 2
        sse += np.bincount(cls.ravel(), weights=e.ravel(), minlength=len(REGION_NAMES))
        cnt += np.bincount(cls.ravel(), minlength=len(REGION_NAMES))
        keep = cls[0:H - H % 2:2, 0:W - W % 2:2] != 3  # chroma samples outside the noise panel
        cnt_m += int(keep.sum())
        for c in range(2):
            d = ru[:H // 2, c:W:2].astype(np.int64) - su[:H // 2, c:W:2].astype(np.int64)
            suv[c] += float((d * d).sum())
            suv_m[c] += float((d * d)[keep].sum())

    def psnr(e, k):
        return 99.0 if e <= 0 else round(min(99.0, 10 * np.log10(65025.0 * k / e)), 2)

    regions = {REGION_NAMES[k]: psnr(sse[k], cnt[k]) for k in range(len(REGION_NAMES)) if cnt[k] > 0}
    y = psnr(sse.sum(), cnt.sum())
    out = {"frames": n, "psnr_y_db": y, "psnr_u_db": psnr(suv[0], n * (W // 2) * (H // 2)),
           "psnr_v_db": psnr(suv[1], n * (W // 2) * (H // 2)), "regions_psnr_y_db": regions,
           # chroma with the incompressible noise panel left out, as the masked luma figure
           "psnr_u_db_noise_masked": psnr(suv_m[0], cnt_m), "psnr_v_db_noise_masked": psnr(suv_m[1], cnt_m)}
    scored = {k: v for k, v in regions.items() if k not in ("noise", "barcode")}
    out["worst_region_below_frame_db"] = round(y - min(scored.values()), 2) if scored else None
    return out


def density_probe(N, cfg, fps: int, k0: int = 8, k_max: int = 1024, seconds: float = 1.0,
                  threads: int = 8, idr_storm: bool = False, cpu_noise: int | None = None) -> dict:
    """Paced concurrent sessions on this GPU: K sessions (same config, pipeline depth 1) driven by
    `threads` host threads (N.run_sessions_paced: every 1/fps slot each thread submits one frame
    per session it owns, then collects them); K is sustained if no slot overran (every frame of
    every session encoded before the next slot starts) over `seconds`.  K doubles from k0 until a
    K fails, then bisects between the last sustained and the first failing K (to within 1/16), so
    `sustained` is a measured limit -- the first failing K minus the resolution -- not a list cap.
    The whole serving path per session (render, CSC, encode, bitstream to host) runs.
    idr_storm: in the middle slot every session codes a forced IDR picture (viewers joining at once,
    a PLI burst); K is sustained only if that slot, too, finishes within its period.
    cpu_noise not None: the no-GPU plumbing configuration -- K CpuSessions (numpy desktop + C++
    CPU encoder) stepped from this thread, each slot's frames due within the slot."""
    out = {"fps": fps, "seconds": seconds, "threads": threads, "idr_storm": idr_storm, "tried": {}}

    def cpu_trial(K: int) -> bool:
        sess = []
        for _ in range(K):
            c = N.SessionConfig()
            c.width, c.height, c.fps = cfg.width, cfg.height, cfg.fps
            c.enc.bitrate_kbps = cfg.enc.bitrate_kbps
            sess.append(CpuSession(N, c, cpu_noise))
        for s in sess:
            s.step(False)
        slots = max(1, round(seconds * fps))
        late, lat = 0, []
        t_next = time.perf_counter()
        for k in range(slots):
            t_next += 1.0 / fps
            for s in sess:
                r = s.step(idr_storm and k == slots // 2, quality=False)
                lat.append((r.t_encoded_us - r.t_capture_us) / 1000.0)
            now = time.perf_counter()
            if now > t_next:
                late += 1
                t_next = now
            else:
                time.sleep(t_next - now)
        lat.sort()
        out["tried"][K] = {"late_slots": late, "slots": slots, "p50_ms": round(lat[len(lat) // 2], 3)}
        return late == 0

    def trial(K: int) -> bool:
        if cpu_noise is not None:
            return cpu_trial(K)
        sess = []
        try:
            for _ in range(K):
                c = N.SessionConfig()
                for a in ("width", "height", "fps", "noise", "codec", "out_width", "out_height"):
                    setattr(c, a, getattr(cfg, a))
                c.enc.bitrate_kbps = cfg.enc.bitrate_kbps
                c.enc.pipeline_depth = 1
                sess.append(N.Session(c))
            for s in sess:  # warm-up: first IDR + rate-control probe
                s.step(False)
            slots = max(1, round(seconds * fps))
            st = N.run_sessions_paced(sess, fps, seconds, min(threads, K), slots // 2 if idr_storm else -1)
            lat = sorted(st.lat_ms)
            rec = {"late_slots": st.late_slots, "slots": st.slots, "p50_ms": round(lat[len(lat) // 2], 3),
                   "p99_ms": round(lat[int(0.99 * (len(lat) - 1))], 3)}
            if idr_storm:
                il = sorted(st.idr_lat_ms)
                rec.update(idr_slot_late=bool(st.idr_late), idr_p50_ms=round(il[len(il) // 2], 3),
                           idr_max_ms=round(il[-1], 3))
            out["tried"][K] = rec
            return st.late_slots == 0
        except RuntimeError as e:  # out of device memory etc.: counts as a failing K
            out["tried"][K] = {"error": str(e)[:120]}
            return False
        finally:
            del sess

    good, bad = 0, None
    K = k0
    while K <= k_max:
        if trial(K):
            good = K
            K *= 2
        else:
            bad = K
            break
    if bad is not None:
        while bad - good > max(1, good // 16):
            mid = (good + bad) // 2
            if trial(mid):
                good = mid
            else:
                bad = mid
    out["sustained"] = good
    out["first_failing"] = bad
    return out


def launch_ranks(n: int, timeout_s: float | None = None) -> int:
    """`bench.py --gpus N` without WORLD_SIZE: run N rank processes of this script (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them, rendezvous on
    127.0.0.1) and return the first non-zero exit code.  Rank 0 prints the JSON line; the ranks
    share this process's stdout.  All children are polled: when one fails (e.g. before or during
    init_process_group, which would leave the others blocked in the rendezvous) the rest are
    terminated and its code returned; an overall time limit (MXDESK_BENCH_TIMEOUT seconds,
    default 1800) ends a hung job with 124."""
    import signal
    import socket
    import subprocess

    if timeout_s is None:
        timeout_s = float(os.environ.get("MXDESK_BENCH_TIMEOUT", "") or 1800)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        t_kill = time.monotonic() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_kill - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    deadline = time.monotonic() + timeout_s
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            print(f"bench.py: a rank exited with {bad[0]}; stopping the others", file=sys.stderr)
            stop_all()
            return bad[0]
        if all(c == 0 for c in codes):
            return 0
        if time.monotonic() > deadline:
            print(f"bench.py: ranks still running after {timeout_s:.0f} s; stopping them", file=sys.stderr)
            stop_all()
            return 124
        time.sleep(0.05)


class CpuSession:
    """The plumbing configuration's session (BASELINE config 1, no GPU): the numpy desktop
    (mxdesk.models.synthetic.CpuSyntheticDesktop) -> BT.709 NV12 -> the C++ CPU H.264 encoder
    (the GPU encoder's bit-exact oracle).  step() returns the FrameResult fields bench.py reads."""

    def __init__(self, N, cfg, noise: int):
        from mxdesk.models.synthetic import CpuSyntheticDesktop, bgrx_to_nv12

        self._conv = bgrx_to_nv12
        self.desk = CpuSyntheticDesktop(cfg.width, cfg.height, noise=bool(noise))
        cfg.enc.width, cfg.enc.height, cfg.enc.fps = cfg.width, cfg.height, cfg.fps
        self.enc = N.CpuH264Encoder(cfg.enc)
        self.fps = cfg.fps
        self.n = 0

    def step(self, force_idr: bool = False, quality: bool = True):
        import types

        import numpy as np

        t0 = time.monotonic()
        img = self.desk.render(self.n, self.n / self.fps, int(t0 * 1e6))
        y, uv = self._conv(img)
        au = self.enc.encode(y, uv, force_idr)
        t1 = time.monotonic()
        st = self.enc.stats
        self.n += 1
        if not quality:
            return types.SimpleNamespace(au=au, qp=st.qp, t_capture_us=t0 * 1e6, t_encoded_us=t1 * 1e6)
        w, h = self.desk.w, self.desk.h
        ry, ruv = self.enc.recon()

        def sse(a, b):
            d = a.astype(np.int64) - b.astype(np.int64)
            return float((d * d).sum())

        def psnr(e, k):
            return 99.0 if e <= 0 else min(99.0, 10 * math.log10(65025.0 * k / e))

        py_ = psnr(sse(ry[:h, :w], y[:h, :w]), w * h)
        su = sse(ruv[:h // 2, 0:w:2], uv[:h // 2, 0:w:2])
        sv = sse(ruv[:h // 2, 1:w:2], uv[:h // 2, 1:w:2])
        return types.SimpleNamespace(au=au, qp=st.qp, psnr_y=py_, psnr_y_masked=py_, psnr_u=psnr(su, w * h / 4),
                                     psnr_v=psnr(sv, w * h / 4), gpu_ms=0.0, t_capture_us=t0 * 1e6,
                                     t_encoded_us=t1 * 1e6)


def serving_probe(args, dev_index: int) -> dict | None:
    """The density probes in the serving path's configuration: a child process of this one (never an
    exec) with GPU_MAX_HW_QUEUES=16, as `mxdesk serve --sessions K` runs its sessions (mxdesk/cli.py),
    on this rank's GPU, outside any process group.  More hardware queues let the sessions' IDR
    wavefronts -- long serial chains on few workgroups -- run side by side instead of queueing
    (profiles/r06_density/NOTES.md); the in-process probes keep HIP's default."""
    import subprocess

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["GPU_MAX_HW_QUEUES"] = "16"
    cmd = [sys.executable, str(Path(__file__).resolve()), *sys.argv[1:], "--gpus", "1", "--density-only", "1",
           "--device-index", str(dev_index), "--quality-probe", "0"]
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    except subprocess.TimeoutExpired:
        print("bench.py: serving probe timed out", file=sys.stderr)
        return None
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        print(f"bench.py: serving probe failed (rc {p.returncode}): {p.stderr[-500:]}", file=sys.stderr)
        return None
    return json.loads(lines[-1])


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fps", type=int, default=60)
    ap.add_argument("--out-width", type=int, default=0, help="encode width (0 = desktop width; else fused Lanczos-3 + CSC)")
    ap.add_argument("--out-height", type=int, default=0)
    ap.add_argument("--bitrate-kbps", type=int, default=8000)
    ap.add_argument("--codec", default="h264", choices=["h264", "hevc", "vp8"],
                    help="h264 (headline, mxh264enc), hevc (mxh265enc, BASELINE config '4K60 HEVC') or vp8 "
                         "(mxvp8enc, the reference's WEBRTC_ENCODER=vp8enc)")
    ap.add_argument("--tu-split", type=int, default=None,
                    help="HEVC: let inter CUs split their transform tree into 8x8 / 4x4 TUs (default: encoder default)")
    ap.add_argument("--sao", type=int, default=None, help="HEVC sample adaptive offset (default on)")
    ap.add_argument("--hevc-slice-cost", type=int, default=None,
                    help="HEVC P-picture slice work target (more = fewer, longer slices)")
    ap.add_argument("--hevc-wpp", type=int, default=None,
                    help="HEVC wavefront substreams (1) or cost-balanced slices (0, default)")
    ap.add_argument("--hevc-wpp-rows", type=int, default=None,
                    help="HEVC with WPP: CTU rows per P slice (0 = one slice per picture)")
    ap.add_argument("--search-range", type=int, default=16)
    ap.add_argument("--subpel", type=int, default=1)
    ap.add_argument("--me-coarse", type=int, default=None,
                    help="1: even-offset grid + integer neighbours, 0: exhaustive search (encoder default)")
    ap.add_argument("--intra4x4", type=int, default=None, help="0: intra MBs Intra16x16 only")
    ap.add_argument("--noise", type=int, default=1, help="animated white-noise panel (incompressible content)")
    ap.add_argument("--content", default="desktop", choices=["desktop", "motion", "subpel"],
                    help="synthetic source: the desktop, motion content (the whole desktop pans 3 px / frame "
                         "under a screen-fixed video-like panel; no noise panel), or subpel (a fractional pan of "
                         "2.5 px right / 0.75 px down per frame, bilinearly resampled, under a zooming video panel: "
                         "quarter-sample motion, the interpolation filters and the deblocking decision exercised)")
    ap.add_argument("--quality-probe", type=int, default=30,
                    help="untimed frames after the run with per-region / chroma PSNR read back (0: off)")
    ap.add_argument("--aq", type=int, default=None,
                    help="adaptive quantisation: 0 off, 1 coarser QP for noise-like MBs, 2 + rate-distortion "
                         "residual drop for them (default: the encoder's)")
    ap.add_argument("--deblock", type=int, default=None,
                    help="in-loop deblocking filter 0 off / 1 on / 2 adaptive per picture (H.264: "
                         "from the picture's temporal classes; default: the encoder's)")
    ap.add_argument("--hevc-intra-split", type=int, default=None,
                    help="HEVC I pictures: 16x16 intra units may split into four 8x8 luma / 4x4 chroma TUs "
                         "(1, the encoder's default) or not (0)")
    ap.add_argument("--hevc-chroma-keep", type=int, default=None,
                    help="HEVC: changing content keeps its chroma residual (1) instead of dropping it (0)")
    ap.add_argument("--chroma-qp-offset", type=int, default=None,
                    help="chroma QP offset against luma (H.264 chroma_qp_index_offset / HEVC pps_cb/cr_qp_offset; "
                         "default: the encoder's)")
    ap.add_argument("--intra-in-p", type=int, default=None,
                    help="H.264: P-slice macroblocks may switch to intra (default: encoder default)")
    ap.add_argument("--vp8-bpred", type=int, default=None, help="VP8 key frames: B_PRED macroblocks (default 1)")
    ap.add_argument("--vp8-intra", type=int, default=None, help="VP8 inter frames: intra macroblocks (default 1)")
    ap.add_argument("--depth", type=int, default=None,
                    help="GPU frames in flight per session (2: entropy coding of frame n overlaps analysis of n+1; "
                         "3: also the next frame's launches stay queued while the host collects, so the host "
                         "turnaround overlaps GPU work; 1: strictly one frame at a time, lowest back-to-back latency; "
                         "default 3, VP8 4: its host bitstream writers run one per frame in flight)")
    ap.add_argument("--capture-stream", type=int, default=-1,
                    help="depth > 1: render + convert on a capture stream, one NV12 buffer per frame in flight "
                         "(frame n+1's capture overlaps frame n's analysis); -1 = H.264 and HEVC (measured gains), "
                         "1 = every codec, 0 = one analysis stream")
    ap.add_argument("--graph", type=int, default=0,
                    help="replay the per-frame chain as a hipGraph (eager launches measured faster: profiles/r01_graph)")
    ap.add_argument("--sessions-per-gpu", type=int, default=1,
                    help="concurrent sessions per GPU (density): each has its own HIP stream and one frame in flight")
    ap.add_argument("--density-probe", type=int, default=1,
                    help="after the timed run, measure how many paced 1080p60 sessions this GPU sustains in this "
                         "process (doubling K until a 60 fps slot is missed, then bisecting); reported, never part "
                         "of `value`")
    ap.add_argument("--serving-probe", type=int, default=1,
                    help="GPU: also run the paced and IDR-storm density probes in the serving path's configuration "
                         "(a child process with the 16 hardware queues `mxdesk serve --sessions K` sets, "
                         "mxdesk/cli.py); reported beside the in-process probes, never part of `value`")
    ap.add_argument("--density-only", type=int, default=0, help=argparse.SUPPRESS)  # the serving-probe child
    ap.add_argument("--device-index", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for N>1 (nccl = RCCL on ROCm; gloo only to rehearse the "
                         "multi-rank plumbing with several ranks on one GPU)")
    ap.add_argument("--py-loop", type=int, default=0,
                    help="1: drive a single session from this Python thread instead of the native session driver")
    ap.add_argument("--json-out", type=str, default="")
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"],
                    help="cpu: the no-GPU plumbing configuration (BASELINE config 1): numpy-rendered desktop + the "
                         "C++ CPU H.264 encoder, one process per rank over gloo; never the headline number")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} (one rank per GPU: "
                  "launch with --nproc-per-node equal to --gpus)", file=sys.stderr)
            sys.exit(2)
    elif args.gpus > 1:
        # no launcher: start one fresh rank process per GPU ourselves.  Nothing in this parent has
        # touched the GPU (no torch / HIP import yet); the ranks are children, never an exec.
        sys.exit(launch_ranks(args.gpus))
    gpu = args.device == "gpu"
    if not gpu:  # plumbing configuration: CPU encoder, gloo, no GPU-only probes
        args.codec, args.backend, args.quality_probe = "h264", "gloo", 0
        args.depth, args.sessions_per_gpu, args.out_width, args.out_height = 1, 1, 0, 0
    if args.codec == "vp8":
        args.depth = min(args.depth or 4, 4)  # the VP8 encoder keeps at most four frames in flight
    if args.depth is None:
        args.depth = 3
    content = {"desktop": 0, "motion": 1, "subpel": 2}[args.content]
    if content:
        args.noise = 0  # the motion content has a video panel instead of the noise panel

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MXDESK_BENCH_FAIL_RANK", "") == str(rank):  # tests: a rank dying before rendezvous
        print(f"bench.py: rank {rank} fails (MXDESK_BENCH_FAIL_RANK)", file=sys.stderr)
        sys.exit(3)

    import torch

    # one rank per GPU; the modulo only matters when rehearsing several ranks on fewer GPUs
    ndev = max(1, torch.cuda.device_count()) if gpu else 1
    dev_index = args.device_index if args.device_index >= 0 else local_rank % ndev
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        if gpu:
            torch.cuda.set_device(dev_index)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(args.backend)
    elif gpu:
        torch.cuda.set_device(dev_index)
    coll_dev = "cuda" if gpu and (dist is None or args.backend == "nccl") else "cpu"

    import mxdesk

    N = mxdesk.native()
    if gpu:
        N.set_device(dev_index)
    cfg = N.SessionConfig()
    cfg.width, cfg.height, cfg.fps = args.width, args.height, args.fps
    cfg.out_width, cfg.out_height = args.out_width, args.out_height
    cfg.enc.bitrate_kbps = args.bitrate_kbps
    cfg.enc.search_range = args.search_range
    cfg.enc.subpel = args.subpel
    if args.tu_split is not None:
        cfg.enc.tu_split = args.tu_split
    if args.sao is not None:
        cfg.enc.sao = args.sao
    if args.hevc_slice_cost is not None:
        cfg.enc.hevc_slice_cost = args.hevc_slice_cost
    if args.hevc_wpp is not None:
        cfg.enc.hevc_wpp = args.hevc_wpp
    if args.hevc_wpp_rows is not None:
        cfg.enc.hevc_wpp_rows = args.hevc_wpp_rows
    if args.hevc_chroma_keep is not None:
        cfg.enc.hevc_chroma_keep = args.hevc_chroma_keep
    if args.hevc_intra_split is not None:
        cfg.enc.hevc_intra_split = args.hevc_intra_split
    if args.chroma_qp_offset is not None:
        cfg.enc.chroma_qp_offset = args.chroma_qp_offset
    if args.intra_in_p is not None:
        cfg.enc.intra_in_p = args.intra_in_p
    if args.vp8_bpred is not None:
        cfg.enc.vp8_bpred = args.vp8_bpred
    if args.vp8_intra is not None:
        cfg.enc.vp8_intra = args.vp8_intra
    if args.deblock is not None:
        cfg.enc.deblock = args.deblock
    if args.aq is not None:
        cfg.enc.aq = args.aq
    if args.me_coarse is not None:
        cfg.enc.me_coarse = args.me_coarse
    if args.intra4x4 is not None:
        cfg.enc.intra4x4 = args.intra4x4
    cfg.noise = args.noise
    cfg.content = content
    cfg.use_graph = args.graph
    cfg.capture_stream = args.capture_stream
    cfg.enc.pipeline_depth = args.depth
    cfg.codec = args.codec
    ow, oh = (args.out_width or args.width), (args.out_height or args.height)
    if args.noise:
        # quality report with the incompressible noise panel masked out (same rectangle as the
        # renderer's desktop_px(), csrc/kernels/pixel.hip, in encoded-picture coordinates)
        cfg.mask_x0, cfg.mask_y0 = int(ow * 0.04), int(oh * 0.55)
        cfg.mask_x1, cfg.mask_y1 = cfg.mask_x0 + int(ow * 0.16) + 1, cfg.mask_y0 + int(oh * 0.22) + 1
    if args.density_only:  # the serving-probe child: the two density probes, one JSON line
        d = density_probe(N, cfg, args.fps)
        st = density_probe(N, cfg, args.fps, k0=max(4, (d["sustained"] or 16) // 4), idr_storm=True)
        print(json.dumps({"density": d, "storm": st, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)
        return
    K = max(1, args.sessions_per_gpu)
    sessions = [N.Session(cfg) if gpu else CpuSession(N, cfg, args.noise) for _ in range(K)]

    def run(n_frames: int, record: bool):
        """n_frames per session, up to `depth` frames in flight each, driven by the native session
        runtime (run_sessions: one host thread per session, submit / collect in C++ -- as the
        serving path's pipeline thread does); --py-loop 1: this Python thread."""
        out = []
        depth = max(1, args.depth)
        if not gpu:
            res = [sessions[0].step(False) for _ in range(n_frames)]
            return res if record else []
        if K > 1 or not args.py_loop:
            per = N.run_sessions(sessions, n_frames, depth)
            if record:
                for f in range(n_frames):
                    out.extend(per[k][f] for k in range(K))
            return out
        sent = [0] * K
        for k, s in enumerate(sessions):
            while sent[k] < min(depth, n_frames):
                s.submit(False)
                sent[k] += 1
        for _ in range(n_frames):
            for k, s in enumerate(sessions):
                r = s.collect()
                if sent[k] < n_frames:
                    s.submit(False)
                    sent[k] += 1
                if record:
                    out.append(r)
        return out

    run(args.warmup, False)

    def barrier():
        if gpu:
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    lat_ms, sizes, qps, gpu_ms, psnrs, psnrs_m, psnr_uv, dbk, dbc = [], [], [], [], [], [], [], [], []
    if K == 1 and args.depth == 1 and gpu:
        results = [sessions[0].step(False) for _ in range(args.steps)]
    else:
        results = run(args.steps, True)
    barrier()
    elapsed = time.perf_counter() - t0
    for r in results:
        lat_ms.append((r.t_encoded_us - r.t_capture_us) / 1000.0)
        sizes.append(len(r.au))
        qps.append(r.qp)
        psnrs.append(r.psnr_y)
        psnrs_m.append(r.psnr_y_masked if args.noise else r.psnr_y)
        psnr_uv.append((r.psnr_u, r.psnr_v))
        gpu_ms.append(r.gpu_ms)
        dbk.append(getattr(r, "deblocked", 0))
        dbc.append((getattr(r, "db_coherent", 0), getattr(r, "db_moving", 0)))

    quality = None
    if args.quality_probe > 0 and rank == 0 and not args.out_width:
        quality = quality_probe(sessions[0], args.width, args.height, content, args.noise, args.quality_probe)
    if args.density_probe:
        density = (density_probe(N, cfg, args.fps) if gpu else
                   density_probe(N, cfg, args.fps, k0=1, k_max=64, seconds=0.25, cpu_noise=args.noise))
    else:
        density = None
    # the same probe with every session's IDR in one slot, from a quarter of the steady-state K
    storm = (density_probe(N, cfg, args.fps, k0=max(4, (density["sustained"] or 16) // 4), idr_storm=True)
             if args.density_probe and gpu else None)
    serving = serving_probe(args, dev_index) if args.density_probe and args.serving_probe and gpu else None

    if dist is not None:
        t = torch.tensor([elapsed], device=coll_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed_max = float(t.item())
        gathered = [None] * world
        dist.all_gather_object(gathered, lat_ms)
        all_lat = [x for g in gathered for x in g]
        gsz = [None] * world
        dist.all_gather_object(gsz, sizes)
        all_sizes = [x for g in gsz for x in g]
        # every rank probed its own GPU: the node's figure is the sum over ranks
        gd = [None] * world
        dist.all_gather_object(gd, [density["sustained"] if density else None, storm["sustained"] if storm else None,
                                    serving["density"]["sustained"] if serving else None,
                                    serving["storm"]["sustained"] if serving else None])
        rank_density, rank_storm = [d[0] for d in gd], [d[1] for d in gd]
        rank_sdensity, rank_sstorm = [d[2] for d in gd], [d[3] for d in gd]
    else:
        elapsed_max, all_lat, all_sizes = elapsed, lat_ms, sizes
        rank_density = [density["sustained"] if density else None]
        rank_storm = [storm["sustained"] if storm else None]
        rank_sdensity = [serving["density"]["sustained"] if serving else None]
        rank_sstorm = [serving["storm"]["sustained"] if serving else None]

    def node_sum(v):
        return None if any(x is None for x in v) else sum(v)

    total_frames = args.steps * world * K
    fps_total = total_frames / elapsed_max
    p50 = statistics.median(all_lat)
    p95 = sorted(all_lat)[int(0.95 * (len(all_lat) - 1))]
    per_gpu = fps_total / world
    kbps = statistics.mean(all_sizes) * 8 * args.fps / 1000.0
    if rank == 0:
        out = {
            # BASELINE.json's metric verbatim for the headline configuration
            "metric": {"h264": "encoded FPS + p50 end-to-end latency at 1080p60 H.264; concurrent sessions/node",
                       "hevc": "encoded FPS (HEVC desktop session, aggregate over GPUs) + p50 E2E latency",
                       "vp8": "encoded FPS (VP8 desktop session, aggregate over GPUs) + p50 E2E latency"}[args.codec]
            if gpu else "encoded FPS, CPU plumbing configuration (numpy desktop + C++ CPU H.264; no GPU)",
            "value": round(fps_total, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1000.0, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "vs_operating_point": round(fps_total / (60.0 * world), 3),
            "p50_e2e_latency_ms": round(p50, 3),
            "p95_e2e_latency_ms": round(p95, 3),
            "encoded_fps_per_gpu": round(per_gpu, 2),
            "sessions_per_gpu": K,
            "hip_graph": bool(args.graph),
            "capture_stream": bool(sessions[0].capture_stream_active) if gpu else False,
            "device": args.device,
            "pipeline_depth": args.depth,
            "deblock": int(cfg.enc.deblock),
            # -1 resolves to adaptive for every codec (csrc/codec/h264_encoder.h deblock)
            "deblock_mode": {0: "off", 1: "on", 2: "adaptive"}.get(int(cfg.enc.deblock), "adaptive"),
            "intra_in_p": int(cfg.enc.intra_in_p),
            "vp8_tools": {"bpred": int(cfg.enc.vp8_bpred), "intra": int(cfg.enc.vp8_intra)} if args.codec == "vp8" else None,
            "hevc_intra_split": int(cfg.enc.hevc_intra_split) if args.codec == "hevc" else None,
            "deblocked_frames_pct": round(100.0 * sum(dbk) / max(1, len(dbk)), 1),
            # the adaptive filter's inputs (h264_deblock.h db_auto_decide): mean coherent / moving
            # macroblocks per picture
            "db_classes_mean": [round(statistics.mean(c for c, _ in dbc), 1), round(statistics.mean(m for _, m in dbc), 1)]
            if dbc else None,
            "mean_gpu_encode_ms": round(statistics.mean(gpu_ms), 3),
            "mean_bitrate_kbps_at_60fps": round(kbps, 1),
            "mean_qp": round(statistics.mean(qps), 2),
            "mean_psnr_y_db": round(statistics.mean(psnrs), 2),
            "mean_psnr_y_db_noise_masked": round(statistics.mean(psnrs_m), 2),
            "mean_psnr_u_db": round(statistics.mean(u for u, _ in psnr_uv), 2),
            "mean_psnr_v_db": round(statistics.mean(v for _, v in psnr_uv), 2),
            "mean_psnr_u_db_noise_masked": quality["psnr_u_db_noise_masked"] if quality else None,
            "mean_psnr_v_db_noise_masked": quality["psnr_v_db_noise_masked"] if quality else None,
            "content": args.content,
            "quality_probe": quality,
            # measured, not extrapolated: K paced sessions (one HIP stream each, depth 1) on this
            # GPU from `threads` host threads, every frame of every session encoded within its 1/fps
            # slot; K found by doubling then bisecting up to the first failing K
            "sessions_per_gpu_at_60fps_measured": density["sustained"] if density else None,
            "density_probe": density,
            # the node metric (BASELINE "concurrent sessions/node"): every rank's own measured K,
            # all-gathered, and their sum -- not rank 0's figure times N
            "sessions_per_node_measured": node_sum(rank_density),
            "sessions_per_gpu_measured_min": min(rank_density) if node_sum(rank_density) is not None else None,
            "sessions_per_gpu_measured_max": max(rank_density) if node_sum(rank_density) is not None else None,
            "sessions_per_gpu_measured_by_rank": rank_density,
            "sessions_per_node_idr_storm_measured": node_sum(rank_storm),
            # measured: the sustained K when every session codes a forced IDR in the same slot
            "sessions_per_gpu_idr_storm_measured": storm["sustained"] if storm else None,
            "density_probe_idr_storm": storm,
            # the same two probes in the serving path's configuration (serving_probe: a child process
            # with the 16 hardware queues `mxdesk serve --sessions K` uses)
            "serving_config": {"hw_queues": 16,
                               "sessions_per_node_measured": node_sum(rank_sdensity),
                               "sessions_per_node_idr_storm_measured": node_sum(rank_sstorm),
                               "sessions_per_gpu_measured_by_rank": rank_sdensity,
                               "sessions_per_gpu_idr_storm_by_rank": rank_sstorm} if serving else None,
            "dtype": "uint8 video (8-bit 4:2:0), " + CODEC_LABEL[args.codec][2],
            "data": "synthetic (HIP-rendered animated-noise/gears desktop, random-free deterministic)" if gpu
            else "synthetic (numpy-rendered desktop, mxdesk.models.synthetic.CpuSyntheticDesktop)",
            "config": {
                "model": f"{args.width}x{args.height}@{args.fps} {CODEC_LABEL[args.codec][0]}"
                         " desktop session"
                         + (f" scaled to {args.out_width}x{args.out_height}" if args.out_width else "")
                         + f" ({CODEC_LABEL[args.codec][1]}, CBR "
                         f"{args.bitrate_kbps} kbps, ME +/-{args.search_range} qpel={args.subpel})",
                "global_batch": world * K,
                "seq_len": args.width * args.height,
                "parallelism": f"session-per-gpu x{world}" + (f", {K} sessions/GPU" if K > 1 else ""),
            },
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            Path(args.json_out).write_text(line + "\n")
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
