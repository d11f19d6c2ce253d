"""Per-frame timing breakdown of the tiled wall's encode rank (VERDICT r2 "Next round" #5d).

Starts WORLD ranks as fresh processes on the visible GPU(s) (one GPU: every rank shares it and
the tile exchange goes through gloo host staging, since RCCL needs one GPU per rank), runs the
pipelined wall for FRAMES frames and reports, per frame on the encode rank:

  render     own tile: HIP synthetic desktop + CSC (device time, CUDA events)
  exchange   host time blocked waiting for the posted tile exchange
  composite  k_composite_nv12 (device time)
  encode     encoder GPU time of the frame (FrameStats.encode_ms: submit -> done events)
  step       wall-clock time per delivered frame (host)

    python tools/wall_timing.py --layout 2x2 --tile 1920x1080 --frames 60 --json-out profiles/r03_wall/2x2.json
"""
import argparse
import json
import os
import socket
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cols, rows, tw, th, frames, codec, backend, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    from mxdesk.parallel import wall as W

    ndev = max(1, torch.cuda.device_count())
    dev = torch.device("cuda", rank % ndev)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    geo = W.WallGeometry(cols, rows, tw, th)
    try:
        if rank != 0:
            W.follower_loop(geo, rank, world, dev, "gather", fps=60)
            return
        pipe = W.WallPipeline(geo, 60, 0, world, dev, "gather", bitrate_kbps=8000 * world, codec=codec)
        rec = {"render": [], "exchange": [], "composite": []}
        pend_r = []

        orig_render = pipe.renderer.render

        def render(*a, **k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = orig_render(*a, **k)
            e1.record()
            pend_r.append((e0, e1))
            return out
        pipe.renderer.render = render

        orig_wait = pipe.xchg.wait

        def wait(reqs):
            t = time.perf_counter()
            out = orig_wait(reqs)
            rec["exchange"].append((time.perf_counter() - t) * 1e3)
            return out
        pipe.xchg.wait = wait

        orig_comp = W.composite_nv12

        def comp(*a, **k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            orig_comp(*a, **k)
            e1.record()
            pend_r.append(("c", e0, e1))
        W.composite_nv12 = comp

        # host time of the other per-frame stages (the step exceeded the sum of
        # render + exchange + composite + encode by 0.45 ms)
        class _TimedEncoder:  # the native encoder takes no attributes: a forwarding proxy
            def __init__(self, inner):
                self._inner = inner

            def __getattr__(self, n):
                return getattr(self._inner, n)

        pipe.enc = _TimedEncoder(pipe.enc)
        for name, obj, attr in (("ctrl_host", pipe, "_broadcast_ctrl"), ("post_host", pipe.xchg, "post"),
                                ("submit_host", pipe.enc, "submit"), ("collect_host", pipe.enc, "collect")):
            if not hasattr(obj, attr):
                continue
            rec[name] = []

            def timed(*a, _f=getattr(obj, attr), _n=name, **k):  # noqa: B023
                t = time.perf_counter()
                out = _f(*a, **k)
                rec[_n].append((time.perf_counter() - t) * 1e3)
                return out
            try:
                setattr(obj, attr, timed)
            except (AttributeError, TypeError):  # native objects may not take attributes
                del rec[name]
        enc_ms, step_ms = [], []
        for i in range(frames):
            t = time.perf_counter()
            fr = pipe.step()
            step_ms.append((time.perf_counter() - t) * 1e3)
            enc_ms.append(pipe.enc.stats.encode_ms)
        torch.cuda.synchronize()
        for item in pend_r:
            if item[0] == "c":
                rec["composite"].append(item[1].elapsed_time(item[2]))
            else:
                rec["render"].append(item[0].elapsed_time(item[1]))
        pipe.lockstep_frame(False, stop=True)
        warm = 5
        summ = {k: round(statistics.median(v[warm:]), 4) for k, v in rec.items() if len(v) > warm}
        summ["encode"] = round(statistics.median(enc_ms[warm:]), 4)
        summ["step"] = round(statistics.median(step_ms[warm:]), 4)
        summ["fps"] = round(1e3 / statistics.mean(step_ms[warm:]), 2)
        host = [k for k in ("ctrl_host", "post_host", "exchange", "submit_host", "collect_host") if k in summ]
        summ["host_unaccounted"] = round(summ["step"] - sum(summ[k] for k in host), 4)
        q.put({"layout": f"{cols}x{rows}", "tile": f"{tw}x{th}", "wall": f"{geo.width}x{geo.height}", "codec": pipe.codec,
               "ranks": world, "gpus": ndev, "backend": backend, "frames": frames, "median_ms": summ,
               "last_au_bytes": len(fr.au)})
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="2x2")
    ap.add_argument("--tile", default="1920x1080")
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--codec", default=None)
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import torch.multiprocessing as mp

    cols, rows = (int(v) for v in a.layout.lower().split("x"))
    tw, th = (int(v) for v in a.tile.lower().split("x"))
    world = cols * rows
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cols, rows, tw, th, a.frames, a.codec, a.backend, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
    line = json.dumps(res)
    print(line, flush=True)
    if a.json_out:
        Path(a.json_out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.json_out).write_text(line + "\n")
    sys.exit(0 if all(p.exitcode == 0 for p in procs) else 1)


if __name__ == "__main__":
    main()
