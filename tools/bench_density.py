"""Session density over real WebRTC (VERDICT r2 "Next round" #6): K sessions served by ONE
`mxdesk serve --sessions K` process on one GPU, K headless WHEP viewers (ICE, DTLS-SRTP, NACK,
RTCP) spread over a few client processes, every session paced at 60 fps.

A K passes when every viewer receives its stream at >= 59.5 fps over the measurement window and
the 95th percentile of capture -> viewer latency (RTCP sender-report mapping of the RTP clock to
the wall clock, same host) is below 5 ms.  The sweep stops at the first failing K; the sustained
density is that K minus one step.

    python tools/bench_density.py --sweep 8,16,32,48,64 --frames 300 --json-out profiles/r03_density/density.json
"""
import argparse
import asyncio
import http.client
import json
import os
import resource
import socket
import statistics
import subprocess
import sys
import time
import urllib.request
from pathlib import Path

import psutil

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _free_port_block(n: int) -> int:
    # below the ephemeral range: a readiness probe to a port nobody listens on yet can otherwise
    # connect to itself (source port == destination port) and read its own request back
    import random

    lo = 20000
    try:
        lo = min(lo, int(Path("/proc/sys/net/ipv4/ip_local_port_range").read_text().split()[0]) - n - 1)
    except (OSError, ValueError, IndexError):
        pass
    for _ in range(200):
        base = random.randint(10000, max(10001, lo))
        if all(_port_free(base + i) for i in range(n)):
            return base
    raise RuntimeError("no free port block")


def _port_free(p: int) -> bool:
    with socket.socket() as s:
        try:
            s.bind(("127.0.0.1", p))
            return True
        except OSError:
            return False


def _wait_ready(ports, timeout=180.0):
    t0 = time.monotonic()
    pending = set(ports)
    while pending and time.monotonic() - t0 < timeout:
        for p in list(pending):
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{p}/health", timeout=1.0) as r:
                    if r.status == 200:
                        pending.discard(p)
            except (OSError, http.client.HTTPException):
                pass
        time.sleep(0.5)
    if pending:
        raise RuntimeError(f"sessions not ready: {sorted(pending)[:5]}")


def _client_proc(ports, frames, q, lite=False):
    from mxdesk.server.whep_client import e2e_latency_ms, whep_view

    async def one(p):
        try:
            res = await whep_view(f"http://127.0.0.1:{p}/whep", frames, timeout=frames / 30.0 + 60, lite=lite)
        except Exception as e:  # a stalled session is a failure of this K, not of the tool
            r = getattr(e, "whep_result", None)
            diag = {} if r is None else {"stage": r.stage, "ice_tx": r.ice_tx, "datagrams": r.datagrams,
                                          "aus": len(r.aus), "nacked": r.nacked, "gave_up": r.gave_up,
                                          "dropped_aus": r.dropped_aus}
            return {"port": p, "error": repr(e), "diag": diag}
        arr = res.arrival_wall
        warm = min(30, len(arr) // 4)
        span = arr[-1] - arr[warm] if len(arr) > warm + 1 else 0.0
        fps = (len(arr) - 1 - warm) / span if span > 0 else 0.0
        lat = e2e_latency_ms(res)[warm:]
        return {"port": p, "fps": fps, "lat": lat, "lost": res.lost, "frames": len(arr)}

    async def main():
        return await asyncio.gather(*(one(p) for p in ports))

    out = asyncio.run(main())
    ru = resource.getrusage(resource.RUSAGE_SELF)
    for r in out:  # this client process's CPU seconds, on its first result
        r["client_cpu_s"] = 0.0
    if out:
        out[0]["client_cpu_s"] = ru.ru_utime + ru.ru_stime
    q.put(out)


def run_k(k, frames, per_proc, width, height, codec_env, server_procs=1, log_dir="", lite=False):
    import multiprocessing as mp

    base = _free_port_block(k)
    env = dict(os.environ, PYTHONPATH=str(ROOT), WEBRTC_ENCODER=codec_env, SIZEW=str(width), SIZEH=str(height),
               REFRESH="60", ENABLE_BASIC_AUTH="false", SELKIES_ENABLE_AUDIO="false", MXDESK_GAMEPAD="false",
               MXDESK_SOURCE="synthetic", MXDESK_WEBRTC_HOST="127.0.0.1", MXDESK_SELKIES_PEER="false")
    # K sessions over `server_procs` serve processes on the same GPU (one event loop each: a single
    # loop's WebRTC stack -- DTLS, SRTP, SCTP timers, pacing -- saturated near 48 viewers)
    n_srv = max(1, min(server_procs, k))
    split = [k // n_srv + (1 if i < k % n_srv else 0) for i in range(n_srv)]
    srvs, at = [], base
    logs = []
    for j, n in enumerate(split):
        out = subprocess.DEVNULL
        if log_dir:
            Path(log_dir).mkdir(parents=True, exist_ok=True)
            out = open(Path(log_dir) / f"serve_k{k}_{j}_port{at}.log", "w")
            logs.append(out)
        srvs.append(subprocess.Popen([sys.executable, "-m", "mxdesk", "serve", "--port", str(at), "--sessions", str(n)],
                                     cwd=ROOT, env=env, stdout=out, stderr=subprocess.STDOUT, text=True))
        at += n
    try:
        ports = [base + i for i in range(k)]
        _wait_ready(ports)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        groups = [ports[i:i + per_proc] for i in range(0, k, per_proc)]
        procs = [ctx.Process(target=_client_proc, args=(g, frames, q, lite)) for g in groups]
        def server_cpu_s():
            tot = 0.0
            for srv in srvs:
                try:
                    ct = psutil.Process(srv.pid).cpu_times()
                    tot += ct.user + ct.system
                except psutil.Error:
                    pass
            return tot

        cpu0 = server_cpu_s()
        t_clients = time.monotonic()
        for p in procs:
            p.start()
        results = []
        for _ in procs:
            results += q.get(timeout=frames / 30.0 + 240)
        for p in procs:
            p.join(timeout=30)
        t_run = time.monotonic() - t_clients
        server_cpu = server_cpu_s() - cpu0
    finally:
        for srv in srvs:
            srv.terminate()
        for srv in srvs:
            try:
                srv.wait(timeout=30)
            except subprocess.TimeoutExpired:
                srv.kill()
        for f in logs:
            f.close()
    errs = [r for r in results if "error" in r]
    ok = [r for r in results if "error" not in r]
    lat = sorted(v for r in ok for v in r["lat"])
    p95 = lat[int(0.95 * (len(lat) - 1))] if lat else float("inf")
    p50 = statistics.median(lat) if lat else float("inf")
    fps = [r["fps"] for r in ok]
    passed = not errs and len(ok) == k and min(fps) >= 59.5 and p95 < 5.0
    return {"k": k, "passed": passed, "min_fps": round(min(fps), 2) if fps else 0.0,
            "mean_fps": round(statistics.mean(fps), 2) if fps else 0.0, "p50_e2e_ms": round(p50, 3),
            "p95_e2e_ms": round(p95, 3), "lost_packets": sum(r["lost"] for r in ok), "errors": [e["error"] for e in errs][:3],
            "failed_ports": sorted(e["port"] - base for e in errs), "failed_diag": [e.get("diag") for e in errs][:16],
            # host CPU: cores kept busy on average over the clients' run (ICE / DTLS set-up included)
            "cpus": len(os.sched_getaffinity(0)), "client_run_s": round(t_run, 2),
            "client_cores": round(sum(r.get("client_cpu_s", 0.0) for r in results) / max(t_run, 1e-6), 2),
            "server_cores": round(server_cpu / max(t_run, 1e-6), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", default="8,16,32")
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--per-proc", type=int, default=8, help="viewers per client process")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--encoder", default="mxh264enc")
    ap.add_argument("--server-procs", type=int, default=1, help="serve processes sharing the GPU (sessions split evenly)")
    ap.add_argument("--log-dir", default="", help="write each serve process's output here")
    ap.add_argument("--client", choices=["full", "lite", "native"], default="full",
                    help="viewer: full (decrypt + depacketise every packet), lite (frames from the plaintext RTP "
                         "headers; the server side is identical -- for K where the Python viewers saturate the host) "
                         "or native (the lite count by a native recvmmsg loop, GIL released)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    rows, sustained = [], 0
    for k in (int(v) for v in a.sweep.replace("+", ",").split(",")):
        r = run_k(k, a.frames, a.per_proc, a.width, a.height, a.encoder, a.server_procs, a.log_dir, {"full": False, "lite": True, "native": "native"}[a.client])
        r["server_procs"] = min(a.server_procs, k)
        r["client"] = a.client
        rows.append(r)
        print(json.dumps(r), flush=True)
        if not r["passed"]:
            break
        sustained = k
    out = {"metric": f"concurrent 1080p60 WebRTC sessions from {a.server_procs} serve process(es) on one GPU",
           "sustained": sustained, "server_procs": a.server_procs,
           "first_failing": rows[-1]["k"] if rows and not rows[-1]["passed"] else None, "frames_per_viewer": a.frames,
           "client": a.client,
           "criteria": "every viewer >= 59.5 fps and p95 capture->viewer latency < 5 ms", "runs": rows}
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        Path(a.json_out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.json_out).write_text(line + "\n")


if __name__ == "__main__":
    main()
