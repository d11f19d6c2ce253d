"""bench.py's multi-rank path rehearsed on the one GPU this tier has (VERDICT r2 "Next round" #5a).

The driver launches `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` on an
8-GPU node; that run is not ours to start.  Here two ranks share GPU 0 (gloo for the collectives,
so two processes on one device need no RCCL peer setup) and the JSON contract is checked: the
aggregate is 2 * steps over the slowest rank's elapsed time, latencies are gathered from both
ranks.  The ranks are fresh child processes started before anything in them touches the GPU."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_on_one_gpu_gloo():
    steps = 12
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=str(ROOT))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "bench.py"), "--gpus", "2",
           "--steps", str(steps), "--warmup", "3", "--backend", "gloo", "--density-probe", "0",
           "--width", "640", "--height", "360", "--bitrate-kbps", "2000"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == steps and out["config"]["global_batch"] == 2
    # value = total frames (both ranks) / the slowest rank's timed region
    assert out["value"] == pytest.approx(2 * steps / (out["ms_per_step"] * steps / 1000.0), rel=2e-3)
    assert out["encoded_fps_per_gpu"] == pytest.approx(out["value"] / 2, rel=1e-3)
    assert out["p50_e2e_latency_ms"] > 0 and out["p95_e2e_latency_ms"] >= out["p50_e2e_latency_ms"]
