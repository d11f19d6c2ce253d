"""Session-per-GPU launcher (SURVEY.md C57, §2.6 "DP" analogue).

The reference runs exactly one desktop per container/GPU and scales out with more pods
(xgl.yml:10, README.md:180-182).  Here one node serves N independent sessions, one per
visible MI355X: session i is pinned to GPU i with ``HIP_VISIBLE_DEVICES`` and listens on
``base_port + i``.  Children are run by the mxdesk supervisor (autorestart with backoff,
process-group kill, readiness = the HTTP port accepting connections).
"""
from __future__ import annotations

import os
import sys
from typing import Any

from ..utils.supervisor import Program, Ready, Supervisor


# Sessions per serving process: one event loop carries the WebRTC stack (ICE, DTLS, SRTP, SCTP
# timers, pacing) of its sessions; 4 processes x 16 sessions held 64 1080p60 viewers per GPU at
# p95 2.2 ms where one process topped out at 48 (profiles/r05_density/NOTES.md).
SESSIONS_PER_PROCESS = 16


def session_programs(n_gpus: int, base_port: int = 8080, extra_args: list[str] | None = None,
                     sessions_per_gpu: int = 1, python: str = sys.executable,
                     sessions_per_process: int = SESSIONS_PER_PROCESS) -> list[Program]:
    """`mxdesk serve` processes for every GPU: K sessions per GPU on ports base + K*gpu .., split
    over ceil(K / sessions_per_process) processes of that GPU (each `--sessions n`, one HIP context
    and one event loop), so a node is capped neither by a per-GPU process limit nor by one event
    loop's serving rate."""
    progs = []
    k = max(1, sessions_per_gpu)
    per = max(1, sessions_per_process)
    nproc = (k + per - 1) // per
    for gpu in range(n_gpus):
        port = base_port + k * gpu
        for j in range(nproc):
            n = k // nproc + (1 if j < k % nproc else 0)
            env = {"HIP_VISIBLE_DEVICES": str(gpu), "MXDESK_GPU": "0", "SELKIES_PORT": str(port),
                   "MXDESK_SESSION": str(gpu) if nproc == 1 else f"{gpu}.{j}"}
            cmd = [python, "-m", "mxdesk", "serve", "--port", str(port)]
            if k > 1:
                cmd += ["--sessions", str(n)]
            name = f"gpu{gpu}" + (f"-x{k}" if k > 1 else "") + (f"-p{j}" if nproc > 1 else "")
            progs.append(Program(name=name, command=cmd + list(extra_args or []), priority=10 + gpu,
                                 environment=env, ready=Ready("tcp", f"127.0.0.1:{port}", 120.0),
                                 wait_ready=False, startsecs=2.0, startretries=5))
            port += n
    return progs


def launch_sessions(cfg: Any, base_port: int = 8080, n_gpus: int | None = None, sessions_per_gpu: int = 1) -> None:
    from ..utils import devices as D

    if n_gpus is None:
        n_gpus = len(D.visible_gpus(D.enumerate_gpus())) or 1
    progs = session_programs(n_gpus, base_port, sessions_per_gpu=sessions_per_gpu)
    k = max(1, sessions_per_gpu)
    print(f"mxdesk launch: {n_gpus * k} session(s) in {len(progs)} process(es) on {n_gpus} GPU(s), ports "
          f"{base_port}..{base_port + n_gpus * k - 1}", flush=True)
    Supervisor(progs, log_dir=getattr(cfg, "log_dir", "/tmp")).run()


if __name__ == "__main__":
    os.environ.setdefault("PYTHONUNBUFFERED", "1")
