"""One-process-per-GPU rank launcher for commands that need a process group.

``mxdesk wall`` needs cols x rows ranks.  Under ``torchrun`` (WORLD_SIZE set) the ranks exist
already; started bare it used to initialise a one-rank group and crash in ``TileExchange``
(VERDICT r5 weak #3a).  ``run_ranks`` starts the ranks itself: fresh child processes of the same
command with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as ``torch.distributed.run`` sets them
(rendezvous on 127.0.0.1).  The parent never touches the GPU (nothing here imports torch or
HIP) and never execs: the children are started before any GPU call.

The parent polls every child: the first non-zero exit stops the others (a rank that dies before
or during ``init_process_group`` would leave the rest blocked in the rendezvous) and becomes the
return code; SIGTERM / SIGINT to the parent are forwarded, so a supervisor stopping the wall
stops all of its ranks.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Sequence


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket() as so:
        so.bind((addr, 0))
        return so.getsockname()[1]


def rank_env(rank: int, world: int, port: int, base: dict | None = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def run_ranks(cmd: Sequence[str], world: int, timeout_s: float | None = None, poll_s: float = 0.05) -> int:
    """Run ``cmd`` as ``world`` rank processes; return 0 when all exit 0, else the first failing
    code (124 after ``timeout_s``)."""
    port = free_port()
    procs = [subprocess.Popen(list(cmd), env=rank_env(r, world, port)) for r in range(world)]
    stopping = {"sig": None}

    def forward(sig, _frame):
        stopping["sig"] = sig

    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}

    def stop_all(sig=signal.SIGTERM) -> None:
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
        t_kill = time.monotonic() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_kill - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    deadline = None if timeout_s is None else time.monotonic() + timeout_s
    try:
        while True:
            if stopping["sig"] is not None:
                stop_all(stopping["sig"])
                return 128 + int(stopping["sig"])
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                print(f"mxdesk: a rank exited with {bad[0]}; stopping the others", file=sys.stderr, flush=True)
                stop_all()
                return bad[0]
            if all(c == 0 for c in codes):
                return 0
            if deadline is not None and time.monotonic() > deadline:
                print("mxdesk: ranks still running at the time limit; stopping them", file=sys.stderr, flush=True)
                stop_all()
                return 124
            time.sleep(poll_s)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
