"""Process supervisor (replaces supervisord, reference supervisord.conf).

Keeps the reference's model -- programs started in priority order, ``autorestart``,
``stopsignal``, logs in /tmp (supervisord.conf:5-43) -- and fixes the hazards the survey
found (§5.2):
  * readiness gates: a program may declare a probe (unix socket / TCP port / file) and
    later-priority programs wait for it, instead of three independent 1 s polls of the X
    socket (entrypoint.sh:117, supervisord.conf:24, selkies-gstreamer-entrypoint.sh:24);
  * every program runs in its own process group and is stopped with ``killpg`` (+ SIGKILL
    after ``stopwaitsecs``), so background children (Xorg, x11vnc, ...) cannot survive a
    restart of their parent;
  * restarts back off exponentially (reset after ``startsecs`` of healthy running) and a
    program that keeps failing before ``startsecs`` goes FATAL after ``startretries``.

It also reads supervisord-style INI files (``[program:x]`` sections, ``%(ENV_X)s``
interpolation), including the reference's own supervisord.conf.
"""
from __future__ import annotations

import configparser
import logging
import os
import shlex
import signal
import socket
import subprocess
import threading
import time
from dataclasses import dataclass, field
from enum import Enum
from pathlib import Path
from typing import Callable, Mapping

log = logging.getLogger("mxdesk.supervisor")


class State(str, Enum):
    STOPPED = "STOPPED"
    STARTING = "STARTING"
    RUNNING = "RUNNING"
    BACKOFF = "BACKOFF"
    EXITED = "EXITED"
    FATAL = "FATAL"


@dataclass
class Ready:
    kind: str          # "socket" (unix socket path exists), "tcp" (host:port accepts), "file", "none"
    target: str = ""
    timeout: float = 60.0

    def check(self) -> bool:
        if self.kind == "none":
            return True
        if self.kind in ("socket", "file"):
            return os.path.exists(self.target)
        if self.kind == "tcp":
            host, _, port = self.target.rpartition(":")
            try:
                with socket.create_connection((host or "127.0.0.1", int(port)), timeout=0.5):
                    return True
            except OSError:
                return False
        raise ValueError(f"unknown readiness probe {self.kind}")


@dataclass
class Program:
    name: str
    command: list[str]
    priority: int = 999
    autostart: bool = True
    autorestart: str = "true"       # "true" | "false" | "unexpected"
    exitcodes: tuple[int, ...] = (0,)
    startsecs: float = 1.0
    startretries: int = 3
    stopsignal: int = signal.SIGTERM
    stopwaitsecs: float = 10.0
    environment: dict[str, str] = field(default_factory=dict)
    directory: str | None = None
    logfile: str | None = None
    ready: Ready = field(default_factory=lambda: Ready("none"))
    wait_ready: bool = True         # block later priorities until ready
    backoff_max: float = 30.0


@dataclass
class ProcState:
    prog: Program
    state: State = State.STOPPED
    proc: subprocess.Popen | None = None
    started_at: float = 0.0
    fast_fails: int = 0
    restarts: int = 0
    next_start: float = 0.0
    backoff: float = 0.5
    exit_codes: list[int] = field(default_factory=list)


class Supervisor:
    def __init__(self, programs: list[Program], log_dir: str = "/tmp", poll: float = 0.1,
                 clock: Callable[[], float] = time.monotonic):
        self.programs = sorted(programs, key=lambda p: p.priority)
        self.log_dir = log_dir
        self.poll = poll
        self.clock = clock
        self.states = {p.name: ProcState(p) for p in self.programs}
        self._stop = threading.Event()
        self._lock = threading.Lock()

    # ------------------------------------------------------------------ process control
    def _spawn(self, ps: ProcState) -> None:
        p = ps.prog
        env = dict(os.environ)
        env.update(p.environment)
        logpath = p.logfile or os.path.join(self.log_dir, f"{p.name}.log")
        Path(os.path.dirname(logpath) or ".").mkdir(parents=True, exist_ok=True)
        out = open(logpath, "ab", buffering=0)
        try:
            ps.proc = subprocess.Popen(p.command, env=env, cwd=p.directory, stdout=out, stderr=subprocess.STDOUT,
                                       stdin=subprocess.DEVNULL, start_new_session=True)
        finally:
            out.close()
        ps.started_at = self.clock()
        ps.state = State.STARTING
        log.info("spawned %s pid=%d", p.name, ps.proc.pid)

    def _kill(self, ps: ProcState, timeout: float | None = None) -> None:
        proc = ps.proc
        if proc is None or proc.poll() is not None:
            return
        try:
            os.killpg(proc.pid, ps.prog.stopsignal)
        except ProcessLookupError:
            return
        try:
            proc.wait(timeout=ps.prog.stopwaitsecs if timeout is None else timeout)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            proc.wait()

    def _wait_ready(self, ps: ProcState) -> bool:
        deadline = self.clock() + ps.prog.ready.timeout
        while not self._stop.is_set() and self.clock() < deadline:
            if ps.proc is not None and ps.proc.poll() is not None:
                return False
            if ps.prog.ready.check():
                return True
            time.sleep(self.poll)
        return False

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        for p in self.programs:
            ps = self.states[p.name]
            if not p.autostart:
                continue
            self._spawn(ps)
            if p.wait_ready and p.ready.kind != "none":
                ok = self._wait_ready(ps)
                log.info("%s ready=%s", p.name, ok)

    def tick(self) -> None:
        """One supervision step: detect exits, schedule/perform restarts."""
        now = self.clock()
        with self._lock:
            for ps in self.states.values():
                p = ps.prog
                if ps.state in (State.STARTING, State.RUNNING) and ps.proc is not None:
                    rc = ps.proc.poll()
                    if rc is None:
                        if ps.state == State.STARTING and now - ps.started_at >= p.startsecs:
                            ps.state = State.RUNNING
                            ps.fast_fails = 0
                            ps.backoff = 0.5
                        continue
                    ps.exit_codes.append(rc)
                    ran = now - ps.started_at
                    expected = rc in p.exitcodes
                    if ran < p.startsecs:
                        ps.fast_fails += 1
                    log.info("%s exited rc=%s after %.2fs", p.name, rc, ran)
                    restart = p.autorestart == "true" or (p.autorestart == "unexpected" and not expected)
                    if ran < p.startsecs and ps.fast_fails > p.startretries:
                        ps.state = State.FATAL
                        log.error("%s: too many fast failures, FATAL", p.name)
                    elif restart and not self._stop.is_set():
                        ps.state = State.BACKOFF
                        ps.next_start = now + ps.backoff
                        ps.backoff = min(ps.backoff * 2, p.backoff_max)
                    else:
                        ps.state = State.EXITED
                elif ps.state == State.BACKOFF and now >= ps.next_start and not self._stop.is_set():
                    ps.restarts += 1
                    self._spawn(ps)

    def run(self, install_signals: bool = True) -> None:
        if install_signals:
            for sig in (signal.SIGTERM, signal.SIGINT):
                signal.signal(sig, lambda *_: self._stop.set())
        self.start()
        while not self._stop.is_set():
            self.tick()
            time.sleep(self.poll)
        self.stop()

    def stop(self) -> None:
        self._stop.set()
        for p in reversed(self.programs):
            ps = self.states[p.name]
            self._kill(ps)
            ps.state = State.STOPPED

    def status(self) -> dict[str, dict]:
        return {n: {"state": s.state.value, "pid": s.proc.pid if s.proc else None, "restarts": s.restarts,
                    "exit_codes": list(s.exit_codes)} for n, s in self.states.items()}


# ------------------------------------------------------------------ INI loading
_SIGNALS = {n[3:]: getattr(signal, n) for n in dir(signal) if n.startswith("SIG") and not n.startswith("SIG_")}


def _parse_env(s: str) -> dict[str, str]:
    out = {}
    for part in shlex.split(s.replace(",", " ")):
        k, _, v = part.partition("=")
        out[k.strip()] = v.strip().strip('"')
    return out


def load_ini(path: str | os.PathLike, env: Mapping[str, str] | None = None) -> tuple[list[Program], dict]:
    """Parse a supervisord-style config.  Returns (programs, [supervisord] section)."""
    env = os.environ if env is None else env
    defaults = {f"ENV_{k}": v.replace("%", "%%") for k, v in env.items()}
    cp = configparser.ConfigParser(interpolation=configparser.BasicInterpolation(), strict=False)
    cp.optionxform = str  # keep the case of %(ENV_X)s names
    cp.read_dict({"DEFAULT": defaults})
    text = Path(path).read_text()
    cp.read_string(text)
    progs = []
    for sec in cp.sections():
        if not sec.startswith("program:"):
            continue
        c = cp[sec]
        name = sec.split(":", 1)[1]
        cmd = shlex.split(c.get("command"))
        ready = Ready("none")
        if c.get("ready_socket", fallback=None):
            ready = Ready("socket", c.get("ready_socket"), float(c.get("ready_timeout", fallback="60")))
        elif c.get("ready_tcp", fallback=None):
            ready = Ready("tcp", c.get("ready_tcp"), float(c.get("ready_timeout", fallback="60")))
        logfile = c.get("stdout_logfile", fallback=None) or c.get("logfile", fallback=None)
        progs.append(Program(
            name=name,
            command=cmd,
            priority=int(c.get("priority", fallback="999")),
            autostart=c.get("autostart", fallback="true").lower() == "true",
            autorestart=c.get("autorestart", fallback="unexpected").lower(),
            exitcodes=tuple(int(x) for x in c.get("exitcodes", fallback="0").split(",")),
            startsecs=float(c.get("startsecs", fallback="1")),
            startretries=int(c.get("startretries", fallback="3")),
            stopsignal=_SIGNALS.get(c.get("stopsignal", fallback="TERM").upper(), signal.SIGTERM),
            stopwaitsecs=float(c.get("stopwaitsecs", fallback="10")),
            environment=_parse_env(c.get("environment", fallback="")),
            directory=c.get("directory", fallback=None),
            logfile=logfile,
            ready=ready,
        ))
    sup = dict(cp["supervisord"]) if cp.has_section("supervisord") else {}
    sup = {k: v for k, v in sup.items() if not k.startswith("ENV_")}
    return progs, sup


def main(argv: list[str] | None = None) -> None:
    import argparse

    ap = argparse.ArgumentParser(description="mxdesk process supervisor")
    ap.add_argument("-c", "--config", required=True)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    progs, sup = load_ini(a.config)
    Supervisor(progs, log_dir=os.path.dirname(sup.get("logfile", "/tmp/supervisord.log")) or "/tmp").run()


if __name__ == "__main__":
    main()
