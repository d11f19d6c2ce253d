"""Sampling profiler for a serve process (``MXDESK_PYPROFILE=<dir>``, VERDICT r5 next #8: name the
serving bound).  cProfile sees one thread; a serve process runs the event loop (WebRTC stack:
ICE, DTLS, SRTP, RTCP, pacing) on the main thread and one frame thread per session (encode
submit / collect, packetisation, sends).  A daemon thread samples every thread's stack
(``sys._current_frames``) every few milliseconds and counts, per thread, the innermost frame
(self time) and the innermost frame inside mxdesk (where mxdesk code spent it, native calls
included); per-thread CPU times come from the kernel (psutil).  Written as JSON at exit."""
from __future__ import annotations

import collections
import json
import os
import sys
import threading
import time


def _where(frame) -> str:
    co = frame.f_code
    return f"{os.path.basename(co.co_filename)}:{co.co_name}:{frame.f_lineno}"


class StackSampler:
    def __init__(self, interval_s: float = 0.005):
        self.interval = interval_s
        self.self_counts: dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
        self.mx_counts: dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
        self.samples: collections.Counter = collections.Counter()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="mxdesk-sampler", daemon=True)
        self.t0 = time.monotonic()

    def start(self) -> "StackSampler":
        self._t.start()
        return self

    def _run(self) -> None:
        me = threading.get_ident()
        while not self._stop.wait(self.interval):
            names = {t.ident: t.name for t in threading.enumerate()}
            for ident, frame in sys._current_frames().items():
                if ident == me:
                    continue
                name = names.get(ident, str(ident))
                self.samples[name] += 1
                self.self_counts[name][_where(frame)] += 1
                f = frame
                while f is not None and "mxdesk" not in f.f_code.co_filename:
                    f = f.f_back
                if f is not None:
                    self.mx_counts[name][_where(f)] += 1

    def report(self) -> dict:
        self._stop.set()
        out = {"wall_s": round(time.monotonic() - self.t0, 3), "interval_s": self.interval, "threads": {}}
        cpu = {}
        try:
            import psutil

            p = psutil.Process()
            cpu = {t.id: (t.user_time, t.system_time) for t in p.threads()}
            out["process_cpu_s"] = sum(p.cpu_times()[:2])
        except Exception:  # noqa: BLE001 -- the report is best effort
            pass
        natives = {t.ident: getattr(t, "native_id", None) for t in threading.enumerate()}
        names = {t.ident: t.name for t in threading.enumerate()}
        cpu_by_name = {}
        for ident, nid in natives.items():
            if nid in cpu:
                cpu_by_name[names[ident]] = [round(v, 3) for v in cpu[nid]]
        for name, n in self.samples.most_common():
            out["threads"][name] = {
                "samples": n,
                "cpu_user_sys_s": cpu_by_name.get(name),
                "self_top": self.self_counts[name].most_common(15),
                "mxdesk_top": self.mx_counts[name].most_common(15),
            }
        return out


def install_from_env() -> None:
    """Start the sampler when MXDESK_PYPROFILE names a directory; write
    <dir>/serve_<pid>.json at exit (SIGTERM included)."""
    d = os.environ.get("MXDESK_PYPROFILE", "")
    if not d:
        return
    import atexit
    import signal

    s = StackSampler().start()

    def dump() -> None:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"serve_{os.getpid()}.json"), "w") as f:
            json.dump(s.report(), f, indent=1)

    atexit.register(dump)

    def on_term(_sig, _frm):  # unwind asyncio.run like ^C, so atexit runs
        raise KeyboardInterrupt

    signal.signal(signal.SIGTERM, on_term)
