"""The serve-process stack sampler (mxdesk/utils/sampler.py, MXDESK_PYPROFILE): every thread's
stack sampled, self frames and the innermost mxdesk frame counted per thread name."""
import threading
import time

from mxdesk.utils.sampler import StackSampler


def _busy(stop):
    x = 0
    while not stop.is_set():
        x += 1


def test_sampler_counts_a_busy_thread():
    stop = threading.Event()
    t = threading.Thread(target=_busy, args=(stop,), name="busy-worker")
    s = StackSampler(interval_s=0.002).start()
    t.start()
    time.sleep(0.3)
    stop.set()
    t.join()
    rep = s.report()
    th = rep["threads"]
    assert "busy-worker" in th and th["busy-worker"]["samples"] > 20
    assert any("_busy" in k for k, _ in th["busy-worker"]["self_top"])
    assert rep["wall_s"] >= 0.3
