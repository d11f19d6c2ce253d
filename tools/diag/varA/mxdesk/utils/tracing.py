"""roctx ranges from Python: ``with trace("mxdesk.webrtc.send"): ...`` shows
up in ``rocprofv3 --marker-trace`` next to the HIP kernels of the same frame."""
from __future__ import annotations

from contextlib import contextmanager


@contextmanager
def trace(name: str):
    from .. import native

    N = native()
    N.trace_push(name)
    try:
        yield
    finally:
        N.trace_pop()
