"""mxdesk -- MI355X-native GPU remote-desktop streaming stack.

Same capabilities as the NVIDIA GLX desktop container (COx2/docker-nvidia-glx-desktop):
an isolated per-GPU desktop session streamed to a browser on port 8080 (WebSocket /
WebRTC, noVNC-compatible RFB fallback), the same environment-variable interface, and
supervised processes -- with the per-frame pipeline (capture, colour conversion, scaling,
H.264 encode) in hand-written HIP kernels for gfx950.

Subpackages:
  codec     H.264 encoder front-end + pure-Python conformance decoder
  ops       Python wrappers of the HIP pixel kernels
  models    frame sources ("desktop models"): synthetic desktop, X11 capture
  pipeline  per-GPU session, frame pacing, metrics hooks
  parallel  session-per-GPU launcher, RCCL tiled video wall
  server    HTTP/WebSocket server, auth, signalling, TURN, RFB bridge
  display   Xorg config + CVT-RB modelines, display launcher
  utils     config schema, logging, metrics, supervisor, device discovery
"""
from __future__ import annotations

__version__ = "0.1.0"


def native():
    """Import the compiled extension (mxdesk/_native*.so); raises if it is missing.

    PyTorch-ROCm bundles its own libamdhip64 with the same SONAME as /opt/rocm's.  Whichever
    is loaded first serves the whole process, and torch's HIP initialisation fails when it
    finds the system runtime already bound ("No HIP GPUs are available"), so torch (when
    installed) is imported before the extension.
    """
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    from . import _native  # noqa: F401

    return _native
