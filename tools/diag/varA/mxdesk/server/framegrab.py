"""Raw desktop frames for the RFB/noVNC front end (which needs pixels, not H.264).

GPU backend: the HIP synthetic desktop renders into a device tensor and is copied to the
host; CPU backend: the numpy desktop; X11: the MIT-SHM capture.
"""
from __future__ import annotations

from typing import Any

import numpy as np

from ..models.synthetic import CpuSyntheticDesktop


class FrameGrabber:
    def __init__(self, width: int, height: int, fps: int, backend: str = "cpu", device: int = 0,
                 capture: Any = None, noise: bool = True):
        self.width, self.height, self.fps = width, height, fps
        self.backend, self.device, self.capture = backend, device, capture
        self.cursor = (-1, -1)
        self.frame_id = 0
        if capture is None and backend == "gpu":
            import torch

            from .. import native

            self.N = native()
            self.N.set_device(device)
            self.torch = torch
            self.pitch = (width * 4 + 255) // 256 * 256
            self.buf = torch.empty((height, self.pitch), dtype=torch.uint8, device=f"cuda:{device}")
        elif capture is None:
            self.desk = CpuSyntheticDesktop(width, height, noise)

    @classmethod
    def for_pipeline(cls, pipe: Any) -> "FrameGrabber":
        return cls(pipe.width, pipe.height, pipe.fps, pipe.backend, pipe.device, pipe.capture)

    def set_cursor(self, x: int, y: int) -> None:
        self.cursor = (x, y)

    def grab(self) -> np.ndarray:
        fid = self.frame_id
        self.frame_id += 1
        if self.capture is not None:
            return np.ascontiguousarray(self.capture.grab())
        if self.backend == "gpu":
            from .. import native

            st = self.torch.cuda.current_stream(self.buf.device).cuda_stream
            self.N.synth(self.buf.data_ptr(), self.width, self.height, self.pitch, fid, native().now_us() & 0xFFFFFFFF,
                         fid / self.fps, 1, 0, 0, self.width, self.height, self.cursor[0], self.cursor[1], st)
            host = self.buf.cpu().numpy()
            return host[:, : self.width * 4].reshape(self.height, self.width, 4)
        self.desk.cursor = self.cursor
        return self.desk.render(fid, fid / self.fps, 0)
