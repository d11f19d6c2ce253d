"""Frame sources ("desktop models").

* ``GpuSyntheticDesktop`` -- the HIP-rendered benchmark desktop (animated noise, glxgears-like
  gears, scrolling terminal, moving window, frame-id/timestamp barcode): SURVEY.md C40.
  Rendering happens inside the native session, so this class only documents/configures it.
* ``CpuSyntheticDesktop`` -- a numpy renderer of a simplified desktop with the same barcode,
  for the no-GPU plumbing configuration (BASELINE.json config 1).
* barcode helpers shared by clients/tests: 64 bits (frame id, capture timestamp) in two rows
  of 32 8x8 cells at (8, 8).
"""
from __future__ import annotations

import numpy as np

BAR_CELL = 8
BAR_X = 8
BAR_Y = 8


def read_barcode(y_plane: np.ndarray, cell: int = BAR_CELL, bx: int = BAR_X, by: int = BAR_Y) -> tuple[int, int]:
    """Decode (frame_id, timestamp_us & 0xffffffff) from a decoded luma plane."""
    vals = []
    for row in range(2):
        v = 0
        for i in range(32):
            cx, cy = bx + i * cell + cell // 2, by + row * cell + cell // 2
            v = (v << 1) | int(y_plane[cy, cx] > 128)
        vals.append(v)
    return vals[0], vals[1]


def draw_barcode(bgrx: np.ndarray, frame_id: int, ts: int) -> None:
    h, w = bgrx.shape[:2]
    x0, y0 = BAR_X - BAR_CELL, BAR_Y - BAR_CELL
    x1, y1 = min(w, BAR_X + 33 * BAR_CELL), min(h, BAR_Y + 3 * BAR_CELL)
    bgrx[y0:y1, x0:x1, :3] = 96
    for row, word in enumerate((frame_id & 0xFFFFFFFF, ts & 0xFFFFFFFF)):
        for i in range(32):
            bit = (word >> (31 - i)) & 1
            ys, xs = BAR_Y + row * BAR_CELL, BAR_X + i * BAR_CELL
            if xs + BAR_CELL <= w and ys + BAR_CELL <= h:
                bgrx[ys: ys + BAR_CELL, xs: xs + BAR_CELL, :3] = 255 if bit else 0


def bgrx_to_nv12(bgrx: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """BT.709 limited-range integer CSC, same coefficients as the HIP kernel."""
    b = bgrx[..., 0].astype(np.int32)
    g = bgrx[..., 1].astype(np.int32)
    r = bgrx[..., 2].astype(np.int32)
    y = ((47 * r + 157 * g + 16 * b + 128) >> 8) + 16

    def avg(c):
        return (c[0::2, 0::2] + c[0::2, 1::2] + c[1::2, 0::2] + c[1::2, 1::2] + 2) >> 2

    ra, ga, ba = avg(r), avg(g), avg(b)
    u = ((-26 * ra - 86 * ga + 112 * ba + 128) >> 8) + 128
    v = ((112 * ra - 102 * ga - 10 * ba + 128) >> 8) + 128
    uv = np.empty((y.shape[0] // 2, y.shape[1]), np.uint8)
    uv[:, 0::2] = u
    uv[:, 1::2] = v
    return y.astype(np.uint8), uv


class CpuSyntheticDesktop:
    """Cheap numpy desktop for the CPU plumbing path (720p30 target)."""

    def __init__(self, width: int, height: int, noise: bool = True):
        self.w, self.h = width, height
        self.noise = noise
        yy, xx = np.mgrid[0:height, 0:width]
        bg = np.zeros((height, width, 4), np.uint8)
        bg[..., 0] = (90 + 110 * (1 - yy / height * 0.5)).astype(np.uint8)
        bg[..., 1] = (40 + 60 * yy / height).astype(np.uint8)
        bg[..., 2] = (20 + 40 * yy / height).astype(np.uint8)
        bg[..., 3] = 255
        # static "document" window
        x0, y0, ww, wh = int(width * .25), int(height * .52), int(width * .24), int(height * .36)
        bg[y0:y0 + wh, x0:x0 + ww, :3] = 248
        rng = np.random.default_rng(1)
        for row in range(y0 + 16, y0 + wh - 14, 14):
            n = int(rng.integers(10, 40))
            bg[row:row + 8, x0 + 8:min(x0 + ww - 8, x0 + 8 + n * 6), :3] = 30
        self.bg = bg
        self.rng = np.random.default_rng(7)
        self.cursor = (-1, -1)

    def render(self, frame_id: int, t: float, ts_us: int) -> np.ndarray:
        img = self.bg.copy()
        w, h = self.w, self.h
        mw, mh = max(48, w // 8), max(32, h // 8)
        wx = int(w * .5 + w * .18 * np.sin(t * .7)) - mw // 2
        wy = int(h * .62 + h * .12 * np.sin(t * 1.1)) - mh // 2
        img[max(0, wy):wy + mh, max(0, wx):wx + mw, 0] = 120
        img[max(0, wy):wy + mh, max(0, wx):wx + mw, 1] = 200
        img[max(0, wy):wy + mh, max(0, wx):wx + mw, 2] = 230
        img[max(0, wy):wy + 10, max(0, wx):wx + mw, :3] = (200, 90, 40)
        if self.noise:
            x0, y0 = int(w * .04), int(h * .55)
            nw, nh = int(w * .08), int(h * .11)
            img[y0:y0 + nh, x0:x0 + nw, :3] = self.rng.integers(0, 256, (nh, nw, 1), dtype=np.uint8)
        cx, cy = self.cursor
        if cx >= 0:
            img[cy:cy + 12, cx:cx + 2, :3] = 255
        draw_barcode(img, frame_id, ts_us)
        return img
