"""Minimal PNG writer (RGBA 8-bit, zlib) for remote-cursor images; libpng headers are not in
the image and the cursors are tiny (<= 64x64), so Python + zlib is enough."""
from __future__ import annotations

import struct
import zlib

import numpy as np


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack("!I", len(data)) + tag + data + struct.pack("!I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def encode_rgba(img: np.ndarray, level: int = 6) -> bytes:
    """(H, W, 4) uint8 RGBA -> PNG bytes (filter type 0 on every row)."""
    img = np.ascontiguousarray(img, np.uint8)
    if img.ndim != 3 or img.shape[2] != 4:
        raise ValueError("expected an (H, W, 4) RGBA array")
    h, w = img.shape[:2]
    raw = np.concatenate([np.zeros((h, 1), np.uint8), img.reshape(h, w * 4)], axis=1).tobytes()
    ihdr = struct.pack("!IIBBBBB", w, h, 8, 6, 0, 0, 0)
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", zlib.compress(raw, level)) + _chunk(b"IEND", b"")
