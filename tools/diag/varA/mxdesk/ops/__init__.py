"""Torch-tensor front ends for the hand-written HIP pixel kernels (csrc/kernels/pixel.hip).

Every op validates shapes/strides/devices on the host BEFORE launching (a bad pitch would
make the kernel read or write out of bounds), enqueues on the current torch HIP stream, and
fails loudly if the native extension is missing -- there is no eager fallback.

Reference parity: these replace the GStreamer elements of the reference's selkies pipeline
(ximagesrc -> cudaupload -> cudaconvert/cudascale -> nvh264enc; Dockerfile:439-444), see
SURVEY.md C52/C56.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import native

__all__ = ["synth_desktop", "bgrx_to_nv12", "scale_to_nv12", "composite", "alloc_nv12", "lanczos_tables"]


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check_gpu_u8(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.dtype != torch.uint8:
        raise ValueError(f"{name} must be uint8")


def _pitch(t: torch.Tensor, bpp: int, name: str) -> int:
    """Row pitch in bytes of a [H, W*bpp] / [H, W, bpp] tensor whose rows may be padded."""
    if t.dim() == 3:
        if t.stride(2) != 1 or t.stride(1) != t.size(2):
            raise ValueError(f"{name}: pixels must be contiguous")
        return t.stride(0)
    if t.dim() == 2:
        if t.stride(1) != 1:
            raise ValueError(f"{name}: rows must be contiguous")
        return t.stride(0)
    raise ValueError(f"{name}: expected a 2-D or 3-D tensor")


def alloc_nv12(width: int, height: int, device=None, pitch: Optional[int] = None):
    """(Y [H, pitch], UV [H/2, pitch]) uint8 planes; pitch defaults to width rounded up to 64."""
    pitch = pitch or ((width + 63) // 64) * 64
    dev = device or torch.device("cuda", torch.cuda.current_device())
    return (torch.empty(height, pitch, dtype=torch.uint8, device=dev),
            torch.empty(height // 2, pitch, dtype=torch.uint8, device=dev))


def synth_desktop(out: torch.Tensor, frame_id: int = 0, timestamp_us: int = 0, t: float = 0.0, noise: bool = True,
                  origin=(0, 0), wall=(0, 0), cursor=(-1, -1)) -> torch.Tensor:
    """Render the synthetic desktop (BGRX, [H, W, 4]) with the frame-id/timestamp barcode."""
    _check_gpu_u8(out, "out")
    h, w = out.shape[0], out.shape[1]
    pitch = _pitch(out, 4, "out")
    if pitch % 16:
        raise ValueError("out pitch must be a multiple of 16 bytes")
    native().synth(out.data_ptr(), w, h, pitch, frame_id=frame_id, timestamp_us=timestamp_us & 0xFFFFFFFF, t=t,
                   noise=int(noise), origin_x=origin[0], origin_y=origin[1], wall_w=wall[0], wall_h=wall[1],
                   cursor_x=cursor[0], cursor_y=cursor[1], stream=_stream())
    return out


def bgrx_to_nv12(bgrx: torch.Tensor, y: Optional[torch.Tensor] = None, uv: Optional[torch.Tensor] = None,
                 coded=None):
    """BT.709 limited-range BGRX -> NV12 (fused 2x2 chroma average); pads to ``coded`` (w, h)
    by edge replication so the encoder sees MB-aligned planes."""
    _check_gpu_u8(bgrx, "bgrx")
    h, w = bgrx.shape[0], bgrx.shape[1] // (4 if bgrx.dim() == 2 else 1)
    in_pitch = _pitch(bgrx, 4, "bgrx")
    cw, ch = coded or (w, h)
    if y is None:
        y, uv = alloc_nv12(cw, ch, bgrx.device)
    _check_gpu_u8(y, "y")
    _check_gpu_u8(uv, "uv")
    op = _pitch(y, 1, "y")
    if _pitch(uv, 1, "uv") != op or y.shape[0] < ch or uv.shape[0] < ch // 2 or op < cw:
        raise ValueError("NV12 planes too small for the coded size")
    native().bgrx_to_nv12(bgrx.data_ptr(), in_pitch, w, h, y.data_ptr(), uv.data_ptr(), op, cw, ch, _stream())
    return y, uv


_tables: dict = {}


def lanczos_tables(in_w: int, in_h: int, out_w: int, out_h: int, device):
    key = (in_w, in_h, out_w, out_h, str(device))
    if key not in _tables:
        N = native()
        sx, wx, tx = N.lanczos_table(in_w, out_w)
        sy, wy, ty = N.lanczos_table(in_h, out_h)
        _tables[key] = tuple(torch.from_numpy(a).to(device) for a in (sx, wx, sy, wy)) + (tx, ty)
    return _tables[key]


def scale_to_nv12(bgrx: torch.Tensor, out_w: int, out_h: int, y: Optional[torch.Tensor] = None,
                  uv: Optional[torch.Tensor] = None, coded=None):
    """Fused separable Lanczos-3 resample + BT.709 CSC, BGRX [H, W, 4] -> NV12 (out_w x out_h)."""
    _check_gpu_u8(bgrx, "bgrx")
    h, w = bgrx.shape[0], bgrx.shape[1] // (4 if bgrx.dim() == 2 else 1)
    in_pitch = _pitch(bgrx, 4, "bgrx")
    cw, ch = coded or (out_w, out_h)
    if y is None:
        y, uv = alloc_nv12(cw, ch, bgrx.device)
    op = _pitch(y, 1, "y")
    if _pitch(uv, 1, "uv") != op or y.shape[0] < ch or uv.shape[0] < ch // 2 or op < cw:
        raise ValueError("NV12 planes too small for the coded size")
    sx, wx, sy, wy, tx, ty = lanczos_tables(w, h, out_w, out_h, bgrx.device)
    native().scale_to_nv12(bgrx.data_ptr(), in_pitch, w, h, out_w, out_h, sx.data_ptr(), wx.data_ptr(), tx,
                           sy.data_ptr(), wy.data_ptr(), ty, y.data_ptr(), uv.data_ptr(), op, cw, ch, _stream())
    return y, uv


def composite(tile: torch.Tensor, dst: torch.Tensor, dx: int, dy: int) -> torch.Tensor:
    """Copy a BGRX ``tile`` [th, tw, 4] into ``dst`` [H, W, 4] at pixel (dx, dy) (wall
    assembly; bounds and 16-byte row alignment are checked on the host)."""
    _check_gpu_u8(tile, "tile")
    _check_gpu_u8(dst, "dst")
    if tile.dim() != 3 or dst.dim() != 3 or tile.size(2) != 4 or dst.size(2) != 4:
        raise ValueError("composite expects BGRX [H, W, 4] tensors")
    th, tw = tile.shape[:2]
    if dx < 0 or dy < 0 or dx + tw > dst.shape[1] or dy + th > dst.shape[0]:
        raise ValueError("tile does not fit in dst")
    tp, dp = _pitch(tile, 4, "tile"), _pitch(dst, 4, "dst")
    if tp % 16 or dp % 16 or tile.data_ptr() % 16 or dst.data_ptr() % 16:
        raise ValueError("composite needs 16-byte aligned rows")
    native().composite(tile.data_ptr(), tp, tw, th, dst.data_ptr(), dp, dx, dy, _stream())
    return dst
