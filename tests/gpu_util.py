"""Helpers for GPU tests: device buffers via PyTorch-ROCm tensors."""
import numpy as np
import torch


def to_dev(arr: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(arr)).to("cuda")


def pitched(arr: np.ndarray, pitch: int, rows: int, uv: bool = False) -> torch.Tensor:
    """Copy a (h, w) uint8 plane into a (rows, pitch) device tensor, replicating the last
    column (last U/V pair for an interleaved chroma plane) and row like the CSC kernel."""
    out = np.zeros((rows, pitch), np.uint8)
    out[: arr.shape[0], : arr.shape[1]] = arr
    if arr.shape[1] < pitch:
        if uv:
            reps = (pitch - arr.shape[1]) // 2
            out[: arr.shape[0], arr.shape[1]: arr.shape[1] + 2 * reps] = np.tile(arr[:, -2:], (1, reps))
        else:
            out[: arr.shape[0], arr.shape[1]:] = arr[:, -1:]
    if arr.shape[0] < rows:
        out[arr.shape[0]:] = out[arr.shape[0] - 1]
    return to_dev(out)


def bt709_nv12_reference(bgrx: np.ndarray):
    """Float BT.709 limited-range reference (H, W, 4 BGRx) -> (Y, U, V) float arrays."""
    b = bgrx[..., 0].astype(np.float64)
    g = bgrx[..., 1].astype(np.float64)
    r = bgrx[..., 2].astype(np.float64)
    y = 16 + (0.2126 * r + 0.7152 * g + 0.0722 * b) * 219.0 / 255.0
    def avg(c):
        return (c[0::2, 0::2] + c[0::2, 1::2] + c[1::2, 0::2] + c[1::2, 1::2]) / 4.0
    ra, ga, ba = avg(r), avg(g), avg(b)
    ya = 0.2126 * ra + 0.7152 * ga + 0.0722 * ba
    u = 128 + (ba - ya) / 1.8556 * 224.0 / 255.0
    v = 128 + (ra - ya) / 1.5748 * 224.0 / 255.0
    return y, u, v
