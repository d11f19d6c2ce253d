"""GPU discovery and selection (replaces nvidia-smi use in the reference).

The reference picks the first GPU UUID from ``nvidia-smi`` when ``NVIDIA_VISIBLE_DEVICES``
is ``all``/unset, else the first listed id (entrypoint.sh:70-79), exits if none is found
(entrypoint.sh:81-84), and converts the hexadecimal PCI bus id into Xorg's decimal
``PCI:b:d:f`` form (entrypoint.sh:94-98).

Here devices come from sysfs (vendor 0x1002 render nodes under /sys/class/drm), with the
KFD topology for NUMA node and xGMI peer links, filtered by ``HIP_VISIBLE_DEVICES`` /
``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` / ``AMD_VISIBLE_DEVICES`` and chosen by
``GPU_SELECT`` / ``MXDESK_GPU`` (index, PCI bus id or unique id).  ``sysfs_root`` lets
tests run against a fake tree.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field
from pathlib import Path
from typing import Mapping, Sequence

AMD_VENDOR = "0x1002"
XGMI_LINK_TYPE = 11  # KFD io_link type for xGMI


@dataclass
class GpuDevice:
    index: int               # enumeration order (sorted by PCI address)
    pci_bdf: str             # e.g. "0000:0a:00.0"
    device_id: str           # e.g. "0x75a3"
    render_node: str         # e.g. "/dev/dri/renderD136"
    card: str = ""           # e.g. "card8"
    numa_node: int = -1
    unique_id: str = ""
    kfd_node: int = -1
    xgmi_peers: list[int] = field(default_factory=list)  # kfd node ids reachable over xGMI
    gfx_target: str = ""

    @property
    def xorg_busid(self) -> str:
        return pci_to_xorg_busid(self.pci_bdf)


def pci_to_xorg_busid(bdf: str) -> str:
    """'0000:0a:00.0' (hex, as nvidia-smi/sysfs report) -> 'PCI:10:0:0' (decimal, Xorg)."""
    m = re.fullmatch(r"(?:([0-9a-fA-F]+):)?([0-9a-fA-F]+):([0-9a-fA-F]+)\.([0-9a-fA-F]+)", bdf.strip())
    if not m:
        raise ValueError(f"bad PCI bus id: {bdf!r}")
    _, bus, dev, fn = m.groups()
    return f"PCI:{int(bus, 16)}:{int(dev, 16)}:{int(fn, 16)}"


def _read(p: Path, default: str = "") -> str:
    try:
        return p.read_text().strip()
    except OSError:
        return default


def _kfd_nodes(root: Path) -> dict[str, tuple[int, list[int], str]]:
    """Map PCI location_id -> (kfd node id, xgmi peer node ids, gfx target)."""
    out: dict[str, tuple[int, list[int], str]] = {}
    nodes = root / "class/kfd/kfd/topology/nodes"
    if not nodes.is_dir():
        return out
    for nd in sorted(nodes.iterdir(), key=lambda p: int(p.name) if p.name.isdigit() else 1 << 30):
        props = {}
        for line in _read(nd / "properties").splitlines():
            parts = line.split()
            if len(parts) == 2:
                props[parts[0]] = parts[1]
        if props.get("simd_count", "0") == "0":
            continue  # CPU node
        loc = int(props.get("location_id", "0"))
        domain = int(props.get("domain", "0"))
        bdf = f"{domain:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        peers = []
        links = nd / "io_links"
        if links.is_dir():
            for ln in links.iterdir():
                lp = {}
                for line in _read(ln / "properties").splitlines():
                    parts = line.split()
                    if len(parts) == 2:
                        lp[parts[0]] = parts[1]
                if int(lp.get("type", "0")) == XGMI_LINK_TYPE:
                    peers.append(int(lp.get("node_to", "-1")))
        gfx = props.get("gfx_target_version", "")
        out[bdf] = (int(nd.name), sorted(peers), gfx)
    return out


def enumerate_gpus(sysfs_root: str | os.PathLike = "/sys", dev_root: str | os.PathLike = "/dev") -> list[GpuDevice]:
    """All AMD GPUs whose render node exists under ``dev_root/dri``."""
    root = Path(sysfs_root)
    drm = root / "class/drm"
    found: dict[str, GpuDevice] = {}
    if not drm.is_dir():
        return []
    kfd = _kfd_nodes(root)
    for ent in sorted(drm.iterdir()):
        if not ent.name.startswith("renderD"):
            continue
        dev = ent / "device"
        if _read(dev / "vendor") != AMD_VENDOR:
            continue
        if not (Path(dev_root) / "dri" / ent.name).exists():
            continue
        try:
            bdf = os.path.basename(os.path.realpath(dev))
        except OSError:
            continue
        if not re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-9a-f]", bdf):
            bdf = _read(dev / "uevent").partition("PCI_SLOT_NAME=")[2].split("\n")[0] or bdf
        numa = _read(dev / "numa_node", "-1")
        g = GpuDevice(index=-1, pci_bdf=bdf, device_id=_read(dev / "device"),
                      render_node=str(Path(dev_root) / "dri" / ent.name),
                      numa_node=int(numa) if numa.lstrip("-").isdigit() else -1,
                      unique_id=_read(dev / "unique_id"))
        for c in drm.iterdir():
            if c.name.startswith("card") and "-" not in c.name:
                try:
                    if os.path.realpath(c / "device") == os.path.realpath(dev):
                        g.card = c.name
                except OSError:
                    pass
        if bdf in kfd:
            g.kfd_node, g.xgmi_peers, g.gfx_target = kfd[bdf]
        found[bdf] = g
    gpus = sorted(found.values(), key=lambda d: d.pci_bdf)
    for i, g in enumerate(gpus):
        g.index = i
    return gpus


VISIBLE_ENV = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "AMD_VISIBLE_DEVICES")


def visible_gpus(gpus: Sequence[GpuDevice], env: Mapping[str, str] | None = None) -> list[GpuDevice]:
    """Apply the *_VISIBLE_DEVICES filters (comma-separated indices, bus ids or unique ids;
    'all' or unset = everything), like NVIDIA_VISIBLE_DEVICES in the reference."""
    env = os.environ if env is None else env
    out = list(gpus)
    for name in VISIBLE_ENV:
        val = env.get(name)
        if val is None or val.strip().lower() in ("", "all"):
            continue
        sel = []
        for tok in val.split(","):
            tok = tok.strip()
            if not tok:
                continue
            d = _match(out, tok)
            if d is not None and d not in sel:
                sel.append(d)
        out = sel
    return out


def _match(gpus: Sequence[GpuDevice], tok: str) -> GpuDevice | None:
    if tok.isdigit():
        i = int(tok)
        return gpus[i] if i < len(gpus) else None
    t = tok.lower()
    for g in gpus:
        if t in (g.pci_bdf, g.pci_bdf[5:], g.unique_id.lower(), g.render_node, g.card) or (
                t.startswith("pci:") and t == g.xorg_busid.lower()):
            return g
    return None


class NoGpuError(RuntimeError):
    pass


def select_gpu(gpus: Sequence[GpuDevice], selector: str | None = None) -> GpuDevice:
    """First visible GPU, or the one named by GPU_SELECT/MXDESK_GPU (falls back to the first
    GPU when the selector does not match, like entrypoint.sh:75-77).  Raises NoGpuError
    when no GPU is visible (entrypoint.sh:81-84 exits 1)."""
    if not gpus:
        raise NoGpuError("No AMD GPUs detected (check /dev/kfd, /dev/dri and the render/video groups)")
    if selector:
        d = _match(gpus, selector.strip())
        if d is not None:
            return d
    return gpus[0]


def hip_device_index(dev: GpuDevice, all_gpus: Sequence[GpuDevice]) -> int:
    """HIP ordinal of ``dev`` when the process sees ``all_gpus`` (sorted by bus id)."""
    for i, g in enumerate(all_gpus):
        if g.pci_bdf == dev.pci_bdf:
            return i
    raise KeyError(dev.pci_bdf)


def gpu_telemetry(pci_bdf: str, sysfs_root: str | os.PathLike = "/sys") -> dict[str, float]:
    """amdgpu sysfs telemetry of one GPU (what ``amd-smi metric`` reports, read without the
    tool): busy %, VRAM used/total, power (W) and edge/junction temperature (deg C).  Missing
    files are simply absent from the result (e.g. inside containers without hwmon)."""
    dev = Path(sysfs_root) / "bus/pci/devices" / pci_bdf
    out: dict[str, float] = {}

    def num(path: Path) -> float | None:
        v = _read(path)
        try:
            return float(v)
        except ValueError:
            return None

    for key, name, scale in (("busy_percent", "gpu_busy_percent", 1.0), ("vram_used_bytes", "mem_info_vram_used", 1.0),
                             ("vram_total_bytes", "mem_info_vram_total", 1.0)):
        v = num(dev / name)
        if v is not None:
            out[key] = v * scale
    hw = dev / "hwmon"
    if hw.is_dir():
        for h in sorted(hw.iterdir()):
            for key, names, scale in (("power_watts", ("power1_average", "power1_input"), 1e-6),
                                      ("temperature_c", ("temp2_input", "temp1_input"), 1e-3)):
                if key in out:
                    continue
                for n in names:  # temp2 is the junction (hotspot) sensor on amdgpu, temp1 the edge
                    v = num(h / n)
                    if v is not None:
                        out[key] = v * scale
                        break
    return out
