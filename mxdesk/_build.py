"""In-tree build of the native extension ``mxdesk/_native*.so`` for gfx950.

Every ``.hip``/``.cpp`` source under ``csrc/`` (except stand-alone probes) is compiled with
``hipcc --offload-arch=gfx950`` and linked into one pybind11 module that lives inside the
package, so the built ``.so`` travels with the repository snapshot to the GPU box.

Usage: ``python -m mxdesk._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shlex
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "obj"
ARCH = os.environ.get("MXDESK_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = ROOT / "mxdesk" / f"_native{EXT_SUFFIX}"
EXCLUDE_DIRS = {"probe", "tools"}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    return "hipcc"


def sources() -> list[Path]:
    out = []
    for p in sorted(CSRC.rglob("*")):
        if p.suffix not in (".hip", ".cpp"):
            continue
        if any(part in EXCLUDE_DIRS for part in p.relative_to(CSRC).parts[:-1]):
            continue
        out.append(p)
    return out


def _includes() -> list[str]:
    import pybind11

    return [
        f"-I{CSRC}",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
        "-I/usr/include/libdrm",
    ]


def _flags() -> list[str]:
    return [
        f"--offload-arch={ARCH}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-fvisibility=hidden",
        "-Wall",
        "-Wno-unused-function",
        "-Wno-unused-variable",
        "-Wno-unused-result",
    ]


# per-source extra flags: the scaler's MFMA accumulators in arch VGPRs (no AGPR copies
# around the f16 conversion between its two products; profiles/r02_scale)
_EXTRA = {"kernels/pixel.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _newest_header() -> float:
    return max((p.stat().st_mtime for p in CSRC.rglob("*.h")), default=0.0)


def _compile(src: Path, force: bool, hdr_mtime: float) -> tuple[Path, str]:
    obj = BUILD / (str(src.relative_to(CSRC)).replace("/", "__") + ".o")
    if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr_mtime):
        return obj, ""
    obj.parent.mkdir(parents=True, exist_ok=True)
    lang = ["-x", "hip"]
    extra = _EXTRA.get(str(src.relative_to(CSRC)), [])
    cmd = [_hipcc(), *lang, *_flags(), *extra, *_includes(), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {shlex.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    srcs = sources()
    hdr = _newest_header()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force, hdr), srcs))
    objs = [o for o, _ in results]
    if verbose:
        for o, err in results:
            if err.strip():
                print(f"[{o.name}] {err}", file=sys.stderr)
    newest = max(o.stat().st_mtime for o in objs)
    if force or not TARGET.exists() or TARGET.stat().st_mtime < newest:
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(TARGET),
               "-ldrm_amdgpu", "-ldrm", "-lssl", "-lcrypto", "-lz", "-lrocprofiler-sdk-roctx"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {shlex.join(cmd)}\n{r.stdout}\n{r.stderr}")
    build_interposer(force)
    return TARGET


INTERPOSER_SRC = CSRC / "interposer" / "js_interposer.c"
INTERPOSER = ROOT / "mxdesk" / "libmxjs_interposer.so"


def build_interposer(force: bool = False) -> Path:
    """Host-only LD_PRELOAD library (plain C, no HIP): the joystick interposer (C60)."""
    if force or not INTERPOSER.exists() or INTERPOSER.stat().st_mtime < INTERPOSER_SRC.stat().st_mtime:
        cc = os.environ.get("CC", "gcc")
        cmd = [cc, "-O2", "-fPIC", "-shared", "-Wall", "-o", str(INTERPOSER), str(INTERPOSER_SRC), "-ldl", "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"interposer build failed: {shlex.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return INTERPOSER


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.j, verbose=a.v))


if __name__ == "__main__":
    main()
