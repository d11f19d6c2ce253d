#!/usr/bin/env bash
# Hardware/environment probes. Writes gpurun_out/probe/*.txt
# Usage on the GPU box: bash tools/probe_hw.sh
set -u
OUT=gpurun_out/probe
mkdir -p "$OUT"
{
  echo "## dev nodes"; ls -la /dev/dri /dev/kfd 2>&1
  echo "## /sys/class/drm"; ls /sys/class/drm 2>&1
  echo "## connectors"; for c in /sys/class/drm/card*-*; do [ -e "$c" ] && echo "$c $(cat $c/status 2>/dev/null)"; done
  echo "## groups"; id
} > "$OUT/devnodes.txt" 2>&1
gcc -O2 -o /tmp/vcn_caps csrc/probe/vcn_caps.c -I/usr/include/libdrm -ldrm_amdgpu -ldrm 2>/dev/null && \
  timeout -k 5 30 /tmp/vcn_caps > "$OUT/vcn_caps.json" 2>&1
timeout -k 5 60 rocminfo > "$OUT/rocminfo.txt" 2>&1
timeout -k 5 60 amd-smi static > "$OUT/amdsmi_static.txt" 2>&1
timeout -k 5 60 amd-smi topology > "$OUT/amdsmi_topology.txt" 2>&1
{
  echo "## radeonsi gfx950 strings"; for f in /usr/lib/x86_64-linux-gnu/dri/radeonsi_dri.so /usr/lib/x86_64-linux-gnu/libgallium*.so; do [ -e "$f" ] && echo "$f: $(strings "$f" | grep -ci gfx950)"; done
  echo "## tools"; for t in Xorg Xvfb x11vnc ffmpeg gst-launch-1.0 vainfo cvt xcvt; do echo "$t: $(command -v $t || echo absent)"; done
  echo "## python"; python3 -c "import importlib;[print(m, bool(importlib.util.find_spec(m))) for m in ['cv2','av','aiortc','PIL','aiohttp','torch']]"
  echo "## cpu"; nproc; grep -m1 "model name" /proc/cpuinfo; free -g
} > "$OUT/env.txt" 2>&1
echo probes-done
