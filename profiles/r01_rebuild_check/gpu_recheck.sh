#!/usr/bin/env bash
# Re-measure the non-default BASELINE configs after a rebuild: 4K HEVC, 4 sessions/GPU 1080p H.264,
# 8K desktop -> 4K HEVC.
set -o pipefail
mkdir -p gpurun_out/recheck
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/recheck/$name.json 2> gpurun_out/recheck/$name.err || { echo "bench $name failed"; tail -5 gpurun_out/recheck/$name.err; exit 1; }; cat gpurun_out/recheck/$name.json; }
b hevc4k --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 120 --warmup 12 \
 && b h264_k4 --steps 400 --warmup 40 --depth 1 --sessions-per-gpu 4 \
 && b hevc8k_to_4k --codec hevc --width 7680 --height 4320 --out-width 3840 --out-height 2160 --bitrate-kbps 25000 --steps 60 --warmup 6
