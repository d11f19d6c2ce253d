#!/usr/bin/env bash
# BASELINE config "Single 4K60 HEVC session, HIP CSC+scale path": bench runs + kernel profile.
set -o pipefail
mkdir -p gpurun_out/hevc_bench
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/hevc_bench/$name.json 2> gpurun_out/hevc_bench/$name.err || { echo "bench $name failed"; tail -5 gpurun_out/hevc_bench/$name.err; exit 1; }; cat gpurun_out/hevc_bench/$name.json; }
b hevc4k --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 120 --warmup 20 &&
b hevc4k_d1 --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 120 --warmup 20 --depth 1 &&
b hevc1080 --codec hevc --bitrate-kbps 8000 --steps 200 --warmup 20 &&
b hevc8k_to_4k --codec hevc --width 7680 --height 4320 --out-width 3840 --out-height 2160 --bitrate-kbps 25000 --steps 60 --warmup 10 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hevc_bench/prof -o run -- python3 bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 60 --warmup 10 > gpurun_out/hevc_bench/prof.log 2>&1 || echo "rocprof rc=$?"
echo done
