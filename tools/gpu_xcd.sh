#!/usr/bin/env bash
# XCD remap check: GPU tests (bit-exact vs CPU oracles), H.264 1080p + HEVC 4K benches, kernel stats.
set -o pipefail
mkdir -p gpurun_out/xcd
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/xcd/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/xcd/pytest_gpu.log; exit 1; }
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/xcd/bench_h264.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 200 --warmup 20 > gpurun_out/xcd/bench_hevc4k.log 2>&1 || { echo hevc bench failed; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xcd/prof -o h264 -- python3 bench.py --steps 100 --warmup 10 > gpurun_out/xcd/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xcd/prof -o hevc -- python3 bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 60 --warmup 10 > gpurun_out/xcd/prof_hevc.log 2>&1 || { echo "rocprof hevc failed"; exit 1; }
echo done
