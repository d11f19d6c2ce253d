#!/usr/bin/env bash
# Density (sessions per GPU) and resolution sweep on one MI355X, plus a kernel profile.
set -o pipefail
mkdir -p gpurun_out/density
export TMPDIR=/tmp
for k in 1 2 4 8; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --sessions-per-gpu $k > gpurun_out/density/k$k.json 2> gpurun_out/density/k$k.err || { echo "density k=$k failed"; exit 1; }
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --width 3840 --height 2160 --bitrate-kbps 25000 > gpurun_out/density/4k.json 2> gpurun_out/density/4k.err || { echo "4k failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --width 7680 --height 4320 --bitrate-kbps 60000 > gpurun_out/density/8k.json 2> gpurun_out/density/8k.err || { echo "8k failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
echo done
