#!/usr/bin/env bash
# Pipelined encode check: GPU tests, bench depth 1 vs 2 (1 and 4 sessions), kernel stats at depth 2.
set -o pipefail
mkdir -p gpurun_out/depth
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit 1; }
b() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 400 --warmup 40 "$@" > gpurun_out/depth/$name.json 2> gpurun_out/depth/$name.err || { echo "bench $name failed"; exit 1; }; }
b d1 && b d2 --depth 2 && b d1k4 --sessions-per-gpu 4 && b d2k4 --depth 2 --sessions-per-gpu 4 && b d2k2 --depth 2 --sessions-per-gpu 2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 --depth 2 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
echo done
