#!/usr/bin/env bash
# ME rewrite check: GPU tests (bit-exact vs CPU oracle), default bench, kernel stats.
set -o pipefail
mkdir -p gpurun_out/me
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit 1; }
timeout -k 10 300 python bench.py --steps 400 --warmup 40 > gpurun_out/me/default.json 2> gpurun_out/me/default.err || exit 1
timeout -k 10 300 python bench.py --steps 400 --warmup 40 --depth 1 > gpurun_out/me/d1.json 2> gpurun_out/me/d1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 --depth 1 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
echo done
