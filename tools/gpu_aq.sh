#!/usr/bin/env bash
# AQ + ME early-exit check: GPU tests, bench (default, no-noise, depth 1), kernel stats.
set -o pipefail
mkdir -p gpurun_out/aq
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit 1; }
b() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 400 --warmup 40 "$@" > gpurun_out/aq/$name.json 2> gpurun_out/aq/$name.err || { echo "bench $name failed"; exit 1; }; }
b default && b d1 --depth 1 && b nonoise --noise 0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 --depth 1 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
echo done
