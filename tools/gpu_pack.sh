#!/usr/bin/env bash
# Pack-kernel rewrite check: GPU tests (bit-exact vs CPU oracle), bench, kernel stats, PMC.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
bash tools/gpu_pmc.sh
