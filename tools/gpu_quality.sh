#!/usr/bin/env bash
# GPU tests + bench with/without the noise panel (PSNR at the 8 Mbps operating point) + profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python bench.py --steps 240 --warmup 20 > gpurun_out/bench.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --steps 240 --warmup 20 --noise 0 > gpurun_out/bench_nonoise.log 2>&1 || { echo bench2 failed; exit 1; }
echo done
