#!/usr/bin/env bash
# First GPU pass: tests, smoke, short bench, rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import mxdesk; print(mxdesk.native().device_name(0))" > gpurun_out/dev.txt 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
# test failures (rc 1) still allow the bench; a crash/timeout/abort ends the call here
[ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python bench.py --steps 120 --warmup 20 > gpurun_out/bench.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
echo done
