#!/usr/bin/env bash
# Round-end style check: every GPU test, smoke, headline bench, kernel statistics.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo bench failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o run -- python3 bench.py --steps 100 --warmup 10 > gpurun_out/final/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log; tail -1 gpurun_out/final/smoke.log; cat gpurun_out/final/bench.json
echo done
