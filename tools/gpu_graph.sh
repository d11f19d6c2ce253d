#!/usr/bin/env bash
# hipGraph replay: GPU tests, then bench graph vs eager launches, then profile of the graph path.
set -o pipefail
mkdir -p gpurun_out/graph
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit 1; }
for g in 0 1; do
  for k in 1 4; do
    timeout -k 10 300 python bench.py --steps 300 --warmup 30 --graph $g --sessions-per-gpu $k > gpurun_out/graph/g${g}_k${k}.json 2> gpurun_out/graph/g${g}_k${k}.err || { echo "bench g=$g k=$k failed"; exit 1; }
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
echo done
