#!/usr/bin/env bash
# GPU tests + default / no-subpel / scaled bench + kernel stats for both paths.
set -o pipefail
mkdir -p gpurun_out/quick
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit 1; }
b() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 300 --warmup 30 "$@" > gpurun_out/quick/$name.json 2> gpurun_out/quick/$name.err || { echo "bench $name failed"; exit 1; }; }
b default && b nosubpel --subpel 0 && b scale4k_to_1080 --width 3840 --height 2160 --out-width 1920 --out-height 1080 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_scale -o run -- python3 bench.py --steps 30 --warmup 5 --width 3840 --height 2160 --out-width 1920 --out-height 1080 > gpurun_out/prof_scale.log 2>&1 || echo "rocprof scale rc=$?"
echo done
