#!/usr/bin/env bash
# GPU tests, then encoder sweeps: ME range / subpel, scaled path (4K desktop -> 1080p encode),
# graph vs eager; kernel stats of the default and the scaled path; LDS counters of the scaler.
set -o pipefail
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit 1; }
b() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 300 --warmup 30 "$@" > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || { echo "bench $name failed"; exit 1; }; }
b default && b graph --graph 1 && b sr8 --search-range 8 && b sr32 --search-range 32 && b nosubpel --subpel 0 \
  && b scale4k_to_1080 --width 3840 --height 2160 --out-width 1920 --out-height 1080 \
  && b k4 --sessions-per-gpu 4 || exit 1
timeout -k 10 300 python tools/bench_e2e.py --frames 600 > gpurun_out/sweep/e2e.json 2> gpurun_out/sweep/e2e.err || { echo "e2e failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/prof.log 2>&1 || echo "rocprof failed rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_scale -o run -- python3 bench.py --steps 30 --warmup 5 --width 3840 --height 2160 --out-width 1920 --out-height 1080 > gpurun_out/prof_scale.log 2>&1 || echo "rocprof scale rc=$?"
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/pmc_scale -o run -- python3 bench.py --steps 10 --warmup 2 --width 3840 --height 2160 --out-width 1920 --out-height 1080 > gpurun_out/pmc_scale.log 2>&1 || echo "pmc scale rc=$?"
echo done
