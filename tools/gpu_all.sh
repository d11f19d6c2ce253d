#!/usr/bin/env bash
# Full GPU tier + HEVC/H.264 timings + kernel profile (stops at the first failing step).
set -o pipefail
mkdir -p gpurun_out/all
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/all/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/all/pytest.log
tail -3 gpurun_out/all/pytest.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; grep -E "FAILED|Error" gpurun_out/all/pytest.log | head; exit 1; }
timeout -k 10 120 python tools/hevc_quick.py 1920 1080 60 8000 > gpurun_out/all/hevc1080.txt 2>&1 || { echo "hevc 1080 failed"; exit 1; }
timeout -k 10 120 python tools/hevc_quick.py 3840 2160 40 25000 > gpurun_out/all/hevc2160.txt 2>&1 || { echo "hevc 4k failed"; exit 1; }
grep hevc gpurun_out/all/hevc*.txt
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/all/bench.json 2> gpurun_out/all/bench.err || { echo "bench failed"; tail gpurun_out/all/bench.err; exit 1; }
cat gpurun_out/all/bench.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/all/prof_hevc -o run -- python3 tools/hevc_quick.py 3840 2160 20 25000 > gpurun_out/all/prof_hevc.log 2>&1 || echo "rocprof rc=$?"
echo done
