#!/usr/bin/env bash
# HEVC GPU check: bit-exact tests vs the CPU encoder, timings, kernel profile.
set -o pipefail
mkdir -p gpurun_out/hevc
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hevc.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/hevc/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/hevc/pytest.log
[ $rc -eq 0 ] || { echo "hevc pytest failed rc=$rc"; tail -30 gpurun_out/hevc/pytest.log; exit 1; }
timeout -k 10 120 python tools/hevc_quick.py 1920 1080 60 8000 > gpurun_out/hevc/t1080.txt 2>&1 || { echo "1080 timing failed"; cat gpurun_out/hevc/t1080.txt; exit 1; }
timeout -k 10 120 python tools/hevc_quick.py 3840 2160 40 25000 > gpurun_out/hevc/t2160.txt 2>&1 || { echo "4k timing failed"; cat gpurun_out/hevc/t2160.txt; exit 1; }
cat gpurun_out/hevc/t1080.txt gpurun_out/hevc/t2160.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hevc/prof -o run -- python3 tools/hevc_quick.py 3840 2160 20 25000 > gpurun_out/hevc/prof.log 2>&1 || echo "rocprof rc=$?"
echo done
