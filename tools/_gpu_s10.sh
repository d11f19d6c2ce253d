set -o pipefail
mkdir -p gpurun_out/s10
timeout -k 10 300 python -u -m pytest tests/test_hevc.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s10/tests.log 2>&1 && \
timeout -k 10 200 python tools/hevc_session_timing.py > gpurun_out/s10/timing.log 2>&1 && \
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0 > gpurun_out/s10/d3.json 2>/dev/null && \
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0 --depth 2 > gpurun_out/s10/d2.json 2>/dev/null && \
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0 --depth 1 > gpurun_out/s10/d1.json 2>/dev/null
