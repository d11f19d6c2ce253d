set -o pipefail
mkdir -p gpurun_out/s14
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s14/gputests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/s14/h264_20.json 2>/dev/null && \
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --density-probe 0 > gpurun_out/s14/h264_300.json 2>/dev/null && \
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --density-probe 0 > gpurun_out/s14/hevc4k_300.json 2>/dev/null && \
timeout -k 10 200 python bench.py --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --density-probe 0 > gpurun_out/s14/h264_4k_300.json 2>/dev/null
