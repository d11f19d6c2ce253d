set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_hevc.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s5_tests.log 2>&1 && \
timeout -k 10 300 python tools/hevc_cabac_timing.py --wpp 0 --frames 16 --report 3 > gpurun_out/s5_timing.log 2>&1 && \
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0 > gpurun_out/s5_hevc4k.json 2>/dev/null && \
tools/prof_kernels.sh p5_hevc4k --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 40 --warmup 5 --quality-probe 0 --density-probe 0
