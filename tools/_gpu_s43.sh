set -o pipefail
o=gpurun_out/s43; mkdir -p $o
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/h264_20.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --steps 300 --warmup 5 --density-probe 0 > $o/h264_300.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 5 --density-probe 0 > $o/h264_4k_300.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --content motion --steps 300 --warmup 5 --density-probe 0 > $o/h264_motion_300.json 2>/dev/null || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || exit 1
