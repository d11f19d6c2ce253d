set -o pipefail
o=gpurun_out/s35; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_hevc.py tests/test_gpu_pipeline.py tests/test_gpu_production_sizes.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || exit 1
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --density-probe 0"
MXDESK_HOST_TIMING=1 timeout -k 10 200 $H > $o/hevc_d3.json 2> $o/hevc_d3.err || exit 1
timeout -k 10 200 $H --depth 2 --quality-probe 0 > $o/hevc_d2.json 2>/dev/null || exit 1
tools/prof_timeline.sh tl_hevc_pub k_hpel --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 40 --warmup 5 --quality-probe 0 --density-probe 0
