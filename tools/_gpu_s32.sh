set -o pipefail
o=gpurun_out/s32; mkdir -p $o
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --quality-probe 0 --density-probe 0"
timeout -k 10 200 $H --capture-stream 0 > $o/hevc_cs0.json 2>/dev/null || exit 1
timeout -k 10 200 $H --capture-stream 1 > $o/hevc_cs1.json 2>/dev/null || exit 1
MXDESK_CAPTURE_PRIORITY=low timeout -k 10 200 $H --capture-stream 1 > $o/hevc_cs1_low.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264.json 2>/dev/null || exit 1
MXDESK_CAPTURE_PRIORITY=low timeout -k 10 200 python bench.py --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264_low.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264_4k.json 2>/dev/null || exit 1
MXDESK_CAPTURE_PRIORITY=low timeout -k 10 200 python bench.py --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264_4k_low.json 2>/dev/null || exit 1
