set -o pipefail
o=gpurun_out/s46; mkdir -p $o
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --quality-probe 0 --density-probe 0"
timeout -k 10 200 $H > $o/hevc_q4_cs0.json 2>/dev/null || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $H > $o/hevc_q8_cs0.json 2>/dev/null || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $H --capture-stream 1 > $o/hevc_q8_cs1.json 2>/dev/null || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264_q8.json 2>/dev/null || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264_4k_q8.json 2>/dev/null || exit 1
