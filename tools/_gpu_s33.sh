set -o pipefail
o=gpurun_out/s33; mkdir -p $o
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --quality-probe 0 --density-probe 0"
timeout -k 10 200 $H --capture-stream 0 > $o/hevc_cs0_es3.json 2>/dev/null || exit 1
MXDESK_HEVC_ESTREAMS=2 timeout -k 10 200 $H --capture-stream 0 > $o/hevc_cs0_es2.json 2>/dev/null || exit 1
MXDESK_HEVC_ESTREAMS=2 timeout -k 10 200 $H --capture-stream 1 > $o/hevc_cs1_es2.json 2>/dev/null || exit 1
timeout -k 10 200 $H --capture-stream 1 > $o/hevc_cs1_es3.json 2>/dev/null || exit 1
MXDESK_HEVC_ESTREAMS=2 timeout -k 10 200 $H --capture-stream 1 --depth 2 > $o/hevc_cs1_d2.json 2>/dev/null || exit 1
timeout -k 10 200 $H --capture-stream 0 --depth 2 > $o/hevc_cs0_d2.json 2>/dev/null || exit 1
