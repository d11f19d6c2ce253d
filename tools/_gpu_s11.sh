set -o pipefail
mkdir -p gpurun_out/s11
B="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0"
for aq in 4 5 6; do timeout -k 10 200 $B --aq $aq > gpurun_out/s11/aq$aq.json 2>/dev/null || exit 1; done
for aq in 4 5; do timeout -k 10 200 python bench.py --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0 --aq $aq > gpurun_out/s11/h264_aq$aq.json 2>/dev/null || exit 1; done
timeout -k 10 200 python bench.py --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0 > gpurun_out/s11/h264_aq3.json 2>/dev/null
