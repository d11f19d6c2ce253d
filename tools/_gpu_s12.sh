set -o pipefail
mkdir -p gpurun_out/s12
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0"
for aq in 3 5; do timeout -k 10 200 $H --aq $aq --content motion > gpurun_out/s12/hevc_motion_aq$aq.json 2>/dev/null || exit 1; done
for aq in 3 4 5; do timeout -k 10 200 python bench.py --steps 300 --warmup 10 --density-probe 0 --aq $aq > gpurun_out/s12/h264_1080_aq$aq.json 2>/dev/null || exit 1; done
for aq in 3 5; do timeout -k 10 200 python bench.py --steps 300 --warmup 10 --density-probe 0 --aq $aq --content motion > gpurun_out/s12/h264_1080_motion_aq$aq.json 2>/dev/null || exit 1; done
