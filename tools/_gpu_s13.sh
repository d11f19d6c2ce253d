set -o pipefail
mkdir -p gpurun_out/s13
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0"
for aq in 4 5 6; do for c in desktop motion; do timeout -k 10 200 $H --aq $aq --content $c > gpurun_out/s13/hevc_${c}_aq$aq.json 2>/dev/null || exit 1; done; done
for aq in 4 5 6; do for c in desktop motion; do timeout -k 10 200 python bench.py --steps 300 --warmup 10 --density-probe 0 --aq $aq --content $c > gpurun_out/s13/h264_${c}_aq$aq.json 2>/dev/null || exit 1; done; done
