set -o pipefail
mkdir -p gpurun_out/s17
echo skip > gpurun_out/s17/tests.log
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0"
for c in desktop motion; do timeout -k 10 200 $H --content $c > gpurun_out/s17/hevc_$c.json 2>/dev/null || exit 1; done
for c in desktop motion; do timeout -k 10 200 python bench.py --steps 300 --warmup 10 --density-probe 0 --content $c > gpurun_out/s17/h264_$c.json 2>/dev/null || exit 1; done
for c in desktop motion; do timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --content $c > gpurun_out/s17/vp8_$c.json 2>/dev/null || exit 1; done
timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --aq 2 > gpurun_out/s17/vp8_desktop_aq2.json 2>/dev/null
