set -o pipefail
B="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0"
mkdir -p gpurun_out/s6
for c in 3072 4096 6144; do timeout -k 10 200 $B --hevc-slice-cost $c > gpurun_out/s6/c$c.json 2>/dev/null || exit 1; done
timeout -k 10 200 $B --depth 2 > gpurun_out/s6/d2.json 2>/dev/null || exit 1
timeout -k 10 200 $B --depth 1 > gpurun_out/s6/d1.json 2>/dev/null || exit 1
timeout -k 10 200 $B --hevc-wpp 1 > gpurun_out/s6/wpp.json 2>/dev/null || exit 1
