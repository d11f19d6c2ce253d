set -o pipefail
o=gpurun_out/s21; mkdir -p $o
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --quality-probe 0 --density-probe 0"
for cs in 0 1; do
  MXDESK_HOST_TIMING=1 timeout -k 10 200 $H --capture-stream $cs > $o/hevc_cs$cs.json 2> $o/hevc_cs$cs.err || exit 1
done
tools/prof_timeline.sh tl_hevc_cs k_synth --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 40 --warmup 5 --quality-probe 0 --density-probe 0
