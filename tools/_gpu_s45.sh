set -o pipefail
tools/prof_kernels.sh p45_h264 --steps 100 --warmup 5 --quality-probe 0 --density-probe 0 || exit 1
tools/prof_kernels.sh p45_vp8 --codec vp8 --steps 100 --warmup 5 --quality-probe 0 --density-probe 0 || exit 1
tools/prof_kernels.sh p45_hevc --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 60 --warmup 5 --quality-probe 0 --density-probe 0 || exit 1
tools/prof_timeline.sh tl_h264_final k_synth --steps 60 --warmup 5 --quality-probe 0 --density-probe 0
