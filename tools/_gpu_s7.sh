set -o pipefail
tools/prof_timeline.sh tl_hevc4k_d1 k_synth --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 30 --warmup 5 --quality-probe 0 --density-probe 0 --depth 1 && \
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0 --graph 1 > gpurun_out/s7_graph.json 2>/dev/null
