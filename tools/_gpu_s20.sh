set -o pipefail
o=gpurun_out/s20; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $o/pipeline.log 2>&1 || exit 1
for cs in 1 0; do
  for st in 20 300; do
    MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --steps $st --warmup 5 --quality-probe 0 --density-probe 0 --capture-stream $cs > $o/h264_cs${cs}_$st.json 2> $o/h264_cs${cs}_$st.err || exit 1
  done
done
timeout -k 10 200 python bench.py --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 --depth 2 > $o/h264_d2_300.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 > $o/hevc4k_300.json 2>/dev/null || exit 1
tools/prof_timeline.sh tl_h264_cs k_synth --steps 60 --warmup 5 --quality-probe 0 --density-probe 0
timeout -k 10 300 python -u -m pytest tests/test_gpu_vp8.py -x -q --timeout 120 --timeout-method thread > $o/vp8tests.log 2>&1 || exit 1
MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 > $o/vp8_desktop.json 2> $o/vp8_desktop.err || exit 1
mkdir -p profiles/r04_wall_timing 2>/dev/null; timeout -k 10 240 python tools/wall_timing.py --layout 2x2 --tile 1920x1080 --frames 60 --json-out $o/wall_2x2.json > $o/wall.log 2>&1 || exit 1
