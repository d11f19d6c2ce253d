set -o pipefail
o=gpurun_out/s34; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
for st in 20 300; do
  MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --steps $st --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264_$st.json 2> $o/h264_$st.err || exit 1
done
timeout -k 10 200 python bench.py --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264_4k.json 2>/dev/null || exit 1
