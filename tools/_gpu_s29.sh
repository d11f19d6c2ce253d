set -o pipefail
o=gpurun_out/s29; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_production_sizes.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || exit 1
for st in 20 300; do
  MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --steps $st --warmup 5 --quality-probe 0 --density-probe 0 > $o/h264_$st.json 2> $o/h264_$st.err || exit 1
done
MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --quality-probe 0 --density-probe 0 --depth 4 > $o/h264_d4_300.json 2> $o/h264_d4_300.err || exit 1
tools/prof_timeline.sh tl_h264_inev k_synth --steps 60 --warmup 5 --quality-probe 0 --density-probe 0
