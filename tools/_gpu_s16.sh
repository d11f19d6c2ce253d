set -o pipefail
mkdir -p gpurun_out/s16
timeout -k 10 300 python -u -m pytest tests/test_gpu_vp8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s16/tests.log 2>&1 && \
timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 > gpurun_out/s16/vp8.json 2>gpurun_out/s16/vp8.err && \
timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --aq 2 > gpurun_out/s16/vp8_aq2.json 2>/dev/null && \
timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --content motion > gpurun_out/s16/vp8_motion.json 2>/dev/null && \
timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --content motion --aq 2 > gpurun_out/s16/vp8_motion_aq2.json 2>/dev/null
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM" tools/prof_pmc.sh pmc_h264 --steps 60 --warmup 5 --quality-probe 0 --density-probe 0
tools/prof_timeline.sh tl_h264_d3 k_synth --steps 60 --warmup 5 --quality-probe 0 --density-probe 0
