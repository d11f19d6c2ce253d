set -o pipefail
mkdir -p gpurun_out/s19
timeout -k 10 300 python -u -m pytest tests/test_gpu_vp8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s19/vp8tests.log 2>&1 || exit 1
tools/prof_kernels.sh p19_vp8 --codec vp8 --steps 40 --warmup 5 --quality-probe 0 --density-probe 0 || exit 1
for c in desktop motion; do timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --content $c > gpurun_out/s19/vp8_$c.json 2>/dev/null || exit 1; done
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM" tools/prof_pmc.sh pmc_h264 --steps 60 --warmup 5 --quality-probe 0 --density-probe 0
tools/prof_timeline.sh tl_h264_d3 k_synth --steps 60 --warmup 5 --quality-probe 0 --density-probe 0
