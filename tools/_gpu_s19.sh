set -o pipefail
mkdir -p gpurun_out/s19
timeout -k 10 300 python -u -m pytest tests/test_gpu_vp8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s19/vp8tests.log 2>&1 || exit 1
tools/prof_kernels.sh p19_vp8 --codec vp8 --steps 40 --warmup 5 --quality-probe 0 --density-probe 0 || exit 1
for c in desktop motion; do timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --content $c > gpurun_out/s19/vp8_$c.json 2>/dev/null || exit 1; done
