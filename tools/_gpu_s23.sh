set -o pipefail
o=gpurun_out/s23; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_vp8.py -x -q --timeout 120 --timeout-method thread > $o/vp8tests.log 2>&1 || exit 1
for c in desktop motion; do
  MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --content $c > $o/vp8_$c.json 2> $o/vp8_$c.err || exit 1
done
MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 --quality-probe 0 --depth 2 > $o/vp8_d2.json 2> $o/vp8_d2.err || exit 1
MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --codec vp8 --steps 20 --warmup 5 --quality-probe 0 --density-probe 0 > $o/vp8_20.json 2> $o/vp8_20.err || exit 1
