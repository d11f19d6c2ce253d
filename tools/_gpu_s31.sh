set -o pipefail
o=gpurun_out/s31; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_vp8.py -x -q --timeout 120 --timeout-method thread > $o/vp8tests.log 2>&1 || exit 1
for d in 3 4; do
  for c in desktop motion; do
    MXDESK_HOST_TIMING=1 timeout -k 10 200 python bench.py --codec vp8 --steps 300 --warmup 10 --density-probe 0 --quality-probe 0 --content $c --depth $d > $o/vp8_d${d}_$c.json 2> $o/vp8_d${d}_$c.err || exit 1
  done
done
