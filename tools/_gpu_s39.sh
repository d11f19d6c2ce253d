set -o pipefail
o=gpurun_out/s39; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_hevc.py tests/test_gpu_pipeline.py tests/test_gpu_production_sizes.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || exit 1
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --density-probe 0"
for c in desktop motion; do
  timeout -k 10 200 $H --content $c > $o/hevc_$c.json 2>/dev/null || exit 1
done
