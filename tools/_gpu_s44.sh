set -o pipefail
o=gpurun_out/s44; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --codec vp8 --steps 300 --warmup 10 --density-probe 0 > $o/vp8_300.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --density-probe 0 > $o/hevc4k_300.json 2>/dev/null || exit 1
