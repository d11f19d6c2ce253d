set -o pipefail
mkdir -p gpurun_out/s18
timeout -k 10 300 python -u -m pytest tests/test_gpu_vp8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s18/vp8tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_hevc.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s18/tests.log 2>&1 || exit 1
tools/prof_kernels.sh p18_vp8 --codec vp8 --steps 40 --warmup 5 --quality-probe 0 --density-probe 0 || exit 1
tools/prof_kernels.sh p18_hevc --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 40 --warmup 5 --quality-probe 0 --density-probe 0 || exit 1
bash tools/_gpu_s17.sh
