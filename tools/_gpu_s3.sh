set -o pipefail
timeout -k 10 300 python tools/hevc_cabac_timing.py --wpp 0 --frames 16 --report 3 > gpurun_out/s3_timing_3072.log 2>&1 && \
timeout -k 10 300 python tools/hevc_cabac_timing.py --wpp 0 --frames 16 --report 3 --slice-cost 1024 > gpurun_out/s3_timing_1024.log 2>&1 && \
timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 100 --warmup 10 --density-probe 0 --hevc-slice-cost 1024 > gpurun_out/s3_hevc4k_c1024.json 2>/dev/null
