#!/usr/bin/env bash
# Rate-distortion spot check: H.264 vs HEVC at equal bitrate on the clean synthetic desktop.
set -o pipefail
mkdir -p gpurun_out/rd
for kbps in 2000 4000; do
  for codec in h264 hevc; do
    timeout -k 10 120 python bench.py --codec $codec --noise 0 --bitrate-kbps $kbps --steps 300 --warmup 60 --depth 1 \
      > gpurun_out/rd/${codec}_${kbps}.json 2>/dev/null || { echo "$codec $kbps failed"; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/rd/${codec}_${kbps}.json').read().strip().splitlines()[-1]);print('$codec',$kbps,d['mean_psnr_y_db'],d['mean_qp'],d['mean_bitrate_kbps_at_60fps'],d['value'])"
  done
done
