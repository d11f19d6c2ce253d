#!/usr/bin/env bash
# HEVC split transform trees on the GPU: bit-exactness vs the CPU oracle, speed and quality at 4K/1080p.
set -o pipefail
mkdir -p gpurun_out/tusplit
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hevc.py -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/tusplit/pytest_hevc_gpu.log 2>&1 || { echo "hevc gpu tests failed"; tail -30 gpurun_out/tusplit/pytest_hevc_gpu.log; exit 1; }
for ts in 0 1; do
  timeout -k 10 200 python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 200 --warmup 20 --tu-split $ts \
    > gpurun_out/tusplit/hevc4k_ts$ts.json 2>/dev/null || { echo "bench 4k ts=$ts failed"; exit 1; }
  for kbps in 2000 4000; do
    timeout -k 10 120 python bench.py --codec hevc --noise 0 --bitrate-kbps $kbps --steps 300 --warmup 60 --depth 1 --tu-split $ts \
      > gpurun_out/tusplit/rd_${kbps}_ts$ts.json 2>/dev/null || { echo "rd $kbps ts=$ts failed"; exit 1; }
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tusplit/prof -o hevc4k_ts1 -- python3 bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 60 --warmup 10 --tu-split 1 > gpurun_out/tusplit/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
for f in gpurun_out/tusplit/*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['p50_e2e_latency_ms'],d['mean_psnr_y_db'],d['mean_qp'],d['mean_bitrate_kbps_at_60fps'])"; done
echo done
