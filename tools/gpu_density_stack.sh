#!/usr/bin/env bash
# Concurrent 1080p60 sessions per GPU through the whole serving stack (tools/bench_density.py).
set -o pipefail
mkdir -p gpurun_out/density_stack
export TMPDIR=/tmp
for k in 1 4 8 12; do
  timeout -k 10 150 python tools/bench_density.py --sessions $k --frames 600 --transport webrtc \
      > gpurun_out/density_stack/webrtc_k$k.json 2> gpurun_out/density_stack/webrtc_k$k.err \
      || { echo "k=$k failed"; tail -5 gpurun_out/density_stack/webrtc_k$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/density_stack/webrtc_k$k.json'));print($k,d['min_session_fps'],d['p50_e2e_latency_ms'],d['p95_e2e_latency_ms_worst'])"
done
echo done
