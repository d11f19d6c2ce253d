set -o pipefail
mkdir -p gpurun_out/s15
for r in 1 2 3; do for d in 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 --depth $d --density-probe 0 --quality-probe 0 > gpurun_out/s15/d${d}_r$r.json 2>/dev/null || exit 1; done; done
timeout -k 10 200 python bench.py --codec vp8 --steps 100 --warmup 10 --density-probe 0 > gpurun_out/s15/vp8.json 2>/dev/null
