set -o pipefail
o=gpurun_out/s25; mkdir -p $o
for c in desktop motion; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --density-probe 0 --deblock 1 --content $c > $o/h264_db1_$c.json 2>/dev/null || exit 1
done
tools/prof_kernels.sh p25_db1 --steps 60 --warmup 5 --quality-probe 0 --density-probe 0 --deblock 1 || exit 1
