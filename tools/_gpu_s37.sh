set -o pipefail
o=gpurun_out/s37; mkdir -p $o
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/h264_20_a.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/h264_20_b.json 2>/dev/null || exit 1
nproc > $o/nproc.txt; uptime >> $o/nproc.txt
