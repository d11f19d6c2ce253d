set -o pipefail
o=gpurun_out/s42; mkdir -p $o
MXDESK_CAPTURE_PRIORITY=normal timeout -k 10 300 python bench.py --steps 20 --warmup 5 --quality-probe 0 > $o/new_normal.json 2>/dev/null || exit 1
(cd old_tree && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --quality-probe 0 > ../$o/old.json 2>/dev/null) || exit 1
