set -o pipefail
o=gpurun_out/s41; mkdir -p $o
(cd old_tree && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --quality-probe 0 > ../$o/old.json 2>/dev/null) || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --quality-probe 0 > $o/new.json 2>/dev/null || exit 1
(cd old_tree && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --quality-probe 0 > ../$o/old2.json 2>/dev/null) || exit 1
uptime > $o/load.txt
