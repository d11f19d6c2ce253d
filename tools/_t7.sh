set -o pipefail
O=gpurun_out/${1:-r02_mf}; mkdir -p $O
B4K="bench.py --width 3840 --height 2160 --out-width 1920 --out-height 1080 --density-probe 0"
export MXDESK_SCALE_DBG=${2:-1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dbg$MXDESK_SCALE_DBG -o run -- python3 $B4K --steps 30 --warmup 5 > $O/prof_dbg.log 2>&1
