set -o pipefail
# scaler experiment: kernel stats with MXDESK_SCALE_DBG variants (0 = normal)
O=gpurun_out/${1:-r02_mf}; mkdir -p $O
B4K="bench.py --width 3840 --height 2160 --out-width 1920 --out-height 1080 --density-probe 0"
for d in ${2:-0}; do
MXDESK_SCALE_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dbg$d -o run -- python3 $B4K --steps 30 --warmup 5 > $O/prof_dbg$d.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "scale" --output-format csv -d $O/pmc_a -o run -- python3 $B4K --steps 10 --warmup 2 > $O/pmc_a.log 2>&1
