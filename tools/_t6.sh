set -o pipefail
# Scaler timing counters: busy cycles vs wall time (effective clock), wait breakdown.
O=gpurun_out/${1:-r02_mf}; mkdir -p $O
B4K="bench.py --width 3840 --height 2160 --out-width 1920 --out-height 1080 --density-probe 0"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM --kernel-include-regex "scale|synth" --output-format csv -d $O/pmc_t1 -o run -- python3 $B4K --steps 10 --warmup 2 > $O/pmc_t1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_VMEM --kernel-include-regex "scale" --output-format csv -d $O/pmc_t2 -o run -- python3 $B4K --steps 10 --warmup 2 > $O/pmc_t2.log 2>&1
