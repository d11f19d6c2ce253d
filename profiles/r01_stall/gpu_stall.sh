#!/usr/bin/env bash
# Where the serial tail (k_cavlc -> k_scan -> k_pack) spends its cycles: per-kernel wave
# cycles vs cycles waiting (memory / dependency) vs issued instructions, one --pmc pass.
set -o pipefail
mkdir -p gpurun_out/stall
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM \
    --kernel-trace --output-format csv -d gpurun_out/stall/sq -o run -- \
    python3 bench.py --steps 20 --warmup 3 > gpurun_out/stall/sq.log 2>&1 || { echo "pmc sq rc=$?"; exit 1; }
echo done
