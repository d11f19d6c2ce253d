#!/usr/bin/env bash
# PMC counters of the HEVC CABAC kernel (one pass; counters chosen within the SQ limit of 8).
set -o pipefail
mkdir -p gpurun_out/hevc_pmc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_hevc_cabac|k_hevc_inter" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d gpurun_out/hevc_pmc -o pmc -- python3 tools/hevc_quick.py 3840 2160 6 25000 > gpurun_out/hevc_pmc/log.txt 2>&1; echo "rc=$?"
