#!/usr/bin/env bash
# Hardware-counter evidence: LDS traffic / bank conflicts of the LDS-tiled
# kernels and HBM bytes, each counter set in its own rocprofv3 run (--pmc with kernel trace only).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc/avail.txt 2>&1 || echo "list-avail rc=$?"
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc/$name -o run -- \
      python3 bench.py --steps 20 --warmup 3 > gpurun_out/pmc/$name.log 2>&1 || echo "pmc $name rc=$?"
}
run lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES
run valu SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES
run mem FETCH_SIZE WRITE_SIZE
echo done
