set -o pipefail
# Scaler / clean-profile pass: GPU scaler tests, 1080p + 4K->1080p kernel stats, scaler PMC
# (compute counters, then FETCH_SIZE and WRITE_SIZE each in a run of its own).
O=gpurun_out/${1:-r02_prof}; mkdir -p $O
B4K="bench.py --width 3840 --height 2160 --out-width 1920 --out-height 1080 --density-probe 0"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py -k "lanczos or csc or scaled" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 60 --warmup 5 --density-probe 0 > $O/prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4k -o run -- python3 $B4K --steps 60 --warmup 5 > $O/prof4k.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex "scale" --output-format csv -d $O/pmc_scale -o run -- python3 $B4K --steps 10 --warmup 2 > $O/pmc_scale.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scale" --output-format csv -d $O/pmc_scale_fetch -o run -- python3 $B4K --steps 10 --warmup 2 > $O/pmc_scale_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "scale" --output-format csv -d $O/pmc_scale_write -o run -- python3 $B4K --steps 10 --warmup 2 > $O/pmc_scale_write.log 2>&1
