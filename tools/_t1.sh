set -o pipefail
O=gpurun_out/${1:-r02_x}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_production_sizes.py tests/test_gpu_rate_control.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/pytest.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out $O/n1.json > $O/n1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 5 --density-probe 0 --json-out $O/n1_300.json > $O/n1_300.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 60 --warmup 5 --density-probe 0 > $O/prof.log 2>&1
