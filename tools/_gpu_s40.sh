set -o pipefail
o=gpurun_out/s40; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $o/bench_default.json 2> $o/bench_default.err || exit 1
