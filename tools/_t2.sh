set -o pipefail
O=gpurun_out/r02_r; mkdir -p $O
for ip in 0 1; do
timeout -k 10 300 python bench.py --steps 300 --warmup 5 --intra-in-p $ip --json-out $O/ip$ip.json > $O/ip$ip.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --intra-in-p $ip --json-out $O/ip${ip}_20.json > $O/ip${ip}_20.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/rc_trace.py --frames 40 --qps 28,32,36,40 > $O/rctrace.log 2>&1
