set -o pipefail
o=gpurun_out/s24; mkdir -p $o
for ip in 0 1; do
  for c in desktop motion; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 5 --density-probe 0 --intra-in-p $ip --content $c > $o/h264_ip${ip}_$c.json 2>/dev/null || exit 1
  done
done
tools/prof_kernels.sh p24_ip1 --steps 60 --warmup 5 --quality-probe 0 --density-probe 0 --intra-in-p 1 || exit 1
tools/prof_kernels.sh p24_ip1_motion --steps 60 --warmup 5 --quality-probe 0 --density-probe 0 --intra-in-p 1 --content motion || exit 1
