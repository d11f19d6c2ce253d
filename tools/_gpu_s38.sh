set -o pipefail
o=gpurun_out/s38; mkdir -p $o
H="python bench.py --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 300 --warmup 10 --density-probe 0"
for c in desktop motion; do
  for q in 0 -2 -4; do
    timeout -k 10 200 $H --content $c --chroma-qp-offset=$q > $o/hevc_${c}_cq$q.json 2>/dev/null || exit 1
  done
done
