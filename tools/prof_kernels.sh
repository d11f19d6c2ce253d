#!/bin/bash
# Kernel time table of one bench configuration: rocprofv3 kernel trace + stats (CSV), then a short
# per-kernel summary (calls, average us, share) in gpurun_out/<tag>/kernels.txt.
# usage: tools/prof_kernels.sh <tag> <bench args...>
set -eo pipefail
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py "$@" > $out/bench.json 2> $out/bench.err
f=$(find $out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $out/kernel_stats.csv
python3 - "$out/kernel_stats.csv" > $out/kernels.txt <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", ""))
    n = re.sub(r"^.*::", "", n).replace("void ", "")
    print(f"{n:32s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1000:9.1f} pct={float(r['Percentage']):6.2f}")
PY
rm -rf $out/prof
