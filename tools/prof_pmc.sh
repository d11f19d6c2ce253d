#!/bin/bash
# Per-kernel PMC counters of one bench configuration (one rocprofv3 pass, counters given in $PMC),
# averaged per dispatch into gpurun_out/<tag>/pmc.txt.  usage: PMC="SQ_WAVES ..." tools/prof_pmc.sh <tag> <bench args...>
set -eo pipefail
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $out/prof -o run -- python3 bench.py "$@" > $out/bench.json 2> $out/bench.err
f=$(find $out/prof -name "*counter_collection.csv" | head -1)
python3 - "$f" > $out/pmc.txt <<'PY'
import csv, re, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
    n = re.sub(r"^.*::", "", n).replace("void ", "")
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[n].add(r["Dispatch_Id"])
for n, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    k = len(cnt[n])
    print(f"{n:28s} disp={k:4d} " + " ".join(f"{c}={v / k:.4g}" for c, v in sorted(d.items())))
PY
rm -rf $out/prof
