#!/bin/bash
# Kernel timeline of one bench configuration: rocprofv3 kernel trace (CSV), then the kernels of a
# few consecutive frames with start offsets / durations / gaps in gpurun_out/<tag>/timeline.txt.
# usage: tools/prof_timeline.sh <tag> <first-kernel-of-frame> <bench args...>
set -eo pipefail
tag=$1; first=$2; shift 2
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/prof -o run -- python3 bench.py "$@" > $out/bench.json 2> $out/bench.err
f=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 - "$f" "$first" > $out/timeline.txt <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2]
def short(n):
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))
    return re.sub(r"^.*::", "", n).replace("void ", "")
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows))
starts = [i for i, e in enumerate(ev) if e[2] == first]
for k in starts[-8:-4]:
    t0 = ev[k][0]
    print(f"--- frame at {t0}")
    for s, e, n, q in ev[k:k + 40]:
        if s - t0 > 3_000_000: break
        print(f"{(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  q{q:>3s} {n}")
PY
rm -rf $out/prof
