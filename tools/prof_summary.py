"""Summarise a rocprofv3 output directory tree: kernel stats + PMC counter means."""
import collections
import csv
import os
import sys

root = sys.argv[1]
for d in sorted(os.listdir(root)):
    p = os.path.join(root, d)
    if not os.path.isdir(p):
        continue
    ks = os.path.join(p, "run_kernel_stats.csv")
    cc = os.path.join(p, "run_counter_collection.csv")
    if os.path.exists(ks):
        print(d)
        for r in list(csv.DictReader(open(ks)))[:int(sys.argv[2]) if len(sys.argv) > 2 else 14]:
            print("  %-48s %6s calls avg %8.1f us  min %8.1f" % (r["Name"][:48], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                                float(r["MinNs"]) / 1e3))
    if os.path.exists(cc):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(cc)):
            agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
        print(d)
        for (k, c), v in sorted(agg.items()):
            print("  %-40s %-24s %14.1f (n=%d)" % (k, c, sum(v) / len(v), len(v)))
