"""Summarise a rocprofv3 kernel_stats.csv: one line per kernel (short name, calls, avg / min us, %).

    python tools/kstats.py gpurun_out/X/prof_Y/run_kernel_stats.csv [N] > profiles/.../kernels.txt
"""
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"\b(k_\w+|__amd_\w+|\w+_kernel\w*)\s*\(", name)
    return m.group(1) if m else name.split("(")[0][-40:]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    for r in rows[:n]:
        print(f"{short(r['Name']):32s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs']) / 1000:9.1f} "
              f"min_us={float(r['MinNs']) / 1000:9.1f} pct={float(r['Percentage']):6.2f}")


if __name__ == "__main__":
    main()
