"""Per-kernel statistics (calls, total / mean / min / max microseconds, share) from a rocprofv3
rocpd SQLite database (the default output of this ROCm's rocprofv3), as a markdown table.

    python tools/rocpd_stats.py gpurun_out/.../run_results.db [--per-frame N] > profiles/.../kernels.md
"""
import argparse
import re
import sqlite3


def stats(path: str):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
    rows = db.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for name, s, e in rows:
        short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
        short = re.sub(r"^.*::", "", short).replace("void ", "")
        d = (e - s) / 1000.0
        a = agg.setdefault(short, [0, 0.0, 1e18, 0.0])
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per-frame", type=int, default=0, help="frames in the run: adds a us/frame column")
    a = ap.parse_args()
    agg = stats(a.db)
    total = sum(v[1] for v in agg.values())
    hdr = "| kernel | calls | total us | mean us | min us | max us | share |" + (" us/frame |" if a.per_frame else "")
    print(hdr)
    print("|" + "---|" * (hdr.count("|") - 1))
    for k, (n, t, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        row = f"| {k} | {n} | {t:.1f} | {t / n:.2f} | {mn:.2f} | {mx:.2f} | {100 * t / total:.1f} % |"
        if a.per_frame:
            row += f" {t / a.per_frame:.2f} |"
        print(row)
    print(f"\ntotal kernel time {total:.1f} us" + (f", {total / a.per_frame:.1f} us/frame" if a.per_frame else ""))


if __name__ == "__main__":
    main()
