"""Per-stream occupancy of a rocprofv3 kernel trace: which stream (hardware queue) is the busy one.

    python tools/queue_timeline.py gpurun_out/<run>/prof_<name>/run_kernel_trace.csv [--skip-ms 50]

For every (queue, stream): busy fraction of the traced window (union of its kernels' intervals), the kernels
it runs with their total time, and the mean gap between consecutive kernels (launch / barrier-packet
overhead).  The queue whose busy fraction is near 1 bounds the pipeline's rate.
"""
import argparse
import csv
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-ms", type=float, default=50.0, help="ignore the first milliseconds (warm-up)")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        m = re.search(r"(k_\w+(?:<\d+>)?)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:28]
        rows.append(((int(r["Queue_Id"]), int(r.get("Stream_Id") or 0)), name, int(r["Start_Timestamp"]),
                     int(r["End_Timestamp"])))
    if not rows:
        return
    t0 = min(r[2] for r in rows) + int(a.skip_ms * 1e6)
    rows = [r for r in rows if r[2] >= t0]
    t1 = max(r[3] for r in rows)
    span = t1 - t0
    byq = defaultdict(list)
    for q, n, s, e in rows:
        byq[q].append((s, e, n))
    print(f"window {span / 1e6:.2f} ms")
    allk = sorted((s, e) for _, _, s, e in rows)
    busy_all, cs, ce = 0, None, None
    for s, e in allk:
        if ce is None or s > ce:
            if ce is not None:
                busy_all += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy_all += ce - cs
    print(f"any kernel running: {100.0 * busy_all / span:5.1f} % of the window")
    for q, ks in sorted(byq.items()):
        ks.sort()
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        for s, e, _ in ks:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append(s - cur_e)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        tot = defaultdict(int)
        cnt = defaultdict(int)
        for s, e, n in ks:
            tot[n] += e - s
            cnt[n] += 1
        top = sorted(tot.items(), key=lambda kv: -kv[1])[:8]
        gap = sum(gaps) / len(gaps) / 1e3 if gaps else 0.0
        print(f"queue {q[0]} stream {q[1]}: busy {100.0 * busy / span:5.1f} %  kernels {len(ks)}  mean gap {gap:.1f} us")
        for n, t in top:
            print(f"    {n:<24} {t / 1e3 / cnt[n]:8.1f} us x {cnt[n]:4d}  ({100.0 * t / span:5.1f} % of window)")


if __name__ == "__main__":
    main()
