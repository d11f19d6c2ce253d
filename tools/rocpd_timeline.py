"""Timeline view of a rocprofv3 kernel trace (rocpd SQLite): per-stream busy time, the union of
all kernels (GPU busy), idle gaps, and per-frame periods cut at a marker kernel (default the
synthetic render, one per frame).  Tells a latency-bound chain (long idle gaps between
dependent kernels, host turnaround) from a throughput-bound one.

    python tools/rocpd_timeline.py gpurun_out/.../run_results.db [--marker k_synth] [--skip 10]
"""
import argparse
import re
import sqlite3
import statistics


def short(name: str) -> str:
    s = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    return re.sub(r"^.*::", "", s).replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="k_synth")
    ap.add_argument("--skip", type=int, default=10, help="frames skipped at the start (warm-up, IDR)")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    ks = [(short(n), sid, s, e) for n, sid, s, e in rows]
    marks = [s for n, _, s, _ in ks if n == a.marker]
    if len(marks) <= a.skip + 2:
        raise SystemExit("not enough frames")
    t0, t1 = marks[a.skip], marks[-1]
    win = [k for k in ks if k[2] >= t0 and k[3] <= t1]
    span = (t1 - t0) / 1000.0
    nfr = len(marks) - 1 - a.skip
    # union of busy intervals
    busy, cur_s, cur_e = 0.0, None, None
    gaps = []
    for _, _, s, e in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1000.0
                gaps.append((s - cur_e) / 1000.0)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += (cur_e - cur_s) / 1000.0
    per_stream = {}
    for n, sid, s, e in win:
        per_stream.setdefault(sid, [0.0, set()])
        per_stream[sid][0] += (e - s) / 1000.0
        per_stream[sid][1].add(n)
    print(f"frames {nfr}, span {span:.1f} us, {span / nfr:.2f} us/frame ({1e6 * nfr / span:.0f} fps)")
    print(f"GPU busy (union) {busy / nfr:.2f} us/frame = {100 * busy / span:.1f} %; idle gaps {len(gaps) / nfr:.1f}/frame, "
          f"mean {statistics.mean(gaps) if gaps else 0:.2f} us, total {sum(gaps) / nfr:.2f} us/frame")
    for sid, (t, names) in sorted(per_stream.items()):
        print(f"stream {sid}: kernel time {t / nfr:.2f} us/frame; {', '.join(sorted(names))}")
    # per kernel: mean start offset from the frame marker
    offs = {}
    for i in range(a.skip, len(marks) - 1):
        m0, m1 = marks[i], marks[i + 1]
        for n, sid, s, e in ks:
            if m0 <= s < m1:
                offs.setdefault(n, []).append(((s - m0) / 1000.0, (e - m0) / 1000.0))
    print("kernel: mean start / end offset from the marker (us)")
    for n, v in sorted(offs.items(), key=lambda kv: statistics.mean(x[0] for x in kv[1])):
        print(f"  {n:24s} {statistics.mean(x[0] for x in v):8.2f} {statistics.mean(x[1] for x in v):8.2f}  (n={len(v)})")


if __name__ == "__main__":
    main()
