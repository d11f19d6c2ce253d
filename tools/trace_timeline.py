"""Per-frame timeline from a rocprofv3 kernel-trace CSV (--kernel-trace --output-format csv):
kernel spans per stream, frame period cut at a marker kernel, GPU-busy union and idle gaps.

    python tools/trace_timeline.py gpurun_out/.../run_kernel_trace.csv [--marker k_synth] [--skip 10] [--frames 4]
"""
import argparse
import csv
import re
import statistics


def short(name: str) -> str:
    s = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    return re.sub(r"^.*::", "", s).replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="k_synth")
    ap.add_argument("--skip", type=int, default=10)
    ap.add_argument("--frames", type=int, default=3, help="frames printed in full")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]))
    rows.sort()
    marks = [r[0] for r in rows if r[2] == a.marker]
    marks = marks[a.skip:]
    periods = [(b - x) / 1e3 for x, b in zip(marks, marks[1:])]
    print(f"frames {len(periods)}: period mean {statistics.mean(periods):.1f} us, median {statistics.median(periods):.1f}")
    t0, t1 = marks[0], marks[-1]
    sel = [r for r in rows if t0 <= r[0] < t1]
    # busy union
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sorted(sel):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"GPU busy {100.0 * busy / (t1 - t0):.1f} % of {(t1 - t0) / 1e3:.0f} us")
    per = {}
    for s, e, n, q in sel:
        per.setdefault((q, n), []).append((e - s) / 1e3)
    for (q, n), v in sorted(per.items()):
        print(f"  q{q} {n:24s} n={len(v):4d} mean {statistics.mean(v):7.1f} us  total/frame {sum(v) / len(periods):7.1f}")
    for f in range(min(a.frames, len(marks) - 1)):
        print(f"--- frame {f} (t=0 at {a.marker})")
        for s, e, n, q in rows:
            if marks[f] - 20000 <= s < marks[f + 1]:
                print(f"  q{q} {n:24s} {(s - marks[f]) / 1e3:8.1f} .. {(e - marks[f]) / 1e3:8.1f}")


if __name__ == "__main__":
    main()
