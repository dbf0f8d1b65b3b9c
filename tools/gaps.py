"""GPU idle-gap analysis of a rocprofv3 kernel trace (host-side stalls between kernels).

    python tools/gaps.py <kernel_trace.csv> [--top 30]

Reports busy/idle totals over the trace window and the largest idle gaps with the kernels on
either side (the gap's cause is usually a host sync or Python work before the next launch)."""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--min-us", type=float, default=50.0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]) for r in rows)
    busy, idle, gaps = 0, 0, []
    end = ev[0][1]
    prev = ev[0][2]
    busy += ev[0][1] - ev[0][0]
    for s, e, n in ev[1:]:
        if s > end:
            idle += s - end
            gaps.append((s - end, prev, n))
        busy += e - max(s, end) if e > end else 0
        if e > end:
            end, prev = e, n
    span = end - ev[0][0]
    print(f"span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  idle {idle / 1e6:.1f} ms  kernels {len(ev)}")
    agg = defaultdict(lambda: [0, 0])
    for g, p, n in gaps:
        if g >= a.min_us * 1e3:
            agg[(p, n)][0] += g
            agg[(p, n)][1] += 1
    print(f"idle in gaps >= {a.min_us} us, grouped by (before -> after):")
    for (p, n), (g, c) in sorted(agg.items(), key=lambda x: -x[1][0])[: a.top]:
        print(f"  {g / 1e6:8.2f} ms  x{c:<5d} {p}  ->  {n}")


if __name__ == "__main__":
    main()
