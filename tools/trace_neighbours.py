"""Which kernels surround a given kernel in a rocprofv3 kernel trace (finds the source of e.g.
__amd_rocclr_copyBuffer launches inside a forward).

    python tools/trace_neighbours.py <kernel_trace.csv> [--name copyBuffer] [--ctx 2] [--top 15]"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--name", default="copyBuffer")
ap.add_argument("--ctx", type=int, default=2)
ap.add_argument("--top", type=int, default=15)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[:70]  # noqa: E731
seq = collections.Counter()
dur = 0
n = 0
for i, r in enumerate(rows):
    if a.name in r["Kernel_Name"]:
        n += 1
        dur += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        before = tuple(short(rows[j]["Kernel_Name"]) for j in range(max(0, i - a.ctx), i))
        after = tuple(short(rows[j]["Kernel_Name"]) for j in range(i + 1, min(len(rows), i + 1 + a.ctx)))
        seq[(before, after)] += 1
print(f"{n} launches of *{a.name}*, {dur / 1e6:.2f} ms")
for (b, f), c in seq.most_common(a.top):
    print(f"{c:5d}  {' > '.join(b)}  [*]  {' > '.join(f)}")
