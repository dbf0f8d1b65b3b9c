"""GPU idle gaps of the timed forward in a rocprofv3 --kernel-trace CSV of one bench run (warm-up + one
step): union of kernel intervals, the gaps between them grouped by (previous kernel, next kernel), and the
largest single gaps with their position in the step.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python3 bench.py --steps 1 \\
        --warmup 1 --no-cpu-baseline --no-validate
    python tools/trace_gaps.py gpurun_out/trace/run_kernel_trace.csv"""
import collections
import csv
import re
import sys


def short(n: str) -> str:
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    n = re.sub(r"[<(].*", "", n)
    return n.split("::")[-1][:36]


def main(path: str) -> None:
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    t1 = max(e[1] for e in ev)
    # the timed forward starts after the last idle gap > 20 ms that lies more than 3 s before the end
    gaps, cur = [], ev[0][1]
    for i, e in enumerate(ev[1:], 1):
        if e[0] - cur > 20e6:
            gaps.append((i, e[0]))
        cur = max(cur, e[1])
    cand = [g for g in gaps if g[1] < t1 - 3.0e9]
    # no such gap (nothing left idle between the warm-up and the timed step): the whole trace, both forwards
    fw = ev[cand[-1][0]:] if cand else ev
    if not cand:
        print("no idle gap > 20 ms separates the forwards: whole trace (warm-up + timed step)")
    t0 = fw[0][0]
    agg, cnt, idle, tl = collections.Counter(), collections.Counter(), 0, []
    cur, prev = fw[0][1], fw[0]
    for e in fw[1:]:
        if e[0] > cur:
            g = e[0] - cur
            idle += g
            k = (short(prev[2]), short(e[2]))
            agg[k] += g
            cnt[k] += 1
            tl.append(((cur - t0) / 1e6, g / 1e6, k))
        if e[1] > cur:
            cur, prev = e[1], e
    print(f"span: {(t1 - t0) / 1e6:.1f} ms, {len(fw)} kernels, GPU idle {idle / 1e6:.1f} ms")
    for k, v in agg.most_common(12):
        print(f"{v / 1e6:8.2f} ms n={cnt[k]:5d} {k[0]:36s} -> {k[1]}")
    print("largest single gaps:")
    for t, g, k in sorted(tl, key=lambda x: -x[1])[:8]:
        print(f"  at {t:8.1f} ms: {g:7.2f} ms {k[0]} -> {k[1]}")


if __name__ == "__main__":
    main(sys.argv[1])
