"""Fabric traffic per kernel and launch shape: the rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes of one bench step (tools/pmc_bench.sh with RDMI_PROF_SEQ set, so each pass also writes
the launch sequence of kernels._Timed), the family's dispatches matched 1:1 in launch order against that
sequence, then per (kernel, shape): fetched + written bytes against the algorithmic bytes (every operand
read once, the output written once) — the ratio says where operands are re-read from beyond the L2.

    python tools/traffic_split.py --fetch DIR --write DIR [--family implicit_gemm|attention_fwd|...] [--top 40]

FETCH_SIZE ×2 (gfx950 16-B streaming rule, MI355X_MICROARCH.md), WRITE_SIZE ×1; L2 → fabric bytes, so
Infinity-Cache hits count as traffic (an upper bound on HBM bytes)."""
import argparse
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_traffic import FAMILIES, family  # noqa: E402


def dispatches(d, counter):
    rows = []
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    rows.sort()
    return rows


def short(name):
    n = name.replace("(anonymous namespace)::", "").removeprefix("void ")
    n = re.sub(r"\(.*", "", n)
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--family", default="implicit_gemm")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--counters", default="FETCH_SIZE,WRITE_SIZE", help="passes to read (a FETCH-only run: FETCH_SIZE)")
    a = ap.parse_args()
    fams = [f for f, _ in FAMILIES]
    res = {}
    want = a.counters.split(",")
    for d, cn, mul in ((a.fetch, "FETCH_SIZE", 2.0), (a.write, "WRITE_SIZE", 1.0)):
        if cn not in want:
            continue
        seq = json.load(open(os.path.join(d, "seq.json")))
        seq = [s for s in seq if s[0] == a.family]
        rows = [r for r in dispatches(d, cn) if family(r[1]) == a.family]
        if len(rows) != len(seq):
            sys.exit(f"{cn}: {len(rows)} {a.family} dispatches vs {len(seq)} timed launches — cannot match")
        for (_, kn, v), (_, shape, flop, nb) in zip(rows, seq):
            e = res.setdefault((short(kn), shape), {"n": 0, "alg": 0.0, "flop": 0.0, "FETCH_SIZE": 0.0,
                                                    "WRITE_SIZE": 0.0})
            if cn == want[0]:
                e["n"] += 1
                e["alg"] += nb
                e["flop"] += flop
            e[cn] += v * mul
    assert all(f in fams for f in [a.family])
    rows = sorted(res.items(), key=lambda kv: -(kv[1]["FETCH_SIZE"] + kv[1]["WRITE_SIZE"]))
    tot = {"alg": 0.0, "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0}
    per_kernel = {}
    print(f"# {a.family}: fabric bytes (FETCH x2 + WRITE) vs algorithmic bytes, one bench step")
    print(f"{'kernel':70s} {'shape':44s} {'n':>4s} {'alg GB':>8s} {'fetch GB':>9s} {'write GB':>9s} {'ratio':>6s}")
    for (kn, shape), e in rows[:a.top]:
        t = e["FETCH_SIZE"] + e["WRITE_SIZE"]
        print(f"{kn:70s} {str(shape):44s} {e['n']:4d} {e['alg'] / 1e9:8.2f} {e['FETCH_SIZE'] / 1e9:9.2f} "
              f"{e['WRITE_SIZE'] / 1e9:9.2f} {t / max(e['alg'], 1):6.2f}")
    for (kn, shape), e in rows:
        for k in tot:
            tot[k] += e[k]
        pk = per_kernel.setdefault(kn, {"n": 0, "alg": 0.0, "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0})
        for k in pk:
            pk[k] += e[k]
    print(f"\n# per kernel\n{'kernel':70s} {'n':>5s} {'alg GB':>8s} {'fetch GB':>9s} {'write GB':>9s} {'ratio':>6s}")
    for kn, e in sorted(per_kernel.items(), key=lambda kv: -(kv[1]["FETCH_SIZE"] + kv[1]["WRITE_SIZE"])):
        t = e["FETCH_SIZE"] + e["WRITE_SIZE"]
        print(f"{kn:70s} {e['n']:5d} {e['alg'] / 1e9:8.2f} {e['FETCH_SIZE'] / 1e9:9.2f} {e['WRITE_SIZE'] / 1e9:9.2f} "
              f"{t / max(e['alg'], 1):6.2f}")
    t = tot["FETCH_SIZE"] + tot["WRITE_SIZE"]
    print(f"\n# total: alg {tot['alg'] / 1e9:.2f} GB, fetch {tot['FETCH_SIZE'] / 1e9:.2f} GB, write "
          f"{tot['WRITE_SIZE'] / 1e9:.2f} GB, ratio {t / max(tot['alg'], 1):.3f}")


if __name__ == "__main__":
    main()
