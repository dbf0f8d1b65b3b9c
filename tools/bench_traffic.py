"""HBM traffic per launch of bench.py's kernel families, from two rocprofv3 --pmc passes over one
bench step (tools/pmc_bench.sh: FETCH_SIZE and WRITE_SIZE need separate passes).

    python tools/bench_traffic.py --fetch gpurun_out/pmc_bench/fetch --write gpurun_out/pmc_bench/write \
        --preset fast --source profiles/r02_pmc_bench_fast.txt --out bench_traffic.json

Reading rules (MI355X_MICROARCH.md § HBM): FETCH_SIZE (KB) reports ½ of the bytes of 16-B-per-lane
streaming reads, `buffer_load … lds` included — doubled here, checked on a known-bytes copy
(profiles/r02_pmc_summary.txt, pass copy_fetch: 1 GiB copy → 524 300 KB); WRITE_SIZE (KB) is exact
for 16-B streaming stores (copy_write: 1 048 576 KB).  Both count L2 → fabric requests, so Infinity-
Cache (MALL) hits are included: the figure is an upper bound on HBM bytes.

The families are the ones bench.py times (kernels._Timed): implicit_gemm = every f16 GEMM / conv
engine, attention_fwd = the f16 flash kernel, and their _f32 twins."""
import argparse
import csv
import json
import os
import re

FAMILIES = [
    ("implicit_gemm_f32x3", re.compile(r"gemm_f32_kernel<\d+, true>|gemm_f32_kernelILi\dELb1E")),
    ("implicit_gemm_f32", re.compile(r"gemm_f32_kernel")),
    ("attention_fwd_f32x6", re.compile(r"attn_fwd_f32s<3>|attn_fwd_f32sILi3E")),
    ("attention_fwd_f32x3", re.compile(r"attn_fwd_f32x3|attn_fwd_f32s<2>|attn_fwd_f32sILi2E")),
    ("attention_fwd_f32", re.compile(r"attn_fwd_f32")),
    ("implicit_gemm", re.compile(r"conv_halo_kernel|conv_halo_occ2_kernel|gemm_pp_kernel|gemm_occ2_kernel|gemm_kernel<|conv1x1_stream_kernel")),
    ("attention_fwd", re.compile(r"attn_fwd_d64")),
]


def family(name: str):
    for fam, rx in FAMILIES:
        if rx.search(name):
            return fam
    return None


def load(d: str, counter: str):
    out = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        fam = family(r["Kernel_Name"])
        if fam is None:
            continue
        e = out.setdefault(fam, [0.0, 0])
        e[0] += float(r["Counter_Value"]) * 1024.0
        e[1] += 1
    return out


def write_summary(fd: str, wd: str, path: str) -> None:
    """Per-kernel totals of both passes (FETCH_SIZE raw and ×2, WRITE_SIZE), largest first."""
    agg = {}
    for d, cn in ((fd, "FETCH_SIZE"), (wd, "WRITE_SIZE")):
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            if r["Counter_Name"] != cn:
                continue
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").removeprefix("void ")
            n = re.sub(r"\(.*", "", n)[:90] if "at::native" not in n else "torch: " + n.split("<")[0][:80]
            e = agg.setdefault(n, {"FETCH_SIZE": [0.0, 0], "WRITE_SIZE": [0.0, 0]})
            e[cn][0] += float(r["Counter_Value"]) * 1024.0
            e[cn][1] += 1
    rows = sorted(agg.items(), key=lambda kv: -(2 * kv[1]["FETCH_SIZE"][0] + kv[1]["WRITE_SIZE"][0]))
    with open(path, "w") as f:
        f.write("# rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE, one bench step, per kernel (bytes; fetch x2 = gfx950 "
                "16-B streaming correction)\n")
        f.write(f"{'kernel':90s} {'launches':>8s} {'fetch_raw_B':>14s} {'fetch_x2_B':>14s} {'write_B':>14s}\n")
        for n, e in rows:
            f.write(f"{n:90s} {e['FETCH_SIZE'][1]:8d} {e['FETCH_SIZE'][0]:14.4e} {2 * e['FETCH_SIZE'][0]:14.4e} "
                    f"{e['WRITE_SIZE'][0]:14.4e}\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--preset", default="fast")
    ap.add_argument("--source", default="")
    ap.add_argument("--out", default="bench_traffic.json")
    ap.add_argument("--summary", default=None, help="also write a per-kernel table here")
    a = ap.parse_args()
    if a.summary:
        write_summary(a.fetch, a.write, a.summary)
    f, w = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    res = json.load(open(a.out)) if os.path.exists(a.out) else {}
    fams = {}
    for fam in sorted(set(f) | set(w)):
        fb, fn = f.get(fam, (0.0, 0))
        wb, wn = w.get(fam, (0.0, 0))
        n = max(fn, wn)
        fams[fam] = {"fetch_B_per_launch": 2.0 * fb / max(fn, 1), "write_B_per_launch": wb / max(wn, 1),
                     "bytes_per_launch": 2.0 * fb / max(fn, 1) + wb / max(wn, 1), "launches": n}
        print(f"{fam:20s} launches {n:6d}  fetch {2 * fb / max(fn, 1) / 1e6:10.2f} MB  "
              f"write {wb / max(wn, 1) / 1e6:10.2f} MB per launch")
    res[a.preset] = {"families": fams, "source": a.source,
                     "rule": "FETCH_SIZE x2 (gfx950 16-B streaming reads), WRITE_SIZE x1; L2->fabric bytes, "
                             "MALL hits included"}
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
