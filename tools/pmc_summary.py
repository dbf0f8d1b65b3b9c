"""Condense rocprofv3 --pmc counter CSVs (tools/pmc_round.sh output) into one text table.

    python tools/pmc_summary.py gpurun_out/pmc_r02 > profiles/r02_pmc_summary.txt

One row per (pass, kernel launch, counter): kernel name shortened, duration from the CSV's own
timestamps, raw counter value and — for FETCH_SIZE / WRITE_SIZE (KB) — bytes.  The reading rules
(FETCH_SIZE's ½ for 16-B streaming loads, checked by the `copy` pass) are applied in DESIGN.md, not
here: this file keeps the raw numbers."""
import csv
import os
import re
import sys


def short(name: str) -> str:
    if "at::native" in name:
        return "torch: " + name.split("<")[0].split("::")[-1][:60]
    name = name.replace("(anonymous namespace)::", "").removeprefix("void ")
    return re.sub(r"\(.*", "", name)[:70]


def main(root: str) -> None:
    for d in sorted(os.listdir(root)):
        f = os.path.join(root, d, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        rows = list(csv.DictReader(open(f)))
        print(f"== pass {d} ({len(rows)} rows)")
        print(f"{'disp':>5} {'kernel':<70} {'us':>9} {'counter':<26} {'value':>16}")
        for r in rows:
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            v = float(r["Counter_Value"])
            extra = f"  = {v * 1024:.4e} B" if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE") else ""
            print(f"{r['Dispatch_Id']:>5} {short(r['Kernel_Name']):<70} {us:9.1f} {r['Counter_Name']:<26} "
                  f"{v:16.1f}{extra}")
        print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_r02")
