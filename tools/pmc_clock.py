"""Effective shader clock and MFMA-busy fraction per kernel family over one bench step, from one
rocprofv3 --pmc pass with GRBM_GUI_ACTIVE and SQ_VALU_MFMA_BUSY_CYCLES (MI355X_MICROARCH.md: effective
clock = GRBM_GUI_ACTIVE ÷ 8 XCDs ÷ kernel time; SQ_VALU_MFMA_BUSY_CYCLES = matrix-pipe cycles summed
over the SIMDs, so busy = it ÷ (GRBM_GUI_ACTIVE / 8 × 1 024 SIMDs)).

    timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv \\
        -d gpurun_out/clk -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-validate
    python tools/pmc_clock.py gpurun_out/clk > profiles/rNN_pmc_clock.txt
"""
import collections
import csv
import glob
import re
import sys

SIMDS = 256 * 4
FAMILIES = [
    ("conv_halo_occ2 GN-input", re.compile(r"conv_halo_occ2_kernel<1, true")),
    ("conv_halo_occ2 plain", re.compile(r"conv_halo_occ2_kernel<1, false")),
    ("conv_halo_occ2 upsample", re.compile(r"conv_halo_occ2_kernel<2")),
    ("attention d64", re.compile(r"attn_fwd_d64")),
    ("attention d512", re.compile(r"attn_fwd_d512")),
    ("gemm_pp", re.compile(r"gemm_pp_kernel")),
    ("gemm_occ2", re.compile(r"gemm_occ2_kernel")),
    ("gn_apply", re.compile(r"gn_apply")),
]


def main(root: str) -> None:
    path = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)[0]
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = disp[r["Dispatch_Id"]]
        d["name"] = r["Kernel_Name"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    print(f"# {path}: {len(disp)} dispatches")
    print(f"{'family':<26} {'launches':>8} {'ms':>9} {'clock GHz':>10} {'MFMA busy':>10}")
    for fam, rx in FAMILIES:
        ds = [d for d in disp.values() if rx.search(d["name"])]
        if not ds:
            continue
        ns = sum(d["ns"] for d in ds)
        gui = sum(d.get("GRBM_GUI_ACTIVE", 0.0) for d in ds) / 8
        busy = sum(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for d in ds)
        print(f"{fam:<26} {len(ds):>8} {ns / 1e6:>9.1f} {gui / ns:>10.2f} {busy / (gui * SIMDS):>10.3f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/clk")
