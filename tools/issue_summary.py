"""Vector-issue-port occupancy per SIMD from the SQ instruction counts of tools/issue_pmc.sh.

    python tools/issue_summary.py gpurun_out/issue_pmc

Per target (the last launch of the profiled kernel): the cycles the SIMD's one vector-issue port is
claimed, priced with MI355X_MICROARCH.md's measured issue costs ('vector-instruction ISSUE cost':
transcendental 8, other VALU 4, an MFMA holds the port 8 cycles), against the kernel's cycles per
SIMD (GRBM_GUI_ACTIVE / 8 XCDs, 1 024 SIMDs).  SQ_INSTS_VALU counts MFMAs too (subtracted).  LDS,
SALU and VMEM instructions issue through other paths and are listed, not priced."""
import csv
import os
import sys


def last_launch(path):
    rows = list(csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))))
    keep = [r for r in rows if any(k in r["Kernel_Name"] for k in ("attn_fwd", "conv_halo", "gemm_f32"))]
    did = max(int(r["Dispatch_Id"]) for r in keep)
    out = {r["Counter_Name"]: float(r["Counter_Value"]) for r in keep if int(r["Dispatch_Id"]) == did}
    r0 = next(r for r in keep if int(r["Dispatch_Id"]) == did)
    out["_us"] = (int(r0["End_Timestamp"]) - int(r0["Start_Timestamp"])) / 1e3
    out["_name"] = r0["Kernel_Name"].split("(")[0][:60]
    return out


def main(root):
    names = sorted({d.rsplit("_", 1)[0] for d in os.listdir(root) if os.path.isdir(os.path.join(root, d))})
    for n in names:
        c = {}
        for p in (1, 2):
            d = os.path.join(root, f"{n}_{p}")
            if os.path.isdir(d):
                c.update(last_launch(d))
        cyc = c["GRBM_GUI_ACTIVE"] / 8 * 1024  # SIMD-cycles of the launch
        mfma = c["SQ_INSTS_MFMA"]
        trans = c["SQ_INSTS_VALU_TRANS_F32"] + c["SQ_INSTS_VALU_TRANS_F16"]
        valu = c["SQ_INSTS_VALU"] - mfma - trans
        issue = 4 * valu + 8 * trans + 8 * mfma
        clock = c["GRBM_GUI_ACTIVE"] / 8 / (c["_us"] * 1e3)
        print(f"{n:12s} {c['_name']}: {c['_us']:.1f} us, {clock:.2f} GHz; per SIMD-cycle: MFMA busy "
              f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / cyc:.3f}, vector-issue port {issue / cyc:.3f} "
              f"(VALU {4 * valu / cyc:.3f} + transcendental {8 * trans / cyc:.3f} + MFMA holds {8 * mfma / cyc:.3f}); "
              f"instructions per MFMA: VALU {valu / mfma:.2f}, trans {trans / mfma:.2f}, cvt "
              f"{c['SQ_INSTS_VALU_CVT'] / mfma:.2f}, LDS {c['SQ_INSTS_LDS'] / mfma:.2f}, SALU {c['SQ_INSTS_SALU'] / mfma:.2f}"
              + (f"; MFMA∥VALU co-exec {c['SQ_VALU_MFMA_COEXEC_CYCLES'] / cyc:.3f}, wave-cycles waiting "
                 f"{c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f} (s_waitcnt/barrier) "
                 f"{c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f} (issue stalls)" if "SQ_WAVE_CYCLES" in c else ""))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/issue_pmc")
