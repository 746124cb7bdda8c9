#!/usr/bin/env python3
"""Summarise an SQ/GRBM rocprofv3 --pmc pass (scripts/gpu_pmc_sq.sh) for the dominant
step kernel: mean counters per dispatch and the wave-cycle split (SQ counters count
quad-cycles; SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES,
MI355X_MICROARCH.md 'rocprofv3 PMC slots'), plus the effective clock GRBM_GUI_ACTIVE / 8 XCDs
/ kernel duration when a kernel-trace average is given -- only for dispatches of at least
0.3 ms: GRBM_GUI_ACTIVE counts busy cycles across the dispatch boundaries, so on shorter
dispatches the quotient reads high (MI355X_MICROARCH.md 'DVFS give-back'; round 5's C2
figure of 2.59 GHz on 71 us dispatches was above the part's 2.4 GHz maximum). Dispatches of
a single workgroup (mm_prepare's priming of a kernel, no work) are left out."""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    avg_us = float(sys.argv[2]) if len(sys.argv) > 2 else None
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    rows = [r for r in rows if "mm_pass" in r.get("Kernel_Name", "") or "mm_wide" in r.get("Kernel_Name", "")]
    # mm_prepare's priming dispatches (one workgroup of no work) are not passes
    rows = [r for r in rows if r.get("Grid_Size") is None or r.get("Grid_Size") != r.get("Workgroup_Size")]
    if not rows:
        sys.exit("no step-kernel dispatches")
    by_kernel = {}
    for r in rows:
        by_kernel.setdefault(r["Kernel_Name"], []).append(r)
    name = max(by_kernel, key=lambda k: len(by_kernel[k]))
    per = {}
    for r in by_kernel[name]:
        per.setdefault((r.get("Dispatch_Id"), r["Counter_Name"]), 0.0)
        per[(r.get("Dispatch_Id"), r["Counter_Name"])] += float(r["Counter_Value"])
    counters = {}
    for (disp, c), v in per.items():
        counters.setdefault(c, []).append(v)
    out = {"kernel": name[:120], "dispatches": len({d for d, _ in per})}
    out.update({c: statistics.mean(v) for c, v in sorted(counters.items())})
    wc = out.get("SQ_WAVE_CYCLES")
    if wc:
        for key, c in (("frac_wait_mem", "SQ_WAIT_ANY"), ("frac_issue_stall", "SQ_WAIT_INST_ANY"),
                       ("frac_active", "SQ_ACTIVE_INST_ANY"), ("frac_active_valu", "SQ_ACTIVE_INST_VALU")):
            if c in out:
                out[key] = out[c] / wc
    if avg_us and "GRBM_GUI_ACTIVE" in out:
        out["kernel_avg_us"] = avg_us
        clk = out["GRBM_GUI_ACTIVE"] / 8.0 / (avg_us * 1e-6) / 1e9
        if avg_us >= 300.0:
            out["effective_clock_GHz"] = clk
        else:
            out["effective_clock_GHz"] = None
            out["effective_clock_note"] = (f"GRBM quotient {clk:.2f} GHz not a clock: dispatch "
                                           f"{avg_us:.0f} us < 300 us (MI355X_MICROARCH.md DVFS)")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
