#!/usr/bin/env python3
"""Per-pass decomposition of a split-schedule run from a rocprofv3 kernel trace.

`tools/gpu.sh thintrace` traces `bench.py --self-halo` on the thin slabs of the c3 N = 8 /
N = 4 runs (4096 / 8192 x 32768, /root/reference/src/Model.hpp:63-76 partition) and the
same slabs without a halo. A K-step pass of the split schedule is

    comm stream:    exchange k (RCCL kernels) -> [wait interior k-1] -> border k
    compute stream: [wait border k-1] -> interior k

This script takes the trace's step-kernel dispatches (mm_wide_kernel / mm_passk_kernel:
the interior launch is the one with the most workgroups of its pass, the border launch the
small one) and the RCCL kernels, and reports per pass: the interior kernel's duration, the
border kernel's, the exchange kernels', the gap on the compute stream between one
interior's end and the next one's start, and the pass period (interior start to interior
start). Medians over the steady passes (the timed run's own and the timing pass's; the
first pass of each is skipped as cold). Usage: thin_trace.py TRACE_DIR [LABEL]
"""
import csv
import glob
import json
import os
import statistics
import sys

STEP = ("mm_wide_kernel", "mm_passk_kernel")


def load(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    for r in out:
        r["t0"] = int(r["Start_Timestamp"]) / 1e3
        r["t1"] = int(r["End_Timestamp"]) / 1e3
        r["grid"] = int(r.get("Grid_Size_X") or 0)
    out.sort(key=lambda r: r["t0"])
    return out


def med(xs):
    return round(statistics.median(xs), 2) if xs else None


def main():
    d = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(d.rstrip("/"))
    tr = load(d)
    step = [r for r in tr if any(s in r["Kernel_Name"] for s in STEP)]
    rccl = [r for r in tr if "nccl" in r["Kernel_Name"].lower() or "rccl" in r["Kernel_Name"].lower()]
    if not step:
        print(json.dumps({"label": label, "error": "no step kernels"}))
        return
    big = max(r["grid"] for r in step)
    # interior launches: the large grids of the pass length that dominates the run
    interior = [r for r in step if r["grid"] >= big // 4]
    border = [r for r in step if r["grid"] < big // 4]
    passes = []
    for i, it in enumerate(interior):
        nxt = interior[i + 1] if i + 1 < len(interior) else None
        # border k is launched beside interior k (the two streams start together): the
        # border launch whose start is nearest this interior's; exchange k+1 follows it on
        # the comm stream (the RCCL kernels between that border's end and the next
        # interior's start)
        b = min(border, key=lambda r: abs(r["t0"] - it["t0"])) if border else None
        if b is not None and abs(b["t0"] - it["t0"]) > 100.0:
            b = None
        hi = nxt["t0"] if nxt else it["t1"] + 1e9
        e = [r for r in rccl if b is not None and b["t1"] <= r["t0"] < hi]
        rec = {
            "interior_us": it["t1"] - it["t0"],
            "interior_grid": it["grid"],
            "border_us": (b["t1"] - b["t0"]) if b else None,
            "exchange_us": sum(r["t1"] - r["t0"] for r in e) if e else None,
            "gap_after_interior_us": (nxt["t0"] - it["t1"]) if nxt else None,
            "period_us": (nxt["t0"] - it["t0"]) if nxt else None,
            # the comm stream's work of the pass (border, then the next exchange) ends this
            # long before (< 0) or after the interior kernel
            "comm_end_minus_interior_end_us": ((max([b["t1"]] + [r["t1"] for r in e]) - it["t1"])
                                               if b else None),
        }
        passes.append(rec)
    # steady passes: drop the cold first pass of each back-to-back run (a gap > 1 ms)
    steady = [p for i, p in enumerate(passes)
              if i > 0 and passes[i - 1]["gap_after_interior_us"] is not None
              and passes[i - 1]["gap_after_interior_us"] < 1000 and p["period_us"] is not None]
    out = {"label": label, "passes": len(passes), "steady_passes": len(steady)}
    for k in ("interior_us", "border_us", "exchange_us", "gap_after_interior_us", "period_us",
              "comm_end_minus_interior_end_us"):
        out[k + "_median"] = med([p[k] for p in steady if p[k] is not None])
    if steady and out["period_us_median"]:
        out["interior_share_of_period"] = round(out["interior_us_median"] / out["period_us_median"], 4)
    out["interior_grid"] = passes[-1]["interior_grid"] if passes else None
    print(json.dumps(out))
    # the timeline of three steady passes (relative us, queue, grid, duration)
    if len(interior) >= 5:
        a, b = interior[-5]["t0"], interior[-2]["t0"]
        with open(os.path.join(d, "timeline.txt"), "w") as f:
            for r in tr:
                if a <= r["t0"] < b:
                    f.write(f"{r['t0'] - a:10.1f} {r['t1'] - r['t0']:9.1f} q{r.get('Queue_Id', '?'):>3} "
                            f"grid {r['grid']:8d} {r['Kernel_Name'][:70]}\n")


if __name__ == "__main__":
    main()
