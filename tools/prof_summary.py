#!/usr/bin/env python3
"""Summarise rocprofv3 output of `tools/gpu.sh prof` for the step kernel.

Kernel time: the kernel-trace stats CSV (average duration per kernel name) and, from the
per-dispatch trace, the steady state -- the dominant kernel's dispatches after the first
10 % (at least 3), i.e. past the clock ramp and the warmup's shorter passes -- plus the
fixed-order sum kernels (mm_finalize*, mm_level_sums*) per step kernel dispatch.
Per step: (steady step-kernel mean + its sum kernels) / steps per launch, to set beside the
bench line's ms_per_step (the profiled run's own JSON line, in trace.log).
HBM traffic per launch: FETCH_SIZE and WRITE_SIZE (KB) per dispatch of the step kernel,
averaged; FETCH_SIZE doubled, the gfx950 correction of MI355X_MICROARCH.md 'HBM' (it
counts 64 B per 128-B request of a wide coalesced stream).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

KERNEL_RE = re.compile(r"mm_(pass[2k]?|wide)_kernel")
SUM_RE = re.compile(r"mm_(finalize|level_sums|hist_advance)")


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def bench_line(path):
    try:
        with open(path) as f:
            lines = [ln for ln in f if ln.startswith("{")]
        return json.loads(lines[-1]) if lines else None
    except OSError:
        return None


def priming(r):
    """mm_prepare's priming dispatch of a kernel: one workgroup, no work (not a pass)."""
    g = r.get("Grid_Size_X", r.get("Grid_Size"))
    w = r.get("Workgroup_Size_X", r.get("Workgroup_Size"))
    return g is not None and g == w


def steady(trace, name):
    """Durations (us) of `name`'s dispatches in start order, and the steady-state window."""
    d = sorted(((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                for r in trace if r.get("Kernel_Name") == name and not priming(r)))
    durs = [x for _, x in d]
    skip = max(3, len(durs) // 10) if len(durs) > 6 else 0
    return durs, durs[skip:], skip


def main():
    d, wl = sys.argv[1], sys.argv[2]
    res = {"workload": wl}
    stats = [r for r in rows(os.path.join(d, "trace", "**", "*kernel_stats.csv"))
             if KERNEL_RE.search(r.get("Name", ""))]
    # the dominant step kernel: largest total time
    stats.sort(key=lambda r: float(r["TotalDurationNs"]), reverse=True)
    name = None
    if stats:
        r = stats[0]
        name = r["Name"]
        res["kernel_name"] = name[:120]
        res["calls"] = int(r["Calls"])
        res["avg_us"] = float(r["AverageNs"]) / 1e3
        res["min_us"] = float(r["MinNs"]) / 1e3
        res["max_us"] = float(r["MaxNs"]) / 1e3
        res["share_of_gpu_time"] = float(r.get("Percentage", 0.0))
    trace = rows(os.path.join(d, "trace", "**", "*kernel_trace.csv"))
    line = bench_line(os.path.join(d, "trace.log"))
    if name and trace:
        durs, st, skip = steady(trace, name)
        # the kernel's own statistics without priming dispatches (kernel_stats.csv counts them)
        if durs:
            res["calls"] = len(durs)
            res["avg_us"] = statistics.mean(durs)
            res["min_us"] = min(durs)
            res["max_us"] = max(durs)
        if st:
            res["steady_dispatches"] = len(st)
            res["steady_skipped_first"] = skip
            res["steady_avg_us"] = statistics.mean(st)
            res["steady_median_us"] = statistics.median(st)
            res["steady_min_us"] = min(st)
            res["steady_max_us"] = max(st)
        sums = {}
        for r in trace:
            k = r.get("Kernel_Name", "")
            if SUM_RE.search(k):
                sums.setdefault(SUM_RE.search(k).group(0) + k.split(SUM_RE.search(k).group(0))[1].split("(")[0], []).append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        res["sum_kernels"] = {k: {"dispatches": len(v), "avg_us": statistics.mean(v)}
                              for k, v in sums.items()}
        if line and st:
            spl = line["roofline"]["steps_per_launch"]
            per_launch = sum(v["avg_us"] * v["dispatches"] for v in res["sum_kernels"].values()) \
                / max(len(durs), 1)
            res["sum_kernels_us_per_launch"] = per_launch
            res["steady_us_per_step"] = (res["steady_avg_us"] + per_launch) / spl
            res["bench_ms_per_step"] = line["ms_per_step"]
            res["bench_kernel_avg_us"] = line["roofline"]["kernel_avg_us"]
            res["bench_frac"] = line["roofline"]["frac"]
            ab = line["roofline"]["algorithmic_bytes_per_launch"]
            res["steady_frac"] = ab / (res["steady_avg_us"] * 1e-6) / 8e12
            res["steady_frac_vs_bench"] = res["steady_frac"] / line["roofline"]["frac"]
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        vals = [float(r["Counter_Value"]) for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv"))
                if name and r.get("Kernel_Name", "") == name and r.get("Counter_Name") == counter
                and not priming(r)]
        if vals:
            res[counter + "_KB_avg"] = statistics.mean(vals)
            res[counter + "_dispatches"] = len(vals)
    if "FETCH_SIZE_KB_avg" in res and "WRITE_SIZE_KB_avg" in res:
        rd = 2.0 * res["FETCH_SIZE_KB_avg"] * 1024
        wr = res["WRITE_SIZE_KB_avg"] * 1024
        res["hbm_read_bytes_per_launch"] = rd
        res["hbm_write_bytes_per_launch"] = wr
        res["hbm_bytes_per_launch"] = rd + wr
        if line:
            res["hbm_bytes_over_algorithmic"] = (rd + wr) / line["roofline"]["algorithmic_bytes_per_launch"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
