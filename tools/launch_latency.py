#!/usr/bin/env python3
"""Launch-to-start latency of every kernel dispatch in a rocprofv3 --hip-trace
--kernel-trace run: the time from the end of the hipLaunchKernel call that enqueued a
kernel (matched by correlation id) to the kernel's start on the GPU, and its duration.
The first dispatch of a kernel that needs scratch waits for the queue's scratch setup
(172 us for the driver's K = 20 launch, 5.6 us for the next one).

usage: launch_latency.py TRACE_DIR
"""
import csv
import glob
import os
import sys


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    d = sys.argv[1]
    api = {r["Correlation_Id"]: r for r in rows(d, "*hip_api_trace.csv")
           if r["Function"] in ("hipLaunchKernel", "hipExtLaunchKernel", "hipModuleLaunchKernel")}
    ker = sorted(rows(d, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    for k in ker:
        s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
        a = api.get(k["Correlation_Id"])
        lat = f"{(s - int(a['End_Timestamp'])) / 1e3:9.1f}" if a else "        -"
        print(f"launch->start {lat} us  dur {(e - s) / 1e3:9.1f} us  scratch {k.get('Scratch_Size', '?'):>4}  "
              f"{k['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main()
