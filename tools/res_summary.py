#!/usr/bin/env python3
"""Condense hipcc -Rpass-analysis=kernel-resource-usage output to one line per kernel:
demangled-ish name, VGPRs, AGPRs, SGPRs, scratch, occupancy (waves per SIMD), LDS."""
import re
import sys

KEYS = ("VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize", "Occupancy", "LDS Size")


def main(path):
    cur = None
    rows = []
    for ln in open(path, errors="replace"):
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for k in KEYS:
            m = re.search(r"\s%s(?: \[bytes/lane\])?: (\d+)" % re.escape(k), ln)
            if m:
                cur[k] = int(m.group(1))
    for r in rows:
        print(r["name"], " ".join(f"{k.split()[0]}={r.get(k)}" for k in KEYS))


if __name__ == "__main__":
    main(sys.argv[1])
