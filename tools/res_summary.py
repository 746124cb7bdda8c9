#!/usr/bin/env python3
"""Condense hipcc -Rpass-analysis=kernel-resource-usage output to one line per kernel:
demangled-ish name, VGPRs, AGPRs, SGPRs, scratch, occupancy (waves per SIMD), LDS."""
import re
import sys

KEYS = ("VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "TotalSGPRs", "ScratchSize", "Occupancy",
        "LDS Size")


def demangle(name):
    try:
        import subprocess
        return subprocess.run(["c++filt", name], capture_output=True, text=True,
                              timeout=10).stdout.strip().replace("mm::(anonymous namespace)::", "")
    except (OSError, subprocess.SubprocessError):
        return name


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
            m = re.search(r"\s%s(?: \[[^\]]*\])?: (\d+)" % re.escape(k), ln)
            if m:
                cur[k] = int(m.group(1))
    for r in rows:
        print(demangle(r["name"]), " ".join(f"{k.replace(' ', '')}={r.get(k)}" for k in KEYS))


if __name__ == "__main__":
    main(sys.argv[1])
